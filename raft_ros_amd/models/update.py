"""Recurrent update operator: motion encoder, (separable) ConvGRU, flow and mask heads.

Parameter names/shapes match core/update.py:6-136 (checkpoint compatible).
MI355X-specific execution:

* the z and r gates of every GRU stage run as ONE convolution with the two
  weight tensors concatenated (256 output channels instead of 2 x 128), which
  halves the reads of the 384-channel ``[h, x]`` input and the launches;
* the gate nonlinearities and the blend ``h = (1-z) h + z q`` are fused
  elementwise kernels (``raft_ros_amd.ops.gru``);
* the mask head's 0.25 gradient-balancing scale is folded into its last conv.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..ops import gru as gru_ops


class FlowHead(nn.Module):
    def __init__(self, input_dim: int = 128, hidden_dim: int = 256):
        super().__init__()
        self.conv1 = nn.Conv2d(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = nn.Conv2d(hidden_dim, 2, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return self.conv2(self.relu(self.conv1(x)))


def _gru_step(h, x, conv_z, conv_r, conv_q, padding):
    """One GRU stage with fused z||r convolution and fused gate math."""
    hx = torch.cat([h, x], dim=1)
    if gru_ops.get_backend() == "reference":  # the reference's unfused op sequence (baseline only)
        z = torch.sigmoid(conv_z(hx))
        r = torch.sigmoid(conv_r(hx))
        q = torch.tanh(conv_q(torch.cat([r * h, x], dim=1)))
        return (1 - z) * h + z * q
    w = torch.cat([conv_z.weight, conv_r.weight], dim=0)
    b = torch.cat([conv_z.bias, conv_r.bias], dim=0)
    zr = F.conv2d(hx, w, b, padding=padding)
    z, rh = gru_ops.gates_zr(zr, h)  # z = sigmoid, rh = sigmoid(r) * h
    q = F.conv2d(torch.cat([rh, x], dim=1), conv_q.weight, conv_q.bias, padding=padding)
    return gru_ops.blend(z, q, h)  # (1 - z) h + z tanh(q)


class ConvGRU(nn.Module):
    def __init__(self, hidden_dim: int = 128, input_dim: int = 192 + 128):
        super().__init__()
        self.convz = nn.Conv2d(hidden_dim + input_dim, hidden_dim, 3, padding=1)
        self.convr = nn.Conv2d(hidden_dim + input_dim, hidden_dim, 3, padding=1)
        self.convq = nn.Conv2d(hidden_dim + input_dim, hidden_dim, 3, padding=1)

    def forward(self, h, x):
        return _gru_step(h, x, self.convz, self.convr, self.convq, 1)


class SepConvGRU(nn.Module):
    def __init__(self, hidden_dim: int = 128, input_dim: int = 192 + 128):
        super().__init__()
        cin = hidden_dim + input_dim
        self.convz1 = nn.Conv2d(cin, hidden_dim, (1, 5), padding=(0, 2))
        self.convr1 = nn.Conv2d(cin, hidden_dim, (1, 5), padding=(0, 2))
        self.convq1 = nn.Conv2d(cin, hidden_dim, (1, 5), padding=(0, 2))
        self.convz2 = nn.Conv2d(cin, hidden_dim, (5, 1), padding=(2, 0))
        self.convr2 = nn.Conv2d(cin, hidden_dim, (5, 1), padding=(2, 0))
        self.convq2 = nn.Conv2d(cin, hidden_dim, (5, 1), padding=(2, 0))

    def forward(self, h, x):
        h = _gru_step(h, x, self.convz1, self.convr1, self.convq1, (0, 2))  # horizontal
        h = _gru_step(h, x, self.convz2, self.convr2, self.convq2, (2, 0))  # vertical
        return h


class SmallMotionEncoder(nn.Module):
    def __init__(self, args):
        super().__init__()
        cor_planes = args.corr_levels * (2 * args.corr_radius + 1) ** 2
        self.convc1 = nn.Conv2d(cor_planes, 96, 1, padding=0)
        self.convf1 = nn.Conv2d(2, 64, 7, padding=3)
        self.convf2 = nn.Conv2d(64, 32, 3, padding=1)
        self.conv = nn.Conv2d(128, 80, 3, padding=1)

    def forward(self, flow, corr):
        cor = F.relu(self.convc1(corr))
        flo = F.relu(self.convf2(F.relu(self.convf1(flow))))
        out = F.relu(self.conv(torch.cat([cor, flo], dim=1)))
        return torch.cat([out, flow.to(out.dtype)], dim=1)


class BasicMotionEncoder(nn.Module):
    def __init__(self, args):
        super().__init__()
        cor_planes = args.corr_levels * (2 * args.corr_radius + 1) ** 2
        self.convc1 = nn.Conv2d(cor_planes, 256, 1, padding=0)
        self.convc2 = nn.Conv2d(256, 192, 3, padding=1)
        self.convf1 = nn.Conv2d(2, 128, 7, padding=3)
        self.convf2 = nn.Conv2d(128, 64, 3, padding=1)
        self.conv = nn.Conv2d(64 + 192, 128 - 2, 3, padding=1)

    def forward(self, flow, corr):
        cor = F.relu(self.convc2(F.relu(self.convc1(corr))))
        flo = F.relu(self.convf2(F.relu(self.convf1(flow))))
        out = F.relu(self.conv(torch.cat([cor, flo], dim=1)))
        return torch.cat([out, flow.to(out.dtype)], dim=1)


class SmallUpdateBlock(nn.Module):
    def __init__(self, args, hidden_dim: int = 96):
        super().__init__()
        self.encoder = SmallMotionEncoder(args)
        self.gru = ConvGRU(hidden_dim=hidden_dim, input_dim=82 + 64)
        self.flow_head = FlowHead(hidden_dim, hidden_dim=128)

    def forward(self, net, inp, corr, flow):
        motion = self.encoder(flow, corr)
        net = self.gru(net, torch.cat([inp, motion], dim=1))
        return net, None, self.flow_head(net)


class BasicUpdateBlock(nn.Module):
    def __init__(self, args, hidden_dim: int = 128, input_dim: int = 128):
        super().__init__()
        self.args = args
        self.encoder = BasicMotionEncoder(args)
        self.gru = SepConvGRU(hidden_dim=hidden_dim, input_dim=128 + hidden_dim)
        self.flow_head = FlowHead(hidden_dim, hidden_dim=256)
        self.mask = nn.Sequential(
            nn.Conv2d(128, 256, 3, padding=1),
            nn.ReLU(inplace=True),
            nn.Conv2d(256, 64 * 9, 1, padding=0),
        )

    def forward(self, net, inp, corr, flow, upsample: bool = True):
        motion = self.encoder(flow, corr)
        net = self.gru(net, torch.cat([inp, motion], dim=1))
        delta_flow = self.flow_head(net)
        # 0.25 * mask(net): scale folded into the final 1x1 conv (gradient balancing)
        m = self.mask[1](self.mask[0](net))
        mask = F.conv2d(m, 0.25 * self.mask[2].weight, 0.25 * self.mask[2].bias)
        return net, mask, delta_flow
