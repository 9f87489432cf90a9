"""Feature / context encoders (residual CNNs at 1/8 resolution).

Architecture and parameter names match the reference encoders so that
``raft-*.pth`` checkpoints load unchanged (core/extractor.py:6-267):

* ``BasicEncoder``: 7x7/s2 conv (64) -> 3 stages of 2 ``ResidualBlock`` (64, 96/s2,
  128/s2) -> 1x1 conv to ``output_dim``;
* ``SmallEncoder``: same topology with ``BottleneckBlock`` (32, 64/s2, 96/s2).

On the GPU the RAFT orchestrator runs both encoders on the hand-written HIP
kernels of ``ops/encoder.py`` / ``csrc/encoder.hip`` (one autograd node per
encoder, NHWC, fused norm statistics) under bf16 AMP, and for fp32 inference in
their split-bf16 (fp32-faithful) mode; the ``forward`` methods here are the
module path (CPU runs, fp32 training, and the reference op path the GPU tests
compare against).  Passing a list/tuple ``[img1, img2]`` runs both frames as one batch
(core/extractor.py:170-174).
"""
from __future__ import annotations

import torch
import torch.nn as nn

from ..ops.norm import InstanceNorm2dNHWC


def make_norm(kind: str, channels: int, groups: int):
    if kind == "group":
        return nn.GroupNorm(num_groups=groups, num_channels=channels)
    if kind == "batch":
        return nn.BatchNorm2d(channels)
    if kind == "instance":
        # parameter-free like nn.InstanceNorm2d(channels); NHWC HIP kernels with fused ReLU on GPU
        return InstanceNorm2dNHWC(channels)
    if kind == "none":
        return nn.Sequential()
    raise ValueError(f"unknown norm_fn {kind!r}")


def norm_relu(norm: nn.Module, x: torch.Tensor) -> torch.Tensor:
    """relu(norm(x)), fusing the ReLU into the NHWC instance-norm kernel when possible."""
    if isinstance(norm, InstanceNorm2dNHWC):
        return norm(x, relu=True)
    return torch.relu(norm(x))


class ResidualBlock(nn.Module):
    def __init__(self, in_planes: int, planes: int, norm_fn: str = "group", stride: int = 1):
        super().__init__()
        self.conv1 = nn.Conv2d(in_planes, planes, kernel_size=3, padding=1, stride=stride)
        self.conv2 = nn.Conv2d(planes, planes, kernel_size=3, padding=1)
        self.relu = nn.ReLU(inplace=True)
        g = planes // 8
        self.norm1 = make_norm(norm_fn, planes, g)
        self.norm2 = make_norm(norm_fn, planes, g)
        if stride != 1:
            self.norm3 = make_norm(norm_fn, planes, g)
            self.downsample = nn.Sequential(nn.Conv2d(in_planes, planes, kernel_size=1, stride=stride), self.norm3)
        else:
            self.downsample = None

    def forward(self, x):
        y = norm_relu(self.norm1, self.conv1(x))
        y = norm_relu(self.norm2, self.conv2(y))
        if self.downsample is not None:
            x = self.downsample(x)
        return self.relu(x + y)


class BottleneckBlock(nn.Module):
    def __init__(self, in_planes: int, planes: int, norm_fn: str = "group", stride: int = 1):
        super().__init__()
        mid = planes // 4
        self.conv1 = nn.Conv2d(in_planes, mid, kernel_size=1, padding=0)
        self.conv2 = nn.Conv2d(mid, mid, kernel_size=3, padding=1, stride=stride)
        self.conv3 = nn.Conv2d(mid, planes, kernel_size=1, padding=0)
        self.relu = nn.ReLU(inplace=True)
        g = planes // 8
        self.norm1 = make_norm(norm_fn, mid, g)
        self.norm2 = make_norm(norm_fn, mid, g)
        self.norm3 = make_norm(norm_fn, planes, g)
        if stride != 1:
            self.norm4 = make_norm(norm_fn, planes, g)
            self.downsample = nn.Sequential(nn.Conv2d(in_planes, planes, kernel_size=1, stride=stride), self.norm4)
        else:
            self.downsample = None

    def forward(self, x):
        y = norm_relu(self.norm1, self.conv1(x))
        y = norm_relu(self.norm2, self.conv2(y))
        y = norm_relu(self.norm3, self.conv3(y))
        if self.downsample is not None:
            x = self.downsample(x)
        return self.relu(x + y)


class _Encoder(nn.Module):
    block = ResidualBlock
    widths = (64, 64, 96, 128)

    def __init__(self, output_dim: int = 128, norm_fn: str = "batch", dropout: float = 0.0):
        super().__init__()
        self.norm_fn = norm_fn
        stem, w1, w2, w3 = self.widths
        self.norm1 = make_norm(norm_fn, stem, 8)
        self.conv1 = nn.Conv2d(3, stem, kernel_size=7, stride=2, padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        self.in_planes = stem
        self.layer1 = self._make_layer(w1, stride=1)
        self.layer2 = self._make_layer(w2, stride=2)
        self.layer3 = self._make_layer(w3, stride=2)
        self.conv2 = nn.Conv2d(w3, output_dim, kernel_size=1)
        self.dropout = nn.Dropout2d(p=dropout) if dropout > 0 else None
        self._init_weights()

    def _init_weights(self):
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.GroupNorm)):
                if m.weight is not None:
                    nn.init.constant_(m.weight, 1)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    def _make_layer(self, dim: int, stride: int = 1):
        blocks = (self.block(self.in_planes, dim, self.norm_fn, stride=stride),
                  self.block(dim, dim, self.norm_fn, stride=1))
        self.in_planes = dim
        return nn.Sequential(*blocks)

    def forward(self, x):
        paired = isinstance(x, (list, tuple))
        if paired:
            n = x[0].shape[0]
            x = torch.cat(x, dim=0)
        x = norm_relu(self.norm1, self.conv1(x))
        x = self.layer3(self.layer2(self.layer1(x)))
        x = self.conv2(x)
        if self.training and self.dropout is not None:
            x = self.dropout(x)
        if paired:
            return torch.split(x, [n, n], dim=0)
        return x


class BasicEncoder(_Encoder):
    block = ResidualBlock
    widths = (64, 64, 96, 128)


class SmallEncoder(_Encoder):
    block = BottleneckBlock
    widths = (32, 32, 64, 96)
