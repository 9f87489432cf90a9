"""Reference (PyTorch) ops and geometry utilities on CPU."""
import numpy as np
import pytest
import torch
import torch.nn.functional as F

from raft_ros_amd.ops import reference as ref
from raft_ros_amd.utils.utils import InputPadder, forward_interpolate


def test_coords_grid():
    g = ref.coords_grid(2, 3, 4)
    assert g.shape == (2, 2, 3, 4)
    assert torch.equal(g[0, 0, 1], torch.arange(4.0)) and torch.equal(g[1, 1, :, 2], torch.arange(3.0))


def test_window_is_x_major():
    # pure x ramp: channel ix*(2r+1)+iy moves in x with ix
    B, H, W, r = 1, 12, 12, 2
    vol = torch.arange(W, dtype=torch.float32).view(1, 1, 1, W).expand(B * H * W, 1, H, W)
    out = ref.pyramid_lookup([vol], ref.coords_grid(B, H, W), r)
    px = out[0, :, 6, 6].view(2 * r + 1, 2 * r + 1)
    assert torch.allclose(px[:, 0], torch.arange(4.0, 9.0))
    assert torch.allclose(px[2], torch.full((5,), 6.0))


def test_pooling_fmap2_equals_pooling_volume():
    """AlternateCorrBlock pools fmap2 instead of the volume: identical by linearity."""
    torch.manual_seed(0)
    f1 = torch.randn(1, 16, 10, 12)
    f2 = torch.randn(1, 16, 10, 12)
    pyr = ref.build_pyramid(ref.corr_volume(f1, f2), 3)
    coords = ref.coords_grid(1, 10, 12) + torch.randn(1, 2, 10, 12)
    dense = ref.pyramid_lookup(pyr, coords, 2)
    local = []
    f2l = f2
    for lvl in range(3):
        if lvl:
            f2l = F.avg_pool2d(f2l, 2, 2)
        local.append(ref.local_corr(f1, f2l, coords / 2 ** lvl, 2) / 4.0)  # 1/sqrt(16)
    torch.testing.assert_close(torch.cat(local, dim=1), dense, rtol=1e-4, atol=1e-5)


def test_convex_upsample_matches_explicit_formula():
    torch.manual_seed(0)
    flow = torch.randn(1, 2, 3, 4)
    mask = torch.randn(1, 576, 3, 4)
    up = ref.convex_upsample(flow, mask)
    y, x, i, j = 1, 2, 3, 5
    w = torch.softmax(mask[0, :, y, x].view(9, 8, 8)[:, i, j], 0)
    nb = F.pad(8 * flow, (1, 1, 1, 1))[0, :, y:y + 3, x:x + 3].reshape(2, 9)
    torch.testing.assert_close(up[0, :, 8 * y + i, 8 * x + j], (nb * w).sum(1))


def test_upflow8():
    f = torch.ones(1, 2, 4, 5)
    assert torch.allclose(ref.upflow8(f), torch.full((1, 2, 32, 40), 8.0))


@pytest.mark.parametrize("shape,mode,pad", [((436, 1024), "sintel", [0, 0, 2, 2]),
                                            ((375, 1242), "kitti", [3, 3, 0, 1]),
                                            ((1080, 1920), "sintel", [0, 0, 0, 0])])
def test_input_padder(shape, mode, pad):
    p = InputPadder((1, 3) + shape, mode=mode)
    assert p._pad == pad
    x = torch.randn(1, 3, *shape)
    (xp,) = p.pad(x)
    assert xp.shape[-2] % 8 == 0 and xp.shape[-1] % 8 == 0
    assert torch.equal(p.unpad(xp), x)


def test_forward_interpolate_constant_flow():
    flow = torch.zeros(2, 16, 20)
    flow[0] = 2.0
    out = forward_interpolate(flow)
    assert out.shape == (2, 16, 20)
    assert torch.allclose(out[0], torch.full((16, 20), 2.0))


@pytest.mark.reference
def test_flow_viz_matches_reference(reference_core):
    import importlib.util

    spec = importlib.util.spec_from_file_location("ref_flow_viz", "/root/reference/core/utils/flow_viz.py")
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    from raft_ros_amd.utils import flow_viz

    rng = np.random.default_rng(0)
    flow = rng.normal(size=(37, 41, 2)).astype(np.float32) * 5
    assert np.array_equal(flow_viz.make_colorwheel(), mod.make_colorwheel())
    for bgr in (False, True):
        assert np.array_equal(flow_viz.flow_to_image(flow, convert_to_bgr=bgr), mod.flow_to_image(flow, convert_to_bgr=bgr))


def test_blocked_level_layout_matches_kernel_indexing():
    """The dense pyramid stores each level in 16-column blocks; the GEMM operand built by
    _concat_levels must put pixel (y, x) of level l at off_l + ((x//16)*Hl + y)*16 + x%16,
    the index the lookup / unpool kernels use (csrc/corr_volume.hip lvl_off)."""
    import torch
    from raft_ros_amd.ops.corr import _concat_levels

    B, C = 2, 3
    fs = [torch.randn(B, C, 7, 37), torch.randn(B, C, 3, 18)]
    offs, off = [], 0
    for f in fs:
        offs.append(off)
        off += -(-f.shape[3] // 16) * 16 * f.shape[2]
    rows = _concat_levels(fs, off, offs, nchw=False, blocked=True)  # (B, ld, C)
    cols = _concat_levels(fs, off, offs, nchw=True, blocked=True)   # (B, C, ld)
    assert torch.equal(rows, cols.permute(0, 2, 1))
    for f, o in zip(fs, offs):
        Hl, Wl = f.shape[2:]
        nb = -(-Wl // 16)
        for y in range(Hl):
            for x in range(nb * 16):
                idx = o + ((x // 16) * Hl + y) * 16 + x % 16
                want = f[:, :, y, x] if x < Wl else torch.zeros(B, C)
                assert torch.equal(rows[:, idx], want), (y, x)
