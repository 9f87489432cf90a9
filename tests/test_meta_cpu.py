"""Fake (meta) kernels of the native ops: shape/dtype inference without a GPU."""
import pytest
import torch

from raft_ros_amd.ops import _ext

pytestmark = pytest.mark.skipif(not _ext.is_loaded(), reason=f"native library not built: {_ext.load_error()}")


def test_meta_shapes_of_tensor_returning_ops():
    ops = _ext.ops()
    m = torch.device("meta")
    coords = torch.empty(2, 2, 46, 62, device=m)
    pyr = [torch.empty(2 * 46 * 62, 46 * 62, device=m)] * 4
    assert ops.corr_lookup(pyr, coords, 4, torch.bfloat16, 328).shape == (2, 46, 62, 328)
    assert ops.convex_upsample(coords, torch.empty(2, 576, 46, 62, device=m)).shape == (2, 2, 368, 496)
    assert ops.upflow8(coords).shape == (2, 2, 368, 496)
    assert ops.upflow8_backward(torch.empty(2, 2, 368, 496, device=m), 46, 62, None).shape == (2, 2, 46, 62)
    x = torch.empty(4, 92, 124, 64, device=m, dtype=torch.bfloat16)
    w = torch.empty(96, 64, 3, 3, device=m)
    y, st = ops.enc_conv_fwd(x, w, None, 2, 1, True)
    assert y.shape == (4, 46, 62, 96) and st.shape == (4, -(-46 * 62 // 128), 2, 96)
    assert ops.enc_conv_dgrad([y], [w], [2], [1], 92, 124, None, None).shape == x.shape
    img = torch.empty(2, 3, 368, 496, device=m)
    assert ops.enc_prep(img, img).shape == (4, 368, 496, 8)
    A = torch.empty(2, 100, 64, device=m, dtype=torch.bfloat16)
    assert ops.gemm_nt(A, A, 1.0, torch.float32).shape == (2, 100, 100)
    g = torch.empty(2, 46, 62, 64, device=m, dtype=torch.bfloat16)
    out = ops.enc_norm_bwd(g, g, torch.empty(2, 4, 64, device=m), True, g, torch.empty(2, 4, 64, device=m), 2)
    assert out[0].shape == g.shape and out[4].shape == (64,)
