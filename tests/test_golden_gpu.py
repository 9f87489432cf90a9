"""Golden parity on the GPU against the REAL reference implementation's outputs
(tests/fixtures/golden_demo_frames.npz, scripts/make_golden.py: reference core.raft.RAFT on
the CPU in fp32, seed-0 weights, the reference's demo frames, 440x1024, 20 iterations,
test_mode -- the demo.py / ROS node configuration).

* native fp32 path (mixed_precision=False; the reference's default for demo / evaluate /
  ROS): EPE <= 0.01 px from the fixture, on the low-res and the upsampled flow;
* native bf16 path (HIP encoders + fused update kernels): EPE delta <= 3x the delta of
  PyTorch's own bf16 autocast of the module path (the same computation on MIOpen).
"""
import pytest
import torch

from golden import epe, fixture, model, run

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("small", [False, True])
def test_native_fp32_matches_reference_fixture(cuda, small):
    fix = fixture()
    m = model(small, fix, mixed_precision=False).to(cuda)
    name = "small" if small else "base"
    for p in range(2):
        lo, up = run(m, cuda, fix, p)
        d_lo = epe(lo, fix[f"{name}/pair{p}/flow_low"])
        d_up = epe(up, fix[f"{name}/pair{p}/flow_up_sub"])
        print(f"\n{name} pair {p}: native fp32 EPE vs reference  low {d_lo:.2e}  up {d_up:.2e} px")
        assert d_lo <= 1e-2 and d_up <= 1e-2, (p, d_lo, d_up)


@pytest.mark.parametrize("small", [False, True])
def test_native_bf16_within_3x_of_torch_autocast(cuda, small):
    fix = fixture()
    nat = model(small, fix, mixed_precision=True, amp_dtype="bf16").to(cuda)
    amp = model(small, fix, mixed_precision=True, amp_dtype="bf16", fused_update=False,
                native_encoder=False).to(cuda)
    name = "small" if small else "base"
    for p in range(2):
        _, up_n = run(nat, cuda, fix, p)
        _, up_a = run(amp, cuda, fix, p)
        ref = torch.from_numpy(fix[f"{name}/pair{p}/flow_up_sub"])
        dn, da = epe(up_n, ref), epe(up_a, ref)
        print(f"\n{name} pair {p}: bf16 EPE vs reference  native {dn:.4f}  torch autocast {da:.4f} px "
              f"(mean |flow| {float(ref.norm(dim=1).mean()):.2f})")
        assert dn <= max(3 * da, 1e-3), (p, dn, da)
