"""Golden parity on CPU: our RAFT (module path, fp32) vs outputs of the REAL reference
implementation stored in tests/fixtures/golden_demo_frames.npz (scripts/make_golden.py):
seed-0 weights, the reference's demo frames 0016-0018 (436x1024 padded to 440x1024),
20 iterations, test_mode -- the demo.py / ROS configuration."""
import pytest

from golden import epe, fixture, model, run


@pytest.mark.parametrize("small", [False, True])
def test_cpu_module_path_matches_reference_fixture(small):
    fix = fixture()
    m = model(small, fix, mixed_precision=False)
    name = "small" if small else "base"
    for p in range(2):
        lo, up = run(m, "cpu", fix, p)
        d_lo = epe(lo, fix[f"{name}/pair{p}/flow_low"])
        d_up = epe(up, fix[f"{name}/pair{p}/flow_up_sub"])
        assert d_lo <= 1e-3 and d_up <= 1e-3, (p, d_lo, d_up)
