"""Golden parity on CPU: our RAFT (module path, fp32) vs outputs of the REAL reference
implementation stored in tests/fixtures/golden_demo_frames.npz (scripts/make_golden.py):
seed-0 weights, the reference's demo frames 0016-0018 (436x1024 padded to 440x1024),
20 iterations, test_mode -- the demo.py / ROS configuration."""
import pytest
import torch

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


@pytest.mark.parametrize("small", [False, True])
def test_module_path_training_gradients_match_reference(small):
    """The CPU module path (reference op sequence) reproduces the REAL reference's training
    gradients (tests/fixtures/golden_grads.npz, scripts/make_golden_grads.py)."""
    from golden import grad_errors, grad_fixture, grad_step

    fix = grad_fixture()
    name = "small" if small else "base"
    m = model(small, fixture(), mixed_precision=False).train()
    torch.set_num_threads(8)
    loss, _, grads = grad_step(m, torch.device("cpu"))
    assert abs(loss - float(fix[f"{name}/loss"])) <= 1e-5 * abs(float(fix[f"{name}/loss"]))
    errs = grad_errors(grads, fix, name)
    worst = max(errs.values())
    assert worst <= 1e-4, sorted(errs.items(), key=lambda kv: -kv[1])[:5]
