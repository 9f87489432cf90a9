"""RAFT model on CPU: checkpoint schema, parity with the reference, API behaviour."""
import argparse

import pytest
import torch

from raft_ros_amd.models import RAFT


def _args(**kw):
    base = dict(small=False, mixed_precision=False, alternate_corr=False)
    base.update(kw)
    return argparse.Namespace(**base)


@pytest.mark.parametrize("small,params,keys", [(False, 5257536, 179), (True, 990162, 106)])
def test_parameter_count_and_state_dict(small, params, keys):
    m = RAFT(_args(small=small))
    assert sum(p.numel() for p in m.parameters()) == params
    assert len(m.state_dict()) == keys


def test_state_dict_schema_matches_appendix_a():
    sd = RAFT(_args()).state_dict()
    expect = {
        "fnet.conv1.weight": (64, 3, 7, 7),
        "fnet.conv2.weight": (256, 128, 1, 1),
        "cnet.conv2.weight": (256, 128, 1, 1),
        "cnet.layer2.0.downsample.1.running_var": (96,),
        "update_block.encoder.convc1.weight": (256, 324, 1, 1),
        "update_block.encoder.convf1.weight": (128, 2, 7, 7),
        "update_block.encoder.conv.weight": (126, 256, 3, 3),
        "update_block.gru.convz1.weight": (128, 384, 1, 5),
        "update_block.gru.convq2.weight": (128, 384, 5, 1),
        "update_block.flow_head.conv2.weight": (2, 256, 3, 3),
        "update_block.mask.2.weight": (576, 256, 1, 1),
    }
    for k, shape in expect.items():
        assert tuple(sd[k].shape) == shape, k
    assert not any(k.startswith("fnet.") and ".norm" in k for k in sd)  # InstanceNorm: no params
    small = RAFT(_args(small=True)).state_dict()
    assert tuple(small["update_block.encoder.convc1.weight"].shape) == (96, 196, 1, 1)
    assert tuple(small["update_block.gru.convz.weight"].shape) == (96, 242, 3, 3)


def test_args_mutation_like_reference():
    a = argparse.Namespace(small=True, mixed_precision=False)
    RAFT(a)
    assert a.corr_radius == 3 and a.corr_levels == 4 and a.dropout == 0 and a.alternate_corr is False


@pytest.mark.reference
@pytest.mark.parametrize("small", [True, False])
def test_forward_parity_with_reference(reference_core, small):
    torch.manual_seed(0)
    ref = reference_core.RAFT(_args(small=small)).eval()
    ours = RAFT(_args(small=small)).eval()
    ours.load_state_dict(ref.state_dict(), strict=True)
    i1 = torch.rand(1, 3, 128, 160) * 255
    i2 = torch.rand(1, 3, 128, 160) * 255
    with torch.no_grad():
        lo_r, up_r = ref(i1, i2, iters=3, test_mode=True)
        lo, up = ours(i1, i2, iters=3, test_mode=True)
        preds_r = ref(i1, i2, iters=2)
        preds = ours(i1, i2, iters=2)
    torch.testing.assert_close(up, up_r, rtol=1e-4, atol=1e-4)
    torch.testing.assert_close(lo, lo_r, rtol=1e-4, atol=1e-4)
    assert len(preds) == len(preds_r) == 2
    for a, b in zip(preds, preds_r):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-4)


@pytest.mark.reference
def test_backward_parity_with_reference(reference_core):
    torch.manual_seed(1)
    ref = reference_core.RAFT(_args(small=True)).train()
    ours = RAFT(_args(small=True)).train()
    ours.load_state_dict(ref.state_dict())
    i1 = torch.rand(1, 3, 128, 128) * 255
    i2 = torch.rand(1, 3, 128, 128) * 255
    sum(p.abs().mean() for p in ref(i1, i2, iters=2)).backward()
    sum(p.abs().mean() for p in ours(i1, i2, iters=2)).backward()
    gr = dict(ref.named_parameters())
    for n, p in ours.named_parameters():
        if gr[n].grad is None:
            continue
        torch.testing.assert_close(p.grad, gr[n].grad, rtol=2e-3, atol=1e-6)


def test_warm_start_and_shapes():
    m = RAFT(_args(small=True)).eval()
    i1 = torch.rand(2, 3, 128, 136) * 255
    with torch.no_grad():
        lo, up = m(i1, i1, iters=2, test_mode=True)
        lo2, up2 = m(i1, i1, iters=1, flow_init=lo, test_mode=True)
    assert lo.shape == (2, 2, 16, 17) and up.shape == (2, 2, 128, 136)
    assert up2.shape == up.shape


def test_small_inputs_fail_loudly():
    m = RAFT(_args(small=True)).eval()
    with pytest.raises(ValueError):
        m(torch.rand(1, 3, 64, 256), torch.rand(1, 3, 64, 256), iters=1)


def test_alternate_corr_matches_dense_on_cpu():
    torch.manual_seed(0)
    a = RAFT(_args()).eval()
    b = RAFT(_args(alternate_corr=True)).eval()
    b.load_state_dict(a.state_dict())
    i1 = torch.rand(1, 3, 128, 128) * 255
    i2 = torch.rand(1, 3, 128, 128) * 255
    with torch.no_grad():
        _, ua = a(i1, i2, iters=2, test_mode=True)
        _, ub = b(i1, i2, iters=2, test_mode=True)
    torch.testing.assert_close(ua, ub, rtol=1e-3, atol=1e-3)


def test_freeze_bn():
    m = RAFT(_args()).train()
    m.freeze_bn()
    bns = [x for x in m.modules() if isinstance(x, torch.nn.BatchNorm2d)]
    assert bns and all(not x.training for x in bns)


def test_graphed_runner_falls_back_to_eager_on_cpu():
    from argparse import Namespace

    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.runtime import GraphedRAFT

    model = RAFT(Namespace(small=True, mixed_precision=False)).eval()
    i1, i2, _, _ = synthetic_batch(1, 128, 128, seed=0)
    with torch.no_grad():
        ref = model(i1, i2, iters=2, test_mode=True)[1]
    out = GraphedRAFT(model, iters=2)(i1, i2)[1]
    torch.testing.assert_close(out, ref)
