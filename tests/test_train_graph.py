"""GraphedTrainStep: same update as the plain eager step (CPU), graph replay == eager (GPU)."""
import copy
from argparse import Namespace

import pytest
import torch

from raft_ros_amd.data.synthetic import synthetic_batch
from raft_ros_amd.models import RAFT
from raft_ros_amd.runtime import GraphedTrainStep
from raft_ros_amd.train.loss import sequence_loss
from raft_ros_amd.train.optim import fetch_optimizer

OARGS = Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100)


def _plain_step(model, opt, sched, batch, iters):
    opt.zero_grad(set_to_none=True)
    loss, _ = sequence_loss(model(*batch[:2], iters=iters), batch[2], batch[3], 0.8)
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
    opt.step()
    sched.step()
    return loss


def test_graphed_step_eager_matches_plain_step_cpu():
    torch.manual_seed(0)
    m1 = RAFT(Namespace(small=True, mixed_precision=False)).train()
    m2 = copy.deepcopy(m1)
    o1, s1 = fetch_optimizer(OARGS, m1)
    o2, s2 = fetch_optimizer(OARGS, m2)
    runner = GraphedTrainStep(m2, o2, sequence_loss, iters=2, clip=1.0, enabled=False)
    for i in range(2):
        batch = synthetic_batch(1, 128, 128, seed=i)
        l1 = _plain_step(m1, o1, s1, batch, 2)
        l2, _, norm = runner(*batch)
        s2.step()
        torch.testing.assert_close(l1, l2)
        assert torch.isfinite(norm)
    for (n, a), b in zip(m1.named_parameters(), m2.parameters()):
        # biases of convs followed by an (affine-free) instance norm have pure round-off
        # gradients, which AdamW amplifies to +-lr: compare those only to lr scale
        noise = n.startswith("fnet.") and n.endswith(".bias") and n != "fnet.conv2.bias"
        torch.testing.assert_close(a, b, rtol=1e-5, atol=2 * OARGS.lr if noise else 1e-6, msg=n)


@pytest.mark.gpu
def test_graphed_step_replay_matches_eager_gpu(cuda):
    torch.manual_seed(0)
    mk = lambda: RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16")).to(cuda).to(  # noqa: E731
        memory_format=torch.channels_last).train()
    m1 = mk()
    m2 = copy.deepcopy(m1)
    o1, s1 = fetch_optimizer(OARGS, m1, capturable=True)
    o2, s2 = fetch_optimizer(OARGS, m2, capturable=True)
    eager = GraphedTrainStep(m1, o1, sequence_loss, iters=3, enabled=False)
    graphed = GraphedTrainStep(m2, o2, sequence_loss, iters=3, enabled=True, warmup=2)
    for i in range(3):
        batch = synthetic_batch(2, 128, 160, seed=i, device=cuda)
        l1, _, n1 = eager(*batch)
        s1.step()
        l2, _, n2 = graphed(*batch)
        s2.step()
        torch.cuda.synchronize()
        bad = [n for n, p in m2.named_parameters() if not torch.isfinite(p.grad).all()]
        assert not bad, f"step {i}: non-finite graph grads in {bad[:8]} ({len(bad)} params)"
        # identical kernels in identical order; atomics in a few backward kernels -> small drift
        torch.testing.assert_close(l2, l1, rtol=2e-3, atol=2e-3)
        torch.testing.assert_close(n2, n1, rtol=5e-2, atol=1e-3)
    # early AdamW updates are ~lr*sign(g): round-off sign flips of near-zero gradients move
    # single elements by up to 2*lr, so bound the fraction of elements that disagree
    d = torch.cat([(a - b).abs().flatten() for a, b in zip(m1.parameters(), m2.parameters())])
    assert float((d > OARGS.lr).float().mean()) < 0.01, float(d.max())
    assert float(graphed.skipped) == 0.0


@pytest.mark.gpu
def test_trainer_graph_mode_runs_and_tracks_eager(cuda, tmp_path):
    """train.py --graph (the trainer's graphed step: static synthetic batches, capturable AdamW)
    trains like the eager trainer step (native clip + AdamW) from the same initial weights."""
    import train as train_cli
    from raft_ros_amd.train import trainer

    finals = {}
    for graph in (False, True):
        argv = ["--name", f"g{int(graph)}", "--stage", "synthetic", "--batch_size", "1", "--image_size", "128", "160",
                "--num_steps", "3", "--iters", "3", "--num_workers", "0", "--mixed_precision", "--lr", "4e-4",
                "--ckpt_dir", str(tmp_path / f"ck{int(graph)}"), "--log_dir", str(tmp_path / f"runs{int(graph)}"),
                "--gpus", "0"]
        if graph:
            argv.append("--graph")
        args = train_cli.build_parser().parse_args(argv)
        torch.manual_seed(args.seed)
        (tmp_path / f"ck{int(graph)}").mkdir()

        def keep(model, info, graph=graph):
            finals[graph] = {k: v.detach().float().clone() for k, v in model.state_dict().items()}

        trainer.train(args, on_finish=keep)
    moved = 0
    for k, a in finals[True].items():
        b = finals[False][k]
        assert torch.isfinite(a).all(), k
        if a.is_floating_point() and a.numel() > 1:
            d = (a - b).abs()
            # early AdamW updates are ~lr * sign(g): allow a few round-off sign flips
            assert float((d > 4e-4).float().mean()) < 0.02, (k, float(d.max()))
            moved += 1
    assert moved > 50
