"""Debug helper: captured fwd+bwd replays with eager optimizer steps in between."""
import sys
from argparse import Namespace

import torch

sys.path.insert(0, ".")
from raft_ros_amd.data.synthetic import synthetic_batch  # noqa: E402
from raft_ros_amd.models import RAFT  # noqa: E402
from raft_ros_amd.runtime import GraphedTrainStep  # noqa: E402
from raft_ros_amd.train.loss import sequence_loss  # noqa: E402
from raft_ros_amd.train.optim import fetch_optimizer  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
OARGS = Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100)
mode = sys.argv[1] if len(sys.argv) > 1 else "opt"
m = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16")).to(dev).to(
    memory_format=torch.channels_last).train()
o, s = fetch_optimizer(OARGS, m, capturable=True)
r = GraphedTrainStep(m, o, sequence_loss, iters=3)
r._bind_flat_grads()
r.static_in = [t.clone() for t in synthetic_batch(2, 128, 160, seed=0, device=dev)]
side = torch.cuda.Stream()
side.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(side):
    for _ in range(2):
        r._fwd_bwd(*r.static_in)
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=side):
    loss, _ = r._fwd_bwd(*r.static_in)
for i in range(4):
    g.replay()
    torch.cuda.synchronize()
    bad = [n for n, p in m.named_parameters() if not torch.isfinite(p.grad).all()]
    print(f"replay {i}: loss {float(loss):.4f} norm {float(r.flat.norm()):.3f} nonfinite {len(bad)} {bad[:6]}", flush=True)
    with torch.no_grad():
        if mode == "opt":
            o.step()
        elif mode == "perturb":
            for p in m.parameters():
                p.add_(torch.randn_like(p) * 1e-4)
print("done")
