"""Query-pixel sharding on the native kernels (parallel/query_shard.py): two gloo ranks
sharing cuda:0 each build the volume rows of half of the query pixels with the MFMA volume
GEMM and look them up with the dense lookup kernel; the gathered features -- and a whole
RAFT-base inference, bf16 AMP (fused update) and fp32 (split-bf16) -- equal the unsharded
native model's."""
import os
import tempfile
from argparse import Namespace

import pytest
import torch
import torch.multiprocessing as mp

from raft_ros_amd.parallel import ddp

pytestmark = pytest.mark.gpu


def _worker(rank, world, port, out):
    import torch.distributed as dist

    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.ops.corr import CorrPyramid
    from raft_ros_amd.ops import reference as ref
    from raft_ros_amd.parallel.query_shard import ShardedCorrPyramid

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    res = {}
    g = torch.Generator(device=dev).manual_seed(3)
    f1, f2 = torch.randn(2, 256, 24, 40, device=dev, generator=g), torch.randn(2, 256, 24, 40, device=dev, generator=g)
    coords = ref.coords_grid(2, 24, 40, device=dev) + torch.randn(2, 2, 24, 40, device=dev, generator=g) * 3
    for split in (True, False):
        sh = ShardedCorrPyramid(f1, f2, num_levels=4, radius=4, split=split)
        full = CorrPyramid(f1, f2, radius=4, split=split)
        dt = torch.float32 if split else torch.bfloat16
        a, b = sh(coords, out_dtype=dt).float(), full(coords, out_dtype=dt).float()
        res[f"lookup_err_{split}"] = ((a - b).abs().max() / b.abs().max()).item()
        res[f"bytes_ratio_{split}"] = sh.volume_bytes() / full.state.buf.numel() / full.state.buf.element_size()
    i1, i2, _, _ = synthetic_batch(1, 128, 192, seed=9, device=dev)
    for amp in (True, False):
        torch.manual_seed(0)
        model = RAFT(Namespace(small=False, mixed_precision=amp, amp_dtype="bf16")).to(dev).eval()
        with torch.no_grad():
            _, up = model(i1, i2, iters=4, test_mode=True)
            model.args.query_shard = True
            _, up_s = model(i1, i2, iters=4, test_mode=True)
        res[f"flow_epe_{amp}"] = (up_s - up).norm(dim=1).mean().item()
    torch.save(res, f"{out}.{rank}")
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_native_sharded_correlation_matches_unsharded(cuda):
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "r")
        mp.start_processes(_worker, args=(2, ddp.free_port(), out), nprocs=2, start_method="spawn")
        for r in range(2):
            res = torch.load(f"{out}.{r}", weights_only=True)
            print(r, res)
            assert res["lookup_err_True"] < 1e-5 and res["lookup_err_False"] < 1e-2, res
            assert 0.4 < res["bytes_ratio_True"] < 0.6 and 0.4 < res["bytes_ratio_False"] < 0.6, res
            # fp32 (split) is exact up to summation order; bf16 AMP features are rounded the same way
            assert res["flow_epe_False"] < 1e-3 and res["flow_epe_True"] < 2e-2, res
