"""Query-pixel sharding of the correlation volume (parallel/query_shard.py) on two gloo
ranks: the sharded lookup and a whole RAFT-small inference equal the unsharded ones, and
each rank stores half of the volume."""
import os
import tempfile
from argparse import Namespace

import torch
import torch.multiprocessing as mp

from raft_ros_amd.parallel import ddp
from raft_ros_amd.parallel.query_shard import shard_range


def test_shard_range_partitions():
    for n in (1, 7, 64, 1000):
        for w in (1, 2, 3, 8):
            rs = [shard_range(n, r, w) for r in range(w)]
            assert rs[0][0] == 0 and rs[-1][1] == n
            assert all(a[1] == b[0] for a, b in zip(rs, rs[1:]))
            sizes = [hi - lo for lo, hi in rs]
            assert max(sizes) - min(sizes) <= 1


def _worker(rank, world, port, out):
    import torch.distributed as dist

    from raft_ros_amd.models import RAFT
    from raft_ros_amd.ops import reference as ref
    from raft_ros_amd.parallel.query_shard import ShardedCorrPyramid

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    g = torch.Generator().manual_seed(3)
    # >= 16 px per side: the coarsest level keeps 2+ pixels (the reference lookup is NaN on 1)
    f1, f2 = torch.randn(2, 32, 17, 21, generator=g), torch.randn(2, 32, 17, 21, generator=g)
    coords = ref.coords_grid(2, 17, 21) + torch.randn(2, 2, 17, 21, generator=g) * 3
    sh = ShardedCorrPyramid(f1, f2, num_levels=4, radius=3)
    full = ref.pyramid_lookup(ref.build_pyramid(ref.corr_volume(f1, f2), 4), coords, 3)
    lookup_err = (sh(coords) - full).abs().max().item()
    full_bytes = sum(t.numel() * 4 for t in ref.build_pyramid(ref.corr_volume(f1, f2), 4))

    import raft_ros_amd.parallel.query_shard as qs

    calls = [0]
    orig = qs.ShardedCorrPyramid.__call__

    def counted(self, *a, **k):
        calls[0] += 1
        return orig(self, *a, **k)

    qs.ShardedCorrPyramid.__call__ = counted
    torch.manual_seed(0)
    model = RAFT(Namespace(small=True)).eval()
    i1 = torch.rand(1, 3, 128, 160, generator=g) * 255
    i2 = torch.rand(1, 3, 128, 160, generator=g) * 255
    with torch.no_grad():
        lo, up = model(i1, i2, iters=3, test_mode=True)
        model.args.query_shard = True
        lo_s, up_s = model(i1, i2, iters=3, test_mode=True)
    res = {"lookup_err": lookup_err, "flow_err": (up_s - up).abs().max().item(), "calls": calls[0],
           "bytes_ratio": sh.volume_bytes() / full_bytes}
    torch.save(res, f"{out}.{rank}")
    dist.destroy_process_group()


def test_sharded_lookup_and_inference_match_unsharded():
    with tempfile.TemporaryDirectory() as tmp:
        out = os.path.join(tmp, "r")
        mp.start_processes(_worker, args=(2, ddp.free_port(), out), nprocs=2, start_method="spawn")
        for r in range(2):
            res = torch.load(f"{out}.{r}", weights_only=True)
            assert res["lookup_err"] < 1e-4, res
            assert res["flow_err"] < 1e-3, res
            assert 0.4 < res["bytes_ratio"] < 0.6, res
            assert res["calls"] == 3, res  # one sharded lookup per refinement iteration
