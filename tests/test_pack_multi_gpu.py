"""pack_conv_weights_multi (every refinement-step layer in one launch, csrc/weights.hip) ==
the single-layer packs, bitwise, for the bf16 / fp16 layouts of the fused step and the
split-bf16 layouts of the fp32 step (RAFT-base and RAFT-small)."""
from argparse import Namespace

import pytest
import torch

from raft_ros_amd.models import RAFT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("small", [False, True])
@pytest.mark.parametrize("f16", [False, True])
def test_multi_pack_matches_single_layer_packs(cuda, small, f16):
    from raft_ros_amd.ops import conv as C
    from raft_ros_amd.ops import update_fused, update_fused_small

    torch.manual_seed(0)
    m = RAFT(Namespace(small=small, mixed_precision=True)).to(cuda).to(memory_format=torch.channels_last)
    blk = m.update_block
    if small:
        layers = [([x.weight for x in mods(blk)], [x.bias for x in mods(blk)], segs, 1.0, dgrad)
                  for _, mods, segs, dgrad in update_fused_small._LAYERS]
    else:
        layers = [([x.weight for x in mods(blk)], [x.bias for x in mods(blk)], segs, scale, dgrad)
                  for _, mods, segs, scale, dgrad in update_fused._LAYERS]
    got = C.pack_weights_multi(layers, f16=f16)
    for (w, b, segs, scale, dgrad), (wf, wd, bias) in zip(layers, got):
        wf1, wd1, b1 = C.pack_weights(w, b, segs, scale, dgrad=dgrad, f16=f16)
        assert torch.equal(wf, wf1)
        assert (wd is None) == (wd1 is None)
        if wd is not None:
            assert torch.equal(wd, wd1)
        assert torch.equal(bias, b1)


@pytest.mark.parametrize("small", [False, True])
def test_multi_pack_split_matches_single_layer_packs(cuda, small):
    from raft_ros_amd.ops import conv as C
    from raft_ros_amd.ops import update_split, update_split_small

    torch.manual_seed(0)
    m = RAFT(Namespace(small=small, mixed_precision=False)).to(cuda)
    blk = m.update_block
    mod = update_split_small if small else update_split
    layers = []
    for spec in mod._LAYERS:
        _, mods, fsrc, dsegs, dyg = spec[:5]
        scale = spec[5] if len(spec) > 5 else 1.0
        gdy = dyg[0][2] if dsegs is not None else 0
        layers.append(([x.weight for x in mods(blk)], [x.bias for x in mods(blk)],
                       [s for src in fsrc for s in src], scale, gdy))
    got = C.pack_weights_multi(layers, split=True)
    for (w, b, segs, scale, gdy), (wf, wd, bias) in zip(layers, got):
        wf1, wd1, b1 = C.pack_weights_split_native(w, b, segs, scale, gdy)
        assert torch.equal(wf, wf1)
        if gdy:
            assert torch.equal(wd, wd1)
        assert torch.equal(bias, b1)
