"""Optical-flow training data: file manifests, decoding workers, stage mixtures.

Re-design of the reference data layer (core/datasets.py:18-234):

* a dataset is a *manifest* -- a list of ``Sample(img1, img2, flow, kind, extra)``
  records built by one function per on-disk layout (``sintel_manifest``,
  ``chairs_manifest``, ``things_manifest``, ``kitti_manifest``,
  ``hd1k_manifest``; the directory layouts are those of the public datasets);
* DataLoader workers only DECODE (``decode_sample``: PNG/PPM, ``.flo``, PFM,
  KITTI 16-bit PNG) and hand uint8 images + flow to ``collate_padded``;
* augmentation runs batched on the training device (``data.augment``:
  ``BatchAugmentor``), with per-sample ``AugSpec`` so one batch can mix the
  dense and sparse datasets of a stage (``stage_mixture``, the reference's
  proportions: sintel stage = 100 clean + 100 final + 200 KITTI + 5 HD1K +
  things);
* ``fetch_dataloader`` returns an iterator of augmented device batches and
  shards the mixture over DDP ranks (``batch_size`` stays the GLOBAL batch).

The reference class names (``MpiSintel``, ``FlyingChairs``, ``FlyingThings3D``,
``KITTI``, ``HD1K``) remain as manifest-backed map-style datasets with the
reference's item format, for evaluation and per-item use (``aug_params`` then
augments the single item through the same batched code on the CPU).
Dataset roots default to ``datasets/<name>``; ``RAFT_DATASET_ROOT`` redirects.
"""
from __future__ import annotations

import json
import os
import os.path as osp
from glob import glob
from typing import Dict, List, NamedTuple, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.utils.data as data

from . import frame_utils
from .augment import AugSpec, BatchAugmentor, augment_one, collate_padded
from .synthetic import SyntheticFlowDataset


class Sample(NamedTuple):
    img1: str
    img2: str
    flow: Optional[str]  # None for test splits
    kind: str            # 'dense' (.flo / .pfm) or 'sparse' (KITTI-format 16-bit PNG)
    extra: object = None


def _root(default: str, name: Optional[str] = None) -> str:
    base = os.environ.get("RAFT_DATASET_ROOT")
    return osp.join(base, name or osp.basename(default.rstrip("/"))) if base else default


def chairs_split() -> np.ndarray:
    """FlyingChairs train/validation split (1 = training, 2 = validation), 22872 entries."""
    with open(osp.join(osp.dirname(__file__), "chairs_split.rle.json")) as f:
        spec = json.load(f)
    return np.concatenate([np.full(n, v, dtype=np.int32) for v, n in spec["runs"]])


# ----------------------------------------------------------------------------- manifests
def _pairs(frames: Sequence[str]) -> List[Tuple[str, str]]:
    return list(zip(frames[:-1], frames[1:]))


def sintel_manifest(root="datasets/Sintel", split="training", dstype="clean") -> List[Sample]:
    root = _root(root)
    img_root = osp.join(root, split, dstype)
    out: List[Sample] = []
    for scene in sorted(os.listdir(img_root)) if osp.isdir(img_root) else []:
        frames = sorted(glob(osp.join(img_root, scene, "*.png")))
        flows = sorted(glob(osp.join(root, split, "flow", scene, "*.flo"))) if split != "test" else []
        for i, (a, b) in enumerate(_pairs(frames)):
            out.append(Sample(a, b, flows[i] if flows else None, "dense", (scene, i)))
    return out


def chairs_manifest(root="datasets/FlyingChairs_release/data", split="training") -> List[Sample]:
    base = os.environ.get("RAFT_DATASET_ROOT")
    root = osp.join(base, "FlyingChairs_release", "data") if base else root
    images = sorted(glob(osp.join(root, "*.ppm")))
    flows = sorted(glob(osp.join(root, "*.flo")))
    assert len(images) == 2 * len(flows), (len(images), len(flows))
    want = {"training": 1, "validation": 2}[split]
    ids = chairs_split()
    return [Sample(images[2 * i], images[2 * i + 1], f, "dense") for i, f in enumerate(flows) if ids[i] == want]


def things_manifest(root="datasets/FlyingThings3D", dstype="frames_cleanpass") -> List[Sample]:
    """Left camera, both directions: into_future pairs (t, t+1) with flow_t, into_past pairs
    (t+1, t) with flow_{t+1}."""
    root = _root(root)
    out: List[Sample] = []
    for direction in ("into_future", "into_past"):
        img_dirs = sorted(osp.join(d, "left") for d in glob(osp.join(root, dstype, "TRAIN/*/*")))
        flow_dirs = sorted(osp.join(d, direction, "left") for d in glob(osp.join(root, "optical_flow/TRAIN/*/*")))
        for idir, fdir in zip(img_dirs, flow_dirs):
            frames = sorted(glob(osp.join(idir, "*.png")))
            flows = sorted(glob(osp.join(fdir, "*.pfm")))
            for i in range(len(flows) - 1):
                if direction == "into_future":
                    out.append(Sample(frames[i], frames[i + 1], flows[i], "dense"))
                else:
                    out.append(Sample(frames[i + 1], frames[i], flows[i + 1], "dense"))
    return out


def kitti_manifest(root="datasets/KITTI", split="training") -> List[Sample]:
    root = osp.join(_root(root), split)
    a = sorted(glob(osp.join(root, "image_2/*_10.png")))
    b = sorted(glob(osp.join(root, "image_2/*_11.png")))
    flows = sorted(glob(osp.join(root, "flow_occ/*_10.png"))) if split == "training" else [None] * len(a)
    return [Sample(x, y, f, "sparse", [osp.basename(x)]) for x, y, f in zip(a, b, flows)]


def hd1k_manifest(root="datasets/HD1k") -> List[Sample]:
    root = _root(root)
    out: List[Sample] = []
    seq = 0
    while True:
        flows = sorted(glob(osp.join(root, "hd1k_flow_gt", "flow_occ/%06d_*.png" % seq)))
        if not flows:
            return out
        frames = sorted(glob(osp.join(root, "hd1k_input", "image_2/%06d_*.png" % seq)))
        out += [Sample(frames[i], frames[i + 1], flows[i], "sparse") for i in range(len(flows) - 1)]
        seq += 1


# ----------------------------------------------------------------------------- decoding
def _rgb(path: str) -> np.ndarray:
    img = np.asarray(frame_utils.read_gen(path)).astype(np.uint8)
    if img.ndim == 2:
        img = np.repeat(img[..., None], 3, axis=2)
    return np.ascontiguousarray(img[..., :3])


def decode_sample(s: Sample) -> Dict[str, torch.Tensor]:
    """Files -> uint8 HWC images, (H, W, 2) fp32 flow and (H, W) valid (dense: |flow| < 1000)."""
    out = {"img1": torch.from_numpy(_rgb(s.img1)), "img2": torch.from_numpy(_rgb(s.img2))}
    h, w = out["img1"].shape[:2]
    if s.flow is None:
        out["flow"] = torch.zeros(h, w, 2)
        out["valid"] = torch.zeros(h, w)
    elif s.kind == "sparse":
        flow, valid = frame_utils.readFlowKITTI(s.flow)
        out["flow"] = torch.from_numpy(np.ascontiguousarray(flow, dtype=np.float32))
        out["valid"] = torch.from_numpy(np.ascontiguousarray(valid, dtype=np.float32))
    else:
        flow = torch.from_numpy(np.ascontiguousarray(np.asarray(frame_utils.read_gen(s.flow)), dtype=np.float32))
        out["flow"] = flow
        out["valid"] = ((flow[..., 0].abs() < 1000) & (flow[..., 1].abs() < 1000)).float()
    return out


class FlowFiles(data.Dataset):
    """Map-style dataset over (sample, augmentation-spec id) entries; items are decoded
    samples for ``collate_padded`` (augmentation happens batched, on the device)."""

    def __init__(self, entries: List[Tuple[Sample, int]]):
        self.entries = entries

    def __len__(self):
        return len(self.entries)

    def __getitem__(self, i):
        s, spec = self.entries[i]
        out = decode_sample(s)
        out["spec"] = spec
        return out


# ----------------------------------------------------------------------------- reference-style classes
class FlowDataset(data.Dataset):
    """Manifest-backed dataset with the reference's item format:
    ``(img1, img2, flow, valid)`` float CHW tensors, or ``(img1, img2, extra)`` for test
    splits.  With ``aug_params`` each item is augmented (same code as the batched path)."""

    sparse = False

    def __init__(self, aug_params=None, samples: Optional[List[Sample]] = None):
        self.samples: List[Sample] = samples or []
        self.spec = None if aug_params is None else AugSpec(
            crop_size=tuple(aug_params["crop_size"]), min_scale=aug_params.get("min_scale", -0.2),
            max_scale=aug_params.get("max_scale", 0.5), do_flip=aug_params.get("do_flip", not self.sparse),
            sparse=self.sparse)

    @property
    def is_test(self) -> bool:
        return bool(self.samples) and self.samples[0].flow is None

    # reference attribute names
    @property
    def image_list(self):
        return [[s.img1, s.img2] for s in self.samples]

    @property
    def flow_list(self):
        return [s.flow for s in self.samples if s.flow is not None]

    @property
    def extra_info(self):
        return [s.extra for s in self.samples]

    def __len__(self):
        return len(self.samples)

    def __rmul__(self, v: int):
        self.samples = v * self.samples
        return self

    def __getitem__(self, index):
        s = self.samples[index % len(self.samples)]
        d = decode_sample(s)
        if s.flow is None:
            return d["img1"].permute(2, 0, 1).float(), d["img2"].permute(2, 0, 1).float(), s.extra
        if self.spec is not None:
            return augment_one(d, self.spec)
        return (d["img1"].permute(2, 0, 1).float(), d["img2"].permute(2, 0, 1).float(), d["flow"].permute(2, 0, 1),
                d["valid"])


class MpiSintel(FlowDataset):
    def __init__(self, aug_params=None, split="training", root="datasets/Sintel", dstype="clean"):
        super().__init__(aug_params, sintel_manifest(root, split, dstype))


class FlyingChairs(FlowDataset):
    def __init__(self, aug_params=None, split="train", root="datasets/FlyingChairs_release/data"):
        super().__init__(aug_params, chairs_manifest(root, "validation" if split == "validation" else "training"))


class FlyingThings3D(FlowDataset):
    def __init__(self, aug_params=None, root="datasets/FlyingThings3D", dstype="frames_cleanpass"):
        super().__init__(aug_params, things_manifest(root, dstype))


class KITTI(FlowDataset):
    sparse = True

    def __init__(self, aug_params=None, split="training", root="datasets/KITTI"):
        super().__init__(aug_params, kitti_manifest(root, split))


class HD1K(FlowDataset):
    sparse = True

    def __init__(self, aug_params=None, root="datasets/HD1k"):
        super().__init__(aug_params, hd1k_manifest(root))


# ----------------------------------------------------------------------------- stage mixtures
def stage_mixture(stage: str, image_size, train_ds: str = "C+T+K+S+H"):
    """-> [(repeat, manifest, AugSpec)] with the reference's per-stage proportions and
    augmentation ranges (core/datasets.py:199-227)."""
    crop = tuple(image_size)

    def spec(lo, hi, flip=True, sparse=False):
        return AugSpec(crop, lo, hi, flip, sparse)

    if stage == "chairs":
        return [(1, chairs_manifest(split="training"), spec(-0.1, 1.0))]
    if stage == "things":
        s = spec(-0.4, 0.8)
        return [(1, things_manifest(dstype="frames_cleanpass"), s), (1, things_manifest(dstype="frames_finalpass"), s)]
    if stage == "sintel":
        s = spec(-0.2, 0.6)
        mix = [(100, sintel_manifest(dstype="clean"), s), (100, sintel_manifest(dstype="final"), s)]
        if train_ds == "C+T+K+S+H":
            mix += [(200, kitti_manifest(split="training"), spec(-0.3, 0.5, sparse=True)),
                    (5, hd1k_manifest(), spec(-0.5, 0.2, sparse=True))]
        return mix + [(1, things_manifest(dstype="frames_cleanpass"), s)]
    if stage == "kitti":
        return [(1, kitti_manifest(split="training"), spec(-0.2, 0.4, flip=False, sparse=True))]
    raise ValueError(f"unknown stage {stage!r}")


def build_train_dataset(stage: str, image_size, train_ds: str = "C+T+K+S+H"):
    """Stage mixture as a ``FlowFiles`` dataset + its AugSpecs (or the synthetic dataset)."""
    if stage == "synthetic":
        return SyntheticFlowDataset(size=tuple(image_size), length=100000), None
    entries: List[Tuple[Sample, int]] = []
    specs: List[AugSpec] = []
    for repeat, manifest, sp in stage_mixture(stage, image_size, train_ds):
        if sp not in specs:
            specs.append(sp)
        sid = specs.index(sp)
        entries += repeat * [(m, sid) for m in manifest]
    return FlowFiles(entries), specs


class AugmentedLoader:
    """Iterates a DataLoader of decoded, padded batches and yields augmented device batches
    ``(img1, img2, flow, valid)``; exposes ``sampler`` for ``set_epoch``."""

    def __init__(self, loader: data.DataLoader, augmentor: BatchAugmentor):
        self.loader = loader
        self.augmentor = augmentor
        self.sampler = loader.sampler
        self.batch_sampler = loader.batch_sampler

    def __len__(self):
        return len(self.loader)

    def __iter__(self):
        for batch in self.loader:
            yield self.augmentor(batch)


def fetch_dataloader(args, TRAIN_DS: str = "C+T+K+S+H"):
    """Training batches for ``args.stage``.  ``args.batch_size`` is the GLOBAL batch (as in
    the reference): under DDP every rank draws the same shuffled global batch and loads its
    own slice of it (``parallel/batching.py``: uneven splits such as 10 over 8 ranks are
    exact; a rank with no sample gets an :class:`IdleLoader`), and augments with its own
    generator (seeded by ``args.seed`` + rank) on ``args.device``."""
    from ..parallel.batching import GlobalBatchSampler, IdleLoader, rank_batch_sizes

    world = int(getattr(args, "world_size", 1) or 1)
    rank = int(getattr(args, "rank", 0) or 0)
    pool = int(getattr(args, "synthetic_pool", 8) or 0)
    if args.stage == "synthetic" and pool > 0:  # device-resident pool (data/synthetic.py DeviceSyntheticLoader)
        from .synthetic import DeviceSyntheticLoader

        sizes = rank_batch_sizes(args.batch_size, world, getattr(args, "batch_split", "balanced"))
        steps = 100000 // args.batch_size
        if rank == 0:
            # a throughput stage, not a dataset: each rank replays `pool` fixed batches of its own
            # (seeded by rank), so only pool * batch_size distinct pairs are ever seen and the
            # global-batch alignment of GlobalBatchSampler does not apply (--synthetic_pool 0:
            # 100000 distinct pairs generated by the CPU DataLoader, globally aligned)
            print("Training on a device-resident synthetic pool: %d batches per rank replayed for %d steps per epoch "
                  "(%d distinct pairs on rank 0)" % (pool, steps, pool * max(sizes[0], 1)))
        if sizes[rank] == 0:
            return IdleLoader(GlobalBatchSampler(steps * args.batch_size, sizes, rank))
        device = getattr(args, "device", None) or ("cuda" if torch.cuda.is_available() else "cpu")
        return DeviceSyntheticLoader(sizes[rank], args.image_size, device, pool=pool,
                                     seed=int(getattr(args, "seed", 1234)) + 1000 * rank, steps=steps)
    dataset, specs = build_train_dataset(args.stage, args.image_size, TRAIN_DS)
    workers = int(getattr(args, "num_workers", 4))
    kw = dict(num_workers=workers, pin_memory=torch.cuda.is_available(), persistent_workers=workers > 0)
    if world > 1:
        sizes = rank_batch_sizes(args.batch_size, world, getattr(args, "batch_split", "balanced"))
        bs = GlobalBatchSampler(len(dataset), sizes, rank, seed=int(getattr(args, "seed", 1234)))
        if sizes[rank] == 0:
            if rank == 0:
                print("Training with %d image pairs" % len(dataset))
            return IdleLoader(bs)
        kw["batch_sampler"] = bs
    else:
        kw.update(batch_size=args.batch_size, shuffle=True, drop_last=True)
    if rank == 0:
        print("Training with %d image pairs" % len(dataset))
    if specs is None:  # synthetic: already-final tensors
        return data.DataLoader(dataset, **kw)
    loader = data.DataLoader(dataset, collate_fn=collate_padded, **kw)
    device = getattr(args, "device", None) or ("cuda" if torch.cuda.is_available() else "cpu")
    seed = int(getattr(args, "seed", 1234)) + 1000 * rank
    return AugmentedLoader(loader, BatchAugmentor(specs, seed=seed, device=device))
