"""Optical-flow datasets and the stage mixtures (reference core/datasets.py).

Classes keep the reference names, constructor arguments and file layouts
(``MpiSintel``, ``FlyingChairs``, ``FlyingThings3D``, ``KITTI``, ``HD1K``); the
dataset root defaults to ``datasets/<name>`` like the reference and can be
redirected with ``RAFT_DATASET_ROOT`` or ``fetch_dataloader(..., root=...)``.
Differences:

* ``fetch_dataloader`` takes ``args.distributed`` into account (a
  ``DistributedSampler`` per rank with ``batch_size`` = the per-rank share of
  the global batch), pins host memory and supports ``stage='synthetic'``;
* per-worker seeding uses the worker id plus the rank, so DDP ranks do not
  draw identical augmentations;
* the FlyingChairs split ships as ``chairs_split.rle.json`` next to this file.
"""
from __future__ import annotations

import json
import os
import os.path as osp
import random
from glob import glob

import numpy as np
import torch
import torch.utils.data as data

from . import frame_utils
from .augmentor import FlowAugmentor, SparseFlowAugmentor
from .synthetic import SyntheticFlowDataset


def _root(default: str) -> str:
    base = os.environ.get("RAFT_DATASET_ROOT")
    return osp.join(base, osp.basename(default.rstrip("/"))) if base else default


def chairs_split() -> np.ndarray:
    """FlyingChairs train/validation split (1 = training, 2 = validation), 22872 entries."""
    with open(osp.join(osp.dirname(__file__), "chairs_split.rle.json")) as f:
        spec = json.load(f)
    return np.concatenate([np.full(n, v, dtype=np.int32) for v, n in spec["runs"]])


class FlowDataset(data.Dataset):
    def __init__(self, aug_params=None, sparse=False):
        self.augmentor = None
        self.sparse = sparse
        if aug_params is not None:
            self.augmentor = SparseFlowAugmentor(**aug_params) if sparse else FlowAugmentor(**aug_params)
        self.is_test = False
        self.init_seed = False
        self.flow_list = []
        self.image_list = []
        self.extra_info = []

    def __getitem__(self, index):
        if self.is_test:
            img1 = np.array(frame_utils.read_gen(self.image_list[index][0])).astype(np.uint8)[..., :3]
            img2 = np.array(frame_utils.read_gen(self.image_list[index][1])).astype(np.uint8)[..., :3]
            img1 = torch.from_numpy(img1).permute(2, 0, 1).float()
            img2 = torch.from_numpy(img2).permute(2, 0, 1).float()
            return img1, img2, self.extra_info[index]

        if not self.init_seed:
            info = torch.utils.data.get_worker_info()
            if info is not None:
                rank = int(os.environ.get("RANK", "0"))
                seed = info.id + 1000 * rank
                torch.manual_seed(seed)
                np.random.seed(seed)
                random.seed(seed)
                self.init_seed = True

        index = index % len(self.image_list)
        valid = None
        if self.sparse:
            flow, valid = frame_utils.readFlowKITTI(self.flow_list[index])
        else:
            flow = frame_utils.read_gen(self.flow_list[index])
        img1 = frame_utils.read_gen(self.image_list[index][0])
        img2 = frame_utils.read_gen(self.image_list[index][1])

        flow = np.array(flow).astype(np.float32)
        img1 = np.array(img1).astype(np.uint8)
        img2 = np.array(img2).astype(np.uint8)
        if img1.ndim == 2:  # grayscale
            img1 = np.tile(img1[..., None], (1, 1, 3))
            img2 = np.tile(img2[..., None], (1, 1, 3))
        else:
            img1, img2 = img1[..., :3], img2[..., :3]

        if self.augmentor is not None:
            if self.sparse:
                img1, img2, flow, valid = self.augmentor(img1, img2, flow, valid)
            else:
                img1, img2, flow = self.augmentor(img1, img2, flow)

        img1 = torch.from_numpy(img1).permute(2, 0, 1).float()
        img2 = torch.from_numpy(img2).permute(2, 0, 1).float()
        flow = torch.from_numpy(flow).permute(2, 0, 1).float()
        if valid is not None:
            valid = torch.from_numpy(np.asarray(valid))
        else:
            valid = (flow[0].abs() < 1000) & (flow[1].abs() < 1000)
        return img1, img2, flow, valid.float()

    def __rmul__(self, v):
        self.flow_list = v * self.flow_list
        self.image_list = v * self.image_list
        return self

    def __len__(self):
        return len(self.image_list)


class MpiSintel(FlowDataset):
    def __init__(self, aug_params=None, split="training", root="datasets/Sintel", dstype="clean"):
        super().__init__(aug_params)
        root = _root(root)
        flow_root = osp.join(root, split, "flow")
        image_root = osp.join(root, split, dstype)
        if split == "test":
            self.is_test = True
        for scene in sorted(os.listdir(image_root)) if osp.isdir(image_root) else []:
            images = sorted(glob(osp.join(image_root, scene, "*.png")))
            for i in range(len(images) - 1):
                self.image_list.append([images[i], images[i + 1]])
                self.extra_info.append((scene, i))
            if split != "test":
                self.flow_list += sorted(glob(osp.join(flow_root, scene, "*.flo")))


class FlyingChairs(FlowDataset):
    def __init__(self, aug_params=None, split="train", root="datasets/FlyingChairs_release/data"):
        super().__init__(aug_params)
        root = _root(root) if not os.environ.get("RAFT_DATASET_ROOT") else osp.join(
            os.environ["RAFT_DATASET_ROOT"], "FlyingChairs_release", "data")
        images = sorted(glob(osp.join(root, "*.ppm")))
        flows = sorted(glob(osp.join(root, "*.flo")))
        assert len(images) // 2 == len(flows)
        split_list = chairs_split()
        for i in range(len(flows)):
            xid = split_list[i]
            if (split == "training" and xid == 1) or (split == "validation" and xid == 2):
                self.flow_list.append(flows[i])
                self.image_list.append([images[2 * i], images[2 * i + 1]])


class FlyingThings3D(FlowDataset):
    def __init__(self, aug_params=None, root="datasets/FlyingThings3D", dstype="frames_cleanpass"):
        super().__init__(aug_params)
        root = _root(root)
        for cam in ["left"]:
            for direction in ["into_future", "into_past"]:
                image_dirs = sorted(glob(osp.join(root, dstype, "TRAIN/*/*")))
                image_dirs = sorted(osp.join(f, cam) for f in image_dirs)
                flow_dirs = sorted(glob(osp.join(root, "optical_flow/TRAIN/*/*")))
                flow_dirs = sorted(osp.join(f, direction, cam) for f in flow_dirs)
                for idir, fdir in zip(image_dirs, flow_dirs):
                    images = sorted(glob(osp.join(idir, "*.png")))
                    flows = sorted(glob(osp.join(fdir, "*.pfm")))
                    for i in range(len(flows) - 1):
                        if direction == "into_future":
                            self.image_list.append([images[i], images[i + 1]])
                            self.flow_list.append(flows[i])
                        else:
                            self.image_list.append([images[i + 1], images[i]])
                            self.flow_list.append(flows[i + 1])


class KITTI(FlowDataset):
    def __init__(self, aug_params=None, split="training", root="datasets/KITTI"):
        super().__init__(aug_params, sparse=True)
        if split == "testing":
            self.is_test = True
        root = osp.join(_root(root), split)
        images1 = sorted(glob(osp.join(root, "image_2/*_10.png")))
        images2 = sorted(glob(osp.join(root, "image_2/*_11.png")))
        for img1, img2 in zip(images1, images2):
            self.extra_info.append([osp.basename(img1)])
            self.image_list.append([img1, img2])
        if split == "training":
            self.flow_list = sorted(glob(osp.join(root, "flow_occ/*_10.png")))


class HD1K(FlowDataset):
    def __init__(self, aug_params=None, root="datasets/HD1k"):
        super().__init__(aug_params, sparse=True)
        root = _root(root)
        seq = 0
        while True:
            flows = sorted(glob(osp.join(root, "hd1k_flow_gt", "flow_occ/%06d_*.png" % seq)))
            images = sorted(glob(osp.join(root, "hd1k_input", "image_2/%06d_*.png" % seq)))
            if not flows:
                break
            for i in range(len(flows) - 1):
                self.flow_list.append(flows[i])
                self.image_list.append([images[i], images[i + 1]])
            seq += 1


def build_train_dataset(stage: str, image_size, train_ds: str = "C+T+K+S+H"):
    """The reference's stage mixtures (core/datasets.py:199-227)."""
    if stage == "chairs":
        aug = {"crop_size": image_size, "min_scale": -0.1, "max_scale": 1.0, "do_flip": True}
        return FlyingChairs(aug, split="training")
    if stage == "things":
        aug = {"crop_size": image_size, "min_scale": -0.4, "max_scale": 0.8, "do_flip": True}
        return FlyingThings3D(aug, dstype="frames_cleanpass") + FlyingThings3D(aug, dstype="frames_finalpass")
    if stage == "sintel":
        aug = {"crop_size": image_size, "min_scale": -0.2, "max_scale": 0.6, "do_flip": True}
        things = FlyingThings3D(aug, dstype="frames_cleanpass")
        clean = MpiSintel(aug, split="training", dstype="clean")
        final = MpiSintel(aug, split="training", dstype="final")
        if train_ds == "C+T+K+S+H":
            kitti = KITTI({"crop_size": image_size, "min_scale": -0.3, "max_scale": 0.5, "do_flip": True})
            hd1k = HD1K({"crop_size": image_size, "min_scale": -0.5, "max_scale": 0.2, "do_flip": True})
            return 100 * clean + 100 * final + 200 * kitti + 5 * hd1k + things
        return 100 * clean + 100 * final + things
    if stage == "kitti":
        aug = {"crop_size": image_size, "min_scale": -0.2, "max_scale": 0.4, "do_flip": False}
        return KITTI(aug, split="training")
    if stage == "synthetic":
        return SyntheticFlowDataset(size=tuple(image_size), length=100000)
    raise ValueError(f"unknown stage {stage!r}")


def fetch_dataloader(args, TRAIN_DS: str = "C+T+K+S+H"):
    """DataLoader for ``args.stage``.  ``args.batch_size`` is the GLOBAL batch (as in the
    reference); under DDP each rank loads ``batch_size // world_size``."""
    train_dataset = build_train_dataset(args.stage, args.image_size, TRAIN_DS)
    world = int(getattr(args, "world_size", 1) or 1)
    rank = int(getattr(args, "rank", 0) or 0)
    per_rank = max(1, args.batch_size // world)
    sampler = None
    if world > 1:
        sampler = torch.utils.data.distributed.DistributedSampler(train_dataset, num_replicas=world, rank=rank,
                                                                  shuffle=True, drop_last=True)
    workers = int(getattr(args, "num_workers", 4))
    loader = data.DataLoader(train_dataset, batch_size=per_rank, sampler=sampler, shuffle=sampler is None,
                             pin_memory=torch.cuda.is_available(), num_workers=workers, drop_last=True,
                             persistent_workers=workers > 0)
    if rank == 0:
        print("Training with %d image pairs" % len(train_dataset))
    return loader
