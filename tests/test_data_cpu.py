"""Augmentation, datasets (fake on-disk layouts) and the data loader."""
import os
from argparse import Namespace

import numpy as np
import pytest
import torch
from PIL import Image

from raft_ros_amd.data import frame_utils as fu
from raft_ros_amd.data.augmentor import ColorJitter, FlowAugmentor, SparseFlowAugmentor, resize_linear
from raft_ros_amd.data import datasets as D
from raft_ros_amd.data.synthetic import synthetic_batch, warp_backward


def test_resize_linear_matches_half_pixel_bilinear():
    img = np.arange(4 * 6, dtype=np.float32).reshape(4, 6)
    out = resize_linear(img, 2.0, 2.0)
    assert out.shape == (8, 12)
    # half-pixel centres: dst x=1 samples src x=0.25 -> 0.25 (first row)
    assert abs(out[0, 1] - 0.25) < 1e-5 and out[0, 0] == 0.0
    assert resize_linear(np.zeros((10, 10, 3), np.uint8), 0.55, 1.26).shape == (13, 6, 3)


def test_color_jitter_statistics():
    torch.manual_seed(0)
    img = Image.fromarray((np.random.rand(32, 32, 3) * 255).astype(np.uint8))
    cj = ColorJitter(0.4, 0.4, 0.4, 0.5 / 3.14)
    outs = [np.array(cj(img)) for _ in range(8)]
    assert all(o.shape == (32, 32, 3) and o.dtype == np.uint8 for o in outs)
    assert len({o.tobytes() for o in outs}) > 1
    assert np.array_equal(np.array(ColorJitter()(img)), np.array(img))  # all-zero jitter = identity


def test_dense_augmentor_shapes():
    np.random.seed(0)
    aug = FlowAugmentor(crop_size=[96, 128], min_scale=-0.1, max_scale=1.0, do_flip=True)
    img = (np.random.rand(150, 200, 3) * 255).astype(np.uint8)
    flow = np.random.randn(150, 200, 2).astype(np.float32)
    for _ in range(5):
        a, b, f = aug(img, img.copy(), flow)
        assert a.shape == b.shape == (96, 128, 3) and f.shape == (96, 128, 2) and f.dtype == np.float32


def test_hflip_negates_u():
    aug = FlowAugmentor(crop_size=[10, 10], do_flip=True)
    aug.spatial_aug_prob = 0.0
    aug.h_flip_prob, aug.v_flip_prob = 1.0, 0.0
    img = np.zeros((12, 12, 3), np.uint8)
    flow = np.zeros((12, 12, 2), np.float32)
    flow[..., 0], flow[..., 1] = 3.0, -2.0
    _, _, f = aug.spatial_transform(img, img, flow)
    assert np.all(f[..., 0] == -3.0) and np.all(f[..., 1] == -2.0)


def test_sparse_flow_resize_scatters_valid_points():
    flow = np.zeros((10, 10, 2), np.float32)
    valid = np.zeros((10, 10), np.float32)
    flow[4, 6] = [1.0, -2.0]
    valid[4, 6] = 1
    f2, v2 = SparseFlowAugmentor.resize_sparse_flow_map(flow, valid, fx=2.0, fy=2.0)
    assert f2.shape == (20, 20, 2) and v2.sum() == 1
    assert np.allclose(f2[8, 12], [2.0, -4.0]) and v2[8, 12] == 1


def test_sparse_augmentor_shapes():
    np.random.seed(1)
    aug = SparseFlowAugmentor(crop_size=[64, 96], min_scale=-0.2, max_scale=0.4, do_flip=True)
    img = (np.random.rand(100, 150, 3) * 255).astype(np.uint8)
    flow = np.random.randn(100, 150, 2).astype(np.float32)
    valid = (np.random.rand(100, 150) > 0.5).astype(np.float32)
    a, b, f, v = aug(img, img, flow, valid)
    assert a.shape == (64, 96, 3) and f.shape == (64, 96, 2) and v.shape == (64, 96)


def test_synthetic_ground_truth_is_exact():
    i1, i2, flow, valid = synthetic_batch(2, 64, 80, max_disp=5, seed=3)
    assert i1.shape == (2, 3, 64, 80) and flow.shape == (2, 2, 64, 80) and valid.shape == (2, 64, 80)
    torch.testing.assert_close(warp_backward(i2, flow), i1, rtol=0, atol=1e-3)


def _fake_sintel(root, n=3, h=48, w=64):
    for dstype in ("clean", "final"):
        d = os.path.join(root, "Sintel", "training", dstype, "alley_1")
        os.makedirs(d, exist_ok=True)
        for i in range(n):
            Image.fromarray((np.random.rand(h, w, 3) * 255).astype(np.uint8)).save(f"{d}/frame_{i:04d}.png")
    fd = os.path.join(root, "Sintel", "training", "flow", "alley_1")
    os.makedirs(fd, exist_ok=True)
    for i in range(n - 1):
        fu.writeFlow(f"{fd}/frame_{i:04d}.flo", np.random.randn(h, w, 2).astype(np.float32))


def _fake_kitti(root, n=2, h=40, w=70):
    d = os.path.join(root, "KITTI", "training")
    os.makedirs(f"{d}/image_2", exist_ok=True)
    os.makedirs(f"{d}/flow_occ", exist_ok=True)
    for i in range(n):
        for s in ("10", "11"):
            Image.fromarray((np.random.rand(h, w, 3) * 255).astype(np.uint8)).save(f"{d}/image_2/{i:06d}_{s}.png")
        fu.writeFlowKITTI(f"{d}/flow_occ/{i:06d}_10.png", np.random.randn(h, w, 2).astype(np.float32))


def test_sintel_and_kitti_datasets(tmp_path, monkeypatch):
    monkeypatch.setenv("RAFT_DATASET_ROOT", str(tmp_path))
    _fake_sintel(str(tmp_path))
    _fake_kitti(str(tmp_path))
    s = D.MpiSintel(split="training", dstype="clean")
    assert len(s) == 2 and len(s.flow_list) == 2
    i1, i2, flow, valid = s[1]
    assert i1.shape == (3, 48, 64) and flow.shape == (2, 48, 64) and valid.shape == (48, 64)
    k = D.KITTI(split="training")
    assert len(k) == 2
    i1, _, flow, valid = k[0]
    assert flow.shape == (2, 40, 70) and valid.max() == 1
    mix = 3 * D.MpiSintel({"crop_size": [32, 48], "min_scale": -0.2, "max_scale": 0.6, "do_flip": True})
    assert len(mix) == 6
    x = mix[4]
    assert x[0].shape == (3, 32, 48)


def test_fetch_dataloader_synthetic():
    args = Namespace(stage="synthetic", image_size=[64, 96], batch_size=4, num_workers=0)
    loader = D.fetch_dataloader(args)
    i1, i2, flow, valid = next(iter(loader))
    assert i1.shape == (4, 3, 64, 96) and flow.shape == (4, 2, 64, 96)
