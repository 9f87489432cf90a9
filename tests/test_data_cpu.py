"""Augmentation (batched, device-side), datasets (fake on-disk layouts) and the data loader."""
import os
from argparse import Namespace

import numpy as np
import pytest
import torch
from PIL import Image

from raft_ros_amd.data import augment as A
from raft_ros_amd.data import datasets as D
from raft_ros_amd.data import frame_utils as fu
from raft_ros_amd.data.synthetic import synthetic_batch, warp_backward


def _sample(h, w, seed=0, sparse=False):
    g = torch.Generator().manual_seed(seed)
    s = {"img1": (torch.rand(h, w, 3, generator=g) * 255).to(torch.uint8),
         "img2": (torch.rand(h, w, 3, generator=g) * 255).to(torch.uint8),
         "flow": torch.randn(h, w, 2, generator=g) * 3,
         "valid": (torch.rand(h, w, generator=g) > 0.5).float() if sparse else torch.ones(h, w)}
    return s


def test_reference_constants_are_pinned():
    """Probabilities / ranges of core/utils/augmentor.py:16-34,122-140."""
    assert A.DENSE["jitter"] == (0.4, 0.4, 0.4, 0.5 / 3.14) and A.SPARSE["jitter"] == (0.3, 0.3, 0.3, 0.3 / 3.14)
    assert A.DENSE["asym_prob"] == 0.2 and A.SPARSE["asym_prob"] == 0.0
    assert A.DENSE["eraser_prob"] == A.SPARSE["eraser_prob"] == 0.5
    assert A.DENSE["eraser_box"] == (50, 100)
    assert A.DENSE["spatial_prob"] == A.SPARSE["spatial_prob"] == 0.8
    assert A.DENSE["stretch_prob"] == 0.8 and A.DENSE["max_stretch"] == 0.2 and A.SPARSE["stretch_prob"] == 0.0
    assert (A.DENSE["hflip_prob"], A.DENSE["vflip_prob"]) == (0.5, 0.1) and A.SPARSE["vflip_prob"] == 0.0
    assert A.DENSE["crop_pad"] == 8 and A.SPARSE["crop_pad"] == 1 and A.SPARSE["margin"] == (20, 50)


def test_batched_augmentation_shapes_and_mixed_specs():
    specs = [A.AugSpec((64, 96), -0.1, 1.0, True, False), A.AugSpec((64, 96), -0.2, 0.4, True, True)]
    aug = A.BatchAugmentor(specs, seed=0)
    samples = [_sample(100, 150, 0), _sample(80, 120, 1, sparse=True), _sample(120, 110, 2)]
    for s, sid in zip(samples, (0, 1, 0)):
        s["spec"] = sid
    i1, i2, f, v = aug(A.collate_padded(samples))
    assert i1.shape == i2.shape == (3, 3, 64, 96) and f.shape == (3, 2, 64, 96) and v.shape == (3, 64, 96)
    assert i1.min() >= 0 and i1.max() <= 255 and torch.equal(i1, i1.round())  # uint8-valued
    assert set(v[1].unique().tolist()) <= {0.0, 1.0}


def test_statistics_of_random_choices():
    """Over many draws: resize ~80 %, h-flip ~50 %, v-flip ~10 %, eraser ~50 % (dense)."""
    torch.manual_seed(0)
    n = 400
    spec = A.AugSpec((32, 32), 0.0, 0.0, True, False)  # scale 2**0 = 1: resize is identity-sized
    aug = A.BatchAugmentor([spec], seed=3)
    s = _sample(48, 48)
    # a flow field whose sign reveals the flips: u = +1, v = +1 everywhere
    s["flow"] = torch.ones(48, 48, 2)
    s["spec"] = 0
    i1, i2, f, _ = aug(A.collate_padded([s] * n))
    hflip = (f[:, 0, 0, 0] < 0).float().mean().item()
    vflip = (f[:, 1, 0, 0] < 0).float().mean().item()
    assert abs(hflip - 0.5) < 0.08 and abs(vflip - 0.1) < 0.05


def test_hflip_and_crop_are_exact_without_resize():
    spec = A.AugSpec((10, 10), 0.0, 0.0, True, False)
    aug = A.BatchAugmentor([spec], seed=1)
    h = w = 20
    s = _sample(h, w)
    s["flow"] = torch.stack(torch.meshgrid(torch.arange(h).float(), torch.arange(w).float(), indexing="ij")[::-1], -1)
    s["spec"] = 0
    _, _, f, _ = aug(A.collate_padded([s] * 64))
    # u(x) = x resized by sx and multiplied by sx stays a unit-slope field (bilinear is exact
    # on linear data; only crops touching the clamped image border deviate), flipped or not
    du = (f[:, 0, :, 1:] - f[:, 0, :, :-1]).abs()
    assert ((du - 1).abs() < 1e-3).float().mean() > 0.9


def test_sparse_scatter_keeps_samples_on_rounded_positions():
    spec = A.AugSpec((30, 40), 1.0, 1.0, False, True)  # scale 2: every resized sample lands on even coords
    aug = A.BatchAugmentor([spec], seed=2)
    s = _sample(40, 60, sparse=True)
    s["valid"] = torch.zeros(40, 60)
    s["valid"][10:20, 10:30] = 1
    s["flow"][...] = torch.tensor([1.0, -2.0])
    s["spec"] = 0
    _, _, f, v = aug(A.collate_padded([s] * 32))
    on = v > 0
    assert on.any()
    vals = f.permute(0, 2, 3, 1)[on]
    # resized samples carry 2x flow; unresized (20 %) the original
    ok = torch.isclose(vals, torch.tensor([2.0, -4.0])).all(1) | torch.isclose(vals, torch.tensor([1.0, -2.0])).all(1)
    assert ok.all()
    assert (f.permute(0, 2, 3, 1)[~on] == 0).all()


def _numpy_sparse_resize(flow, valid, fx, fy):
    """Oracle with the semantics of core/utils/augmentor.py:161-193 (resize_sparse_flow_map):
    valid samples in row-major order, scaled and rounded, strictly-inside filter, then one
    numpy fancy-index assignment -- duplicates resolve to the LAST sample."""
    ht, wd = flow.shape[:2]
    yy, xx = np.meshgrid(np.arange(ht), np.arange(wd), indexing="ij")
    coords = np.stack([xx, yy], -1).reshape(-1, 2).astype(np.float32)
    f = flow.reshape(-1, 2).astype(np.float32)
    v = valid.reshape(-1) >= 1
    c0, f0 = coords[v] * [fx, fy], f[v] * [fx, fy]
    ht1, wd1 = int(round(ht * fy)), int(round(wd * fx))
    xn = np.round(c0[:, 0]).astype(np.int32)
    yn = np.round(c0[:, 1]).astype(np.int32)
    keep = (xn > 0) & (xn < wd1) & (yn > 0) & (yn < ht1)
    out = np.zeros([ht1, wd1, 2], dtype=np.float32)
    ov = np.zeros([ht1, wd1], dtype=np.int32)
    out[yn[keep], xn[keep]] = f0[keep]
    ov[yn[keep], xn[keep]] = 1
    return out, ov


@pytest.mark.parametrize("device", ["cpu", pytest.param("cuda", marks=pytest.mark.gpu)])
def test_sparse_downscale_duplicates_resolve_like_numpy_last_write(device):
    """Scale < 1 (HD1K min_scale -0.5): several samples round onto one target pixel; the
    batched scatter must keep the reference's last-write-wins winner -- on the
    GPU too, where a plain indexed write with duplicates has no defined winner."""
    if device == "cuda" and not torch.cuda.is_available():
        pytest.skip("no GPU")
    h, w, s = 24, 32, 0.5
    g = torch.Generator().manual_seed(7)
    flow = torch.randn(h, w, 2, generator=g) * 3
    valid = (torch.rand(h, w, generator=g) > 0.3).float()
    ref_f, ref_v = _numpy_sparse_resize(flow.numpy(), valid.numpy(), s, s)
    rh, rw = ref_f.shape[:2]
    aug = A.BatchAugmentor([A.AugSpec((rh, rw), 0.0, 0.0, False, True)], seed=0, device=device)
    one = lambda v: torch.tensor([v], device=device)  # noqa: E731
    sf, sv = aug._sparse_flow(flow.permute(2, 0, 1)[None].to(device), valid[None].to(device), one(s), one(s),
                              one(True), one(False), one(0), one(0), one(rh), one(rw), h, w)
    assert torch.equal(sv[0].cpu(), torch.from_numpy(ref_v).float())
    assert torch.allclose(sf[0].permute(1, 2, 0).cpu(), torch.from_numpy(ref_f), atol=1e-6)


def test_color_jitter_identity_and_ranges():
    img = torch.rand(2, 3, 16, 16) * 255
    img = img.round()
    mask = torch.ones(2, 1, 16, 16)
    ident = torch.tensor([[1.0, 1.0, 1.0, 0.0]] * 2)
    order = torch.tensor([[0, 1, 2, 3], [3, 2, 1, 0]])
    out = A.color_jitter(img, mask, ident, order)
    assert (out - img).abs().max() <= 1.0  # hue round trip through HSV: rounding only
    dark = A.color_jitter(img, mask, torch.tensor([[0.0, 1.0, 1.0, 0.0]] * 2), order)
    assert dark.max() == 0  # brightness 0 -> black regardless of order


def test_per_item_augmentors_numpy_api():
    a = A.FlowAugmentor(crop_size=[96, 128], min_scale=-0.1, max_scale=1.0, do_flip=True, seed=0)
    img = (np.random.rand(150, 200, 3) * 255).astype(np.uint8)
    flow = np.random.randn(150, 200, 2).astype(np.float32)
    i1, i2, f = a(img, img.copy(), flow)
    assert i1.shape == (96, 128, 3) and i1.dtype == np.uint8 and f.shape == (96, 128, 2) and f.dtype == np.float32
    sp = A.SparseFlowAugmentor(crop_size=[64, 96], seed=0)
    valid = (np.random.rand(100, 150) > 0.5).astype(np.float32)
    out = sp((np.random.rand(100, 150, 3) * 255).astype(np.uint8), img[:100, :150], flow[:100, :150], valid)
    assert out[0].shape == (64, 96, 3) and out[3].shape == (64, 96)


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
    assert len(s) == 2 and len(s.flow_list) == 2 and s.extra_info[1] == ("alley_1", 1)
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


def test_stage_mixture_proportions(tmp_path, monkeypatch):
    monkeypatch.setenv("RAFT_DATASET_ROOT", str(tmp_path))
    _fake_sintel(str(tmp_path))
    _fake_kitti(str(tmp_path))
    ds, specs = D.build_train_dataset("sintel", [32, 48])
    # 100 * clean(2) + 100 * final(2) + 200 * kitti(2) + 5 * hd1k(0) + things(0)
    assert len(ds) == 200 + 200 + 400
    sparse = [sp.sparse for sp in specs]
    assert sorted(sparse) == [False, True, True]  # dense sintel/things spec, KITTI, HD1K specs
    n_sparse = sum(specs[sid].sparse for _, sid in ds.entries)
    assert n_sparse == 400


def test_fetch_dataloader_on_disk_mixture(tmp_path, monkeypatch):
    monkeypatch.setenv("RAFT_DATASET_ROOT", str(tmp_path))
    _fake_sintel(str(tmp_path), h=96, w=128)
    _fake_kitti(str(tmp_path), h=96, w=140)
    args = Namespace(stage="sintel", image_size=[64, 96], batch_size=4, num_workers=0, device="cpu")
    loader = D.fetch_dataloader(args)
    i1, i2, flow, valid = next(iter(loader))
    assert i1.shape == (4, 3, 64, 96) and flow.shape == (4, 2, 64, 96) and valid.shape == (4, 64, 96)


def test_fetch_dataloader_synthetic():
    args = Namespace(stage="synthetic", image_size=[64, 96], batch_size=4, num_workers=0)
    loader = D.fetch_dataloader(args)
    i1, i2, flow, valid = next(iter(loader))
    assert i1.shape == (4, 3, 64, 96) and flow.shape == (4, 2, 64, 96)
