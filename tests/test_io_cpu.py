"""File formats: .flo, .pfm, KITTI 16-bit PNG, the PNG codec, read_gen, the chairs split."""
import numpy as np
import pytest
from PIL import Image

from raft_ros_amd.data import frame_utils as fu
from raft_ros_amd.data.datasets import chairs_split
from raft_ros_amd.data.png16 import read_png, write_png


def test_flo_roundtrip(tmp_path):
    flow = np.random.randn(13, 17, 2).astype(np.float32)
    fu.writeFlow(str(tmp_path / "a.flo"), flow)
    assert np.array_equal(fu.readFlow(str(tmp_path / "a.flo")), flow)
    fu.writeFlow(str(tmp_path / "b.flo"), flow[..., 0], flow[..., 1])
    assert np.array_equal(fu.read_gen(str(tmp_path / "b.flo")), flow)
    raw = (tmp_path / "a.flo").read_bytes()
    assert np.frombuffer(raw[:4], np.float32)[0] == 202021.25
    assert np.frombuffer(raw[4:12], np.int32).tolist() == [17, 13]


def test_flo_bad_magic(tmp_path):
    (tmp_path / "x.flo").write_bytes(b"\0" * 32)
    with pytest.raises(ValueError):
        fu.readFlow(str(tmp_path / "x.flo"))


def test_pfm_roundtrip_and_read_gen_drops_third_channel(tmp_path):
    img = np.random.randn(9, 11, 3).astype(np.float32)
    fu.writePFM(str(tmp_path / "a.pfm"), img)
    assert np.array_equal(fu.readPFM(str(tmp_path / "a.pfm")), img)
    assert np.array_equal(fu.read_gen(str(tmp_path / "a.pfm")), img[..., :2])
    gray = np.random.randn(5, 6).astype(np.float32)
    fu.writePFM(str(tmp_path / "g.pfm"), gray)
    assert np.array_equal(fu.read_gen(str(tmp_path / "g.pfm")), gray)


def test_kitti_flow_roundtrip(tmp_path):
    flow = (np.random.rand(20, 30, 2).astype(np.float32) - 0.5) * 200
    fu.writeFlowKITTI(str(tmp_path / "k.png"), flow)
    back, valid = fu.readFlowKITTI(str(tmp_path / "k.png"))
    assert valid.shape == (20, 30) and np.all(valid == 1)
    assert np.abs(back - flow).max() <= 1 / 64 + 1e-6  # 1/64 px quantisation (truncation)
    raw = read_png(str(tmp_path / "k.png"))
    assert raw.dtype == np.uint16 and raw.shape == (20, 30, 3)


def test_kitti_disparity(tmp_path):
    d = np.zeros((4, 5), np.uint16)
    d[1, 2] = 256 * 7
    write_png(str(tmp_path / "d.png"), d)
    flow, valid = fu.readDispKITTI(str(tmp_path / "d.png"))
    assert flow[1, 2, 0] == -7 and valid.sum() == 1


@pytest.mark.parametrize("dtype,ch", [(np.uint16, 3), (np.uint8, 3), (np.uint16, 1), (np.uint8, 4), (np.uint8, 1)])
def test_png_codec_roundtrip(tmp_path, dtype, ch):
    hi = 65535 if dtype == np.uint16 else 255
    a = (np.random.rand(23, 31, ch) * hi).astype(dtype)
    a = a[..., 0] if ch == 1 else a
    write_png(str(tmp_path / "a.png"), a)
    assert np.array_equal(read_png(str(tmp_path / "a.png")), a)


def test_png_reads_pil_filtered_files(tmp_path):
    a = (np.random.rand(40, 64, 3) * 255).astype(np.uint8)
    a[:, :20] = 9
    a[10:20] = np.arange(64, dtype=np.uint8)[None, :, None]
    Image.fromarray(a).save(tmp_path / "p.png", optimize=True)
    assert np.array_equal(read_png(str(tmp_path / "p.png")), a)
    g = (np.random.rand(17, 19) * 65535).astype(np.uint16)
    Image.fromarray(g).save(tmp_path / "g.png")
    assert np.array_equal(read_png(str(tmp_path / "g.png")), g)


def test_read_gen_images(tmp_path):
    a = (np.random.rand(8, 9, 3) * 255).astype(np.uint8)
    Image.fromarray(a).save(tmp_path / "a.ppm")
    assert np.array_equal(np.array(fu.read_gen(str(tmp_path / "a.ppm"))), a)
    assert fu.read_gen(str(tmp_path / "x.unknown")) == []


def test_chairs_split():
    s = chairs_split()
    assert len(s) == 22872 and (s == 1).sum() == 22232 and (s == 2).sum() == 640


@pytest.mark.reference
def test_chairs_split_matches_reference_file(reference_core):
    ref = np.loadtxt("/root/reference/chairs_split.txt", dtype=np.int32)
    assert np.array_equal(chairs_split(), ref)
