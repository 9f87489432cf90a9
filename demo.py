#!/usr/bin/env python3
"""RAFT demo -- same command line as the reference demo.py (:66-75).

    python demo.py --model=models/raft-things.pth --path=demo-frames

Without ``--path`` the frames are read from ``demo-frames/``; when that directory holds no
frames a synthetic sequence (textured background drift + a moving disc,
``data/synthetic.demo_sequence``) is written there first.

Runs every consecutive pair of *.png / *.jpg frames in ``--path`` (sorted) with
20 refinement iterations.  The reference shows [image; flow] in a cv2 window;
here the visualisation is shown with cv2 when it is importable and a display is
available, and is always written to ``--output`` (default ``demo-output/``) as
PNG.  ``--model`` is optional (random weights) so the pipeline can be smoke-
tested without the pretrained files.
"""
from __future__ import annotations

import argparse
import glob
import os
import sys

import numpy as np
import torch
from PIL import Image

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from raft_ros_amd.models import RAFT  # noqa: E402
from raft_ros_amd.utils import checkpoint, flow_viz  # noqa: E402
from raft_ros_amd.utils.utils import InputPadder  # noqa: E402

DEVICE = "cuda" if torch.cuda.is_available() else "cpu"


def load_image(imfile, device=DEVICE):
    img = np.array(Image.open(imfile).convert("RGB")).astype(np.uint8)
    img = torch.from_numpy(img).permute(2, 0, 1).float()
    return img[None].to(device)


def viz(img, flo, out_path=None, show=False):
    img = img[0].permute(1, 2, 0).cpu().numpy()
    flo = flo[0].permute(1, 2, 0).cpu().numpy()
    flo = flow_viz.flow_to_image(flo)
    img_flo = np.concatenate([img, flo], axis=0).astype(np.uint8)
    if out_path:
        Image.fromarray(img_flo).save(out_path)
    if show:
        try:
            import cv2

            cv2.imshow("image", img_flo[:, :, [2, 1, 0]] / 255.0)
            cv2.waitKey()
        except Exception:
            pass
    return img_flo


def write_demo_frames(path, n_frames: int = 6):
    """No frames at ``path``: write a synthetic sequence there (the reference's Sintel demo
    frames are not redistributed with this repository)."""
    from raft_ros_amd.data.synthetic import demo_sequence

    os.makedirs(path, exist_ok=True)
    out = []
    for k, fr in enumerate(demo_sequence(n_frames)):
        f = os.path.join(path, "frame_%04d.png" % (16 + k))
        Image.fromarray(fr.permute(1, 2, 0).numpy()).save(f)
        out.append(f)
    print(f"demo: no frames in {path}; wrote {len(out)} synthetic frames there")
    return out


def demo(args):
    rank = 0
    if getattr(args, "query_shard", False):
        # torchrun --nproc-per-node N demo.py --query_shard: every rank runs the same frames,
        # each holding the correlation-volume rows of 1/N of the query pixels; rank 0 writes
        from raft_ros_amd.parallel import ddp

        info = ddp.init_distributed()
        rank = info.rank
        if info.device.type == "cuda":
            args.device = str(info.device)
    model = RAFT(args)
    if args.model:
        checkpoint.load_weights(model, args.model)
    model.to(args.device).eval()
    os.makedirs(args.output, exist_ok=True)
    images = sorted(glob.glob(os.path.join(args.path, "*.png")) + glob.glob(os.path.join(args.path, "*.jpg")))
    if not images:
        images = write_demo_frames(args.path)
    outs = []
    with torch.inference_mode():
        for k, (imfile1, imfile2) in enumerate(zip(images[:-1], images[1:])):
            image1 = load_image(imfile1, args.device)
            image2 = load_image(imfile2, args.device)
            padder = InputPadder(image1.shape)
            image1, image2 = padder.pad(image1, image2)
            flow_low, flow_up = model(image1, image2, iters=args.iters, test_mode=True)
            out = os.path.join(args.output, "flow_%04d.png" % k)
            if rank == 0:
                viz(image1, flow_up, out, show=args.show)
            outs.append(out)
    return outs


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model", help="restore checkpoint")
    p.add_argument("--path", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "demo-frames"),
                   help="directory of frames (default: demo-frames/, synthesised on first use)")
    p.add_argument("--small", action="store_true", help="use small model")
    p.add_argument("--mixed_precision", action="store_true", help="use mixed precision")
    p.add_argument("--alternate_corr", action="store_true", help="use efficent correlation implementation")
    p.add_argument("--amp_dtype", default="bf16", choices=["bf16", "fp16"])
    p.add_argument("--corr_fp32", action="store_true",
                   help="with --mixed_precision bf16: fp32-faithful correlation volume (the reference's precision)")
    p.add_argument("--device", default=DEVICE)
    p.add_argument("--iters", type=int, default=20)
    p.add_argument("--output", default="demo-output")
    p.add_argument("--show", action="store_true", help="also display with cv2 (if available)")
    p.add_argument("--query_shard", action="store_true",
                   help="under torchrun: shard the correlation volume over the ranks' query pixels "
                        "(high-resolution inference; raft_ros_amd/parallel/query_shard.py)")
    args = p.parse_args(argv)
    return demo(args)


if __name__ == "__main__":
    main()
