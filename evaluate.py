#!/usr/bin/env python3
"""Evaluate RAFT -- same command line as the reference evaluate.py (:169-195).

    python evaluate.py --model=models/raft-things.pth --dataset=sintel --mixed_precision

Extra: ``--dataset synthetic`` (generated pairs with exact ground truth),
``--submission {sintel,kitti}`` (+ ``--warm_start``), ``--device``, ``--iters``.
Checkpoints load with or without the ``module.`` prefix, on any device.
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from raft_ros_amd.eval import validate as V  # noqa: E402
from raft_ros_amd.models import RAFT  # noqa: E402
from raft_ros_amd.utils import checkpoint  # noqa: E402

# reference-style module-level API
create_sintel_submission = V.create_sintel_submission
create_kitti_submission = V.create_kitti_submission
validate_chairs = V.validate_chairs
validate_sintel = V.validate_sintel
validate_kitti = V.validate_kitti
validate_synthetic = V.validate_synthetic


def main(argv=None):
    p = argparse.ArgumentParser()
    p.add_argument("--model", help="restore checkpoint")
    p.add_argument("--dataset", help="dataset for evaluation")
    p.add_argument("--small", action="store_true", help="use small model")
    p.add_argument("--mixed_precision", action="store_true", help="use mixed precision")
    p.add_argument("--alternate_corr", action="store_true", help="use efficent correlation implementation")
    p.add_argument("--amp_dtype", default="bf16", choices=["bf16", "fp16"])
    p.add_argument("--corr_fp32", action="store_true",
                   help="with --mixed_precision bf16: fp32-faithful correlation volume (the reference's precision)")
    p.add_argument("--device", default="cuda" if torch.cuda.is_available() else "cpu")
    p.add_argument("--iters", type=int, default=None)
    p.add_argument("--submission", choices=["sintel", "kitti"], default=None)
    p.add_argument("--warm_start", action="store_true")
    p.add_argument("--dataset_root", default=None)
    args = p.parse_args(argv)
    if args.dataset_root:
        os.environ["RAFT_DATASET_ROOT"] = args.dataset_root

    model = RAFT(args)
    if args.model:
        checkpoint.load_weights(model, args.model)
    model.to(args.device).eval()
    kw = {} if args.iters is None else {"iters": args.iters}

    with torch.inference_mode():
        if args.submission == "sintel":
            return create_sintel_submission(model, warm_start=args.warm_start, **kw)
        if args.submission == "kitti":
            return create_kitti_submission(model, **kw)
        if args.dataset == "chairs":
            return validate_chairs(model, **kw)
        if args.dataset == "sintel":
            return validate_sintel(model, **kw)
        if args.dataset == "kitti":
            return validate_kitti(model, **kw)
        if args.dataset == "synthetic":
            return validate_synthetic(model, **kw)
    raise SystemExit(f"unknown --dataset {args.dataset!r}")


if __name__ == "__main__":
    main()
