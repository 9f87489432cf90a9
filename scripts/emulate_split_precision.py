#!/usr/bin/env python3
"""Which 16-bit-mantissa storage points of the split-bf16 fp32 training path cost gradient
precision?  CPU emulation on the reference gradient fixture (tests/fixtures/golden_grads.npz):
the fp32 module path with every conv wrapped so that chosen tensors are rounded to the split
representation hi + lo (two bf16 planes: a 16-bit mantissa, relative error <= 2^-17):

  op   the GEMM operands: the conv input and weight (x_hi W_hi + x_lo W_hi + x_hi W_lo);
       opx / opw: the input / the weight alone
  out  the conv output as stored (pre-norm activation)
  dy   the loss gradient at the conv output (the dgrad / wgrad GEMM operand)
  dx   the data gradient as stored (the dgrad output)

    python scripts/emulate_split_precision.py [--small] [--variants op,op+dy,...]
    python scripts/emulate_split_precision.py --write   # tests/fixtures/split_format_floor.json

``--write`` records, for base and small with every conv emulated in the storage layout the
native path uses (op+out+dy+dx), the worst and RMS per-parameter relative gradient error vs
the reference: the precision floor of the number format itself, which the GPU tests hold the
native kernels to (tests/test_golden_gpu.py, tests/test_split_train_gpu.py).
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch
import torch.nn as nn
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def r16(x: torch.Tensor) -> torch.Tensor:
    hi = x.to(torch.bfloat16).float()
    return hi + (x - hi).to(torch.bfloat16).float()


class _RoundFwd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return r16(x)

    @staticmethod
    def backward(ctx, g):
        return g


class _RoundBwd(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        return x.clone()

    @staticmethod
    def backward(ctx, g):
        return r16(g)


def patched_forward(flags):
    orig = nn.Conv2d._conv_forward

    def fwd(self, x, w, b):
        if not getattr(self, "_emu", False):
            return orig(self, x, w, b)
        if "dx" in flags:
            x = _RoundBwd.apply(x)
        if "op" in flags or "opx" in flags:
            x = _RoundFwd.apply(x)
        if "op" in flags or "opw" in flags:
            w = _RoundFwd.apply(w)
        y = orig(self, x, w, b)
        if "out" in flags:
            y = _RoundFwd.apply(y)
        if "dy" in flags:
            y = _RoundBwd.apply(y)
        return y

    return orig, fwd


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--small", action="store_true")
    ap.add_argument("--variants", default="none,op,op+dy,op+out+dy,op+dy+dx,op+out+dy+dx")
    ap.add_argument("--scope", default="fnet,cnet", help="module prefixes whose convs are emulated")
    ap.add_argument("--write", action="store_true")
    args = ap.parse_args()
    if args.write:
        floor = {}
        for small in (False, True):
            floor["small" if small else "base"] = run(small, ["op+out+dy+dx"], ("",))[0]
        path = os.path.join(ROOT, "tests", "fixtures", "split_format_floor.json")
        with open(path, "w") as f:
            json.dump(floor, f, indent=1)
        print("wrote", path, floor)
        return
    run(args.small, args.variants.split(","), tuple(args.scope.split(",")))


def run(small, variants, scope):
    from golden import fixture, grad_errors, grad_fixture, grad_step, model

    fix, gfix = fixture(), grad_fixture()
    name = "small" if small else "base"
    res = []
    for var in variants:
        flags = set() if var == "none" else set(var.split("+"))
        m = model(small, fix, mixed_precision=False, fused_update=False, native_encoder=False).train()
        for n, mod in m.named_modules():
            if isinstance(mod, nn.Conv2d) and n.startswith(scope):
                mod._emu = True
        orig, fwd = patched_forward(flags)
        nn.Conv2d._conv_forward = fwd
        try:
            loss, _, grads = grad_step(m, torch.device("cpu"))
        finally:
            nn.Conv2d._conv_forward = orig
        e_all = grad_errors(grads, gfix, name)
        rms_all = (sum(v * v for v in e_all.values()) / len(e_all)) ** 0.5
        e = {k: v for k, v in e_all.items() if k.startswith(scope)}
        worst = sorted(e.items(), key=lambda kv: -kv[1])[:3]
        rms = (sum(v * v for v in e.values()) / len(e)) ** 0.5
        print(f"{name} {var:14s} loss {loss:.6f}  RMS {rms:.2e} (all params {rms_all:.2e})  worst " +
              ", ".join(f"{k} {v:.2e}" for k, v in worst), flush=True)
        res.append({"variant": var, "worst": worst[0][1], "worst_param": worst[0][0], "rms": rms})
    return res


if __name__ == "__main__":
    main()
