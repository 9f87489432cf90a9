#!/usr/bin/env python3
"""Where does the fp32 (split-bf16) training path lose precision?  Compares the native fp32
path with the fp32 module path (MIOpen) and, as the noise floor, the module path against the
reference CPU gradients (tests/fixtures/golden_grads.npz): per-parameter relative errors and
the gradients entering the encoders (d fmap1/fmap2, d context features)."""
from __future__ import annotations

import os
import sys
from argparse import Namespace

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def run(dev, **kw):
    from golden import fixture, grad_step, model

    m = model(False, fixture(), **kw).to(dev).train()
    cap = {}

    def hook(name):
        def f(mod, inp, out):
            o = out if not isinstance(out, (tuple, list)) else out[0]
            if o.requires_grad:
                o.register_hook(lambda g: cap.__setitem__(name, g.detach().float().clone()))
        return f

    hs = [m.fnet.register_forward_hook(hook("fnet_out")), m.cnet.register_forward_hook(hook("cnet_out"))]
    loss, pred, grads = grad_step(m, dev)
    for h in hs:
        h.remove()
    return loss, pred, grads, cap


def main():
    from golden import grad_errors, grad_fixture

    dev = torch.device("cuda", 0)
    fix = grad_fixture()
    mod = dict(mixed_precision=False, fused_update=False, native_encoder=False)
    variants = {
        "module(miopen)": mod,
        "split-update+miopen-enc": dict(mixed_precision=False, native_encoder=False),
        "split-all": dict(mixed_precision=False),
    }
    res = {k: run(dev, **v) for k, v in variants.items()}
    ref_grads = res["module(miopen)"][2]
    for k, (loss, pred, grads, cap) in res.items():
        e_ref = grad_errors(grads, fix, "base")
        worst = sorted(e_ref.items(), key=lambda kv: -kv[1])
        print(f"\n== {k}: loss {loss:.7f}; vs REFERENCE: worst {worst[:4]}")
        groups = {}
        for n, e in e_ref.items():
            g = n.split(".")[0] + ("." + n.split(".")[1] if n.startswith("update_block") else "")
            groups.setdefault(g, []).append(e)
        print("   per group max:", {g: f"{max(v):.1e}" for g, v in groups.items()})
        if k != "module(miopen)":
            rel = {n: float((grads[n] - ref_grads[n]).norm() / ref_grads[n].norm().clamp_min(1e-30)) for n in grads}
            worst = sorted(rel.items(), key=lambda kv: -kv[1])[:6]
            print("   vs module path:", [(n, f"{e:.1e}") for n, e in worst])
            for c in cap:
                r = res["module(miopen)"][3].get(c)
                if r is not None:
                    print(f"   d {c}: rel {float((cap[c] - r).norm() / r.norm()):.2e}")


if __name__ == "__main__":
    main()
