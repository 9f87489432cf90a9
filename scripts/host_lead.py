#!/usr/bin/env python3
"""Is the bench training step host-bound anywhere?  Without a profiler (whose per-dispatch
host overhead inflates idle gaps): after the host has issued step i, query whether the GPU has
already finished step i-1 (an event recorded at its end).  If it has, the GPU sat idle
waiting for the host at the step boundary; if not, the host runs more than a step ahead.
Also: host issue time per step vs GPU time per step (events), and the same per phase
(forward / loss / backward / clip / optimizer) measured from one boundary event to the next.

    python scripts/host_lead.py [--steps 20]
"""
from __future__ import annotations

import argparse
import os
import sys
import time
from argparse import Namespace

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--hp", action="store_true", help="issue on a high-priority stream (bench RAFT_HP_MAIN)")
    ap.add_argument("--gpu_pad_ms", type=float, default=0.0,
                    help="a spin kernel of this length after each step (the host gets that much further ahead)")
    ap.add_argument("--host_pad_ms", type=float, default=0.0, help="host sleep before each step")
    ap.add_argument("--max_lead", type=int, default=0,
                    help="> 0: before issuing step i, wait for step i - max_lead - 1 to finish on the GPU")
    ap.add_argument("--wgrad_timing", action="store_true",
                    help="per step: when the batched weight gradients start / end on the tail stream, relative "
                         "to the step's backward start and to the main stream reaching the weight token")
    ap.add_argument("--torch_opt", action="store_true",
                    help="torch clip_grad_norm_ + fused AdamW instead of the native clip + AdamW op")
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--image_size", type=int, nargs=2, default=[368, 496])
    ap.add_argument("--cprofile", type=int, default=0,
                    help="> 0: also profile the host side of this many steps (cProfile, top functions)")
    args = ap.parse_args()
    from raft_ros_amd.data.synthetic import synthetic_batch
    from raft_ros_amd.models import RAFT
    from raft_ros_amd.train.loss import sequence_loss
    from raft_ros_amd.train.optim import fetch_optimizer

    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    model = RAFT(Namespace(small=False, mixed_precision=True, amp_dtype="bf16", dropout=0.0)).to(dev)
    model = model.to(memory_format=torch.channels_last).train()
    opt, sched = fetch_optimizer(Namespace(lr=4e-4, wdecay=1e-4, epsilon=1e-8, num_steps=100000), model,
                                 clip=None if args.torch_opt else 1.0)
    native_opt = not isinstance(opt, torch.optim.AdamW)
    print("optimizer:", type(opt).__name__)
    pool = [synthetic_batch(args.batch, *args.image_size, seed=i, device=dev) for i in range(4)]
    stream = torch.cuda.Stream(device=dev, priority=-1) if args.hp else torch.cuda.current_stream(dev)
    phases = ["forward", "loss", "backward", "clip", "optimizer"]

    cycles = 0
    if args.gpu_pad_ms > 0:  # calibrate the spin kernel
        s_, e_ = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s_.record()
        torch.cuda._sleep(1000000)
        e_.record()
        torch.cuda.synchronize()
        cycles = int(1000000 * args.gpu_pad_ms / s_.elapsed_time(e_))

    def step(i, ev):
        i1, i2, flow, valid = pool[i % len(pool)]
        if args.host_pad_ms > 0:
            time.sleep(args.host_pad_ms / 1e3)
        ev[6].record()
        opt.zero_grad(set_to_none=True)
        th = [time.perf_counter()]
        ev[0].record()
        preds = model(i1, i2, iters=12)
        th.append(time.perf_counter())
        ev[1].record()
        loss, _ = sequence_loss(preds, flow, valid, gamma=0.8)
        th.append(time.perf_counter())
        ev[2].record()
        loss.backward()
        th.append(time.perf_counter())
        ev[3].record()
        if not native_opt:  # (the native op clips inside its step)
            torch.nn.utils.clip_grad_norm_(model.parameters(), 1.0)
        th.append(time.perf_counter())
        ev[4].record()
        opt.step()
        sched.step()
        th.append(time.perf_counter())
        ev[5].record()
        if cycles:
            torch.cuda._sleep(cycles)
        return th

    if args.wgrad_timing:
        from raft_ros_amd.ops import update_fused

        update_fused.WGRAD_TIMING = []
    with torch.cuda.stream(stream):
        for i in range(5):
            step(i, [torch.cuda.Event(enable_timing=True) for _ in range(8)])
        torch.cuda.synchronize()
        m0 = torch.cuda.memory_stats(dev)
        evs = [[torch.cuda.Event(enable_timing=True) for _ in range(8)] for _ in range(args.steps)]
        ths, done_prev = [], []
        t0 = time.perf_counter()
        for i in range(args.steps):
            if args.max_lead > 0 and i - args.max_lead - 1 >= 0:
                evs[i - args.max_lead - 1][5].synchronize()
            ths.append(step(5 + i, evs[i]))
            evs[i][7].record()  # after step() returned: its autograd graph / locals are freed
            if i > 0:
                done_prev.append(evs[i - 1][5].query())
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / args.steps
        m1 = torch.cuda.memory_stats(dev)
        if args.cprofile > 0:
            import cProfile
            import pstats

            # the backward's Python (autograd Functions) runs on the engine's device thread,
            # which cProfile does not see: run it on this thread for the profiled steps
            torch.autograd.set_multithreading_enabled(False)
            pr = cProfile.Profile()
            pr.enable()
            for i in range(args.cprofile):
                step(i, [torch.cuda.Event(enable_timing=True) for _ in range(8)])
            pr.disable()
            torch.cuda.synchronize()
            st = pstats.Stats(pr)
            st.sort_stats("tottime").print_stats(45)
            st.sort_stats("cumulative").print_stats(45)
    if args.wgrad_timing:
        from raft_ros_amd.ops import update_fused

        tl = update_fused.WGRAD_TIMING[-args.steps:]
        rows = []
        for i, (e_tok, e0, e1) in enumerate(tl):
            # relative to the step's backward start (evs[i][2]: after the loss) and its end (evs[i][3])
            b0 = evs[i][2]
            rows.append((b0.elapsed_time(e0), b0.elapsed_time(e1), b0.elapsed_time(e_tok), b0.elapsed_time(evs[i][3])))
        n = len(rows)
        m = [sum(r[k] for r in rows) / n for k in range(4)]
        print(f"weight gradients (ms after the backward start): start {m[0]:.2f}, end {m[1]:.2f}; main stream "
              f"at the weight token {m[2]:.2f}; backward end (main) {m[3]:.2f}")
    keys = ("num_device_alloc", "num_device_free", "num_alloc_retries", "num_sync_all_streams", "num_ooms")
    print("caching allocator over the timed steps:", {k: m1.get(k, 0) - m0.get(k, 0) for k in keys},
          f"reserved {m0['reserved_bytes.all.current'] / 2**30:.2f} -> {m1['reserved_bytes.all.current'] / 2**30:.2f} GiB")
    gpu = [evs[i][0].elapsed_time(evs[i][5]) for i in range(args.steps)]
    host = [1e3 * (t[-1] - t[0]) for t in ths]
    n = args.steps
    print(f"wall {1e3 * wall:.2f} ms/step; GPU (first to last event of a step) {sum(gpu) / n:.2f} ms; host issue "
          f"{sum(host) / n:.2f} ms; GPU already done with step i-1 when the host finished issuing step i: "
          f"{sum(done_prev)}/{len(done_prev)}")
    # per phase: host issue time vs GPU time between the phase's boundary events
    for k, name in enumerate(phases):
        h = sum(1e3 * (t[k + 1] - t[k]) for t in ths) / n
        g = sum(evs[i][k].elapsed_time(evs[i][k + 1]) for i in range(n)) / n
        print(f"  {name:9s} host {h:6.2f} ms   GPU {g:6.2f} ms")
    # GPU idle between steps: end event of step i -> start event of step i+1
    gaps = [evs[i][5].elapsed_time(evs[i + 1][0]) for i in range(n - 1)]
    print(f"  step-boundary GPU gap (end of step i -> start of i+1): mean {sum(gaps) / len(gaps):.3f} ms, "
          f"max {max(gaps):.3f} ms")
    a = [evs[i][5].elapsed_time(evs[i][7]) for i in range(n - 1)]
    b = [evs[i][7].elapsed_time(evs[i + 1][6]) for i in range(n - 1)]
    c = [evs[i + 1][6].elapsed_time(evs[i + 1][0]) for i in range(n - 1)]
    print(f"    of which: step() return (graph freed) {sum(a) / len(a):.3f} ms, loop {sum(b) / len(b):.3f} ms, "
          f"zero_grad {sum(c) / len(c):.3f} ms")


if __name__ == "__main__":
    main()
