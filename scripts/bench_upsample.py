"""Convex 8x upsampling microbenchmark (forward, backward) at the training (config #2: 8 x 46 x 62)
and 1080p inference (1 x 135 x 240) shapes, channels-last bf16 / fp32 masks as the mask head
writes them: kernel time and effective HBM bandwidth (mask + flow_up bytes; backward adds dmask
and the upsampled gradient)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from raft_ros_amd.ops._ext import ops


def timeit(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000 / reps


def main():
    k = ops()
    for (B, H, W) in [(8, 46, 62), (1, 135, 240)]:
        for dt in (torch.bfloat16, torch.float32):
            for fmt in (torch.channels_last, torch.contiguous_format):
                flow = torch.randn(B, 2, H, W, device="cuda")
                mask = torch.randn(B, 576, H, W, device="cuda", dtype=dt).contiguous(memory_format=fmt)
                g = torch.randn(B, 2, 8 * H, 8 * W, device="cuda")
                mb = mask.numel() * mask.element_size()
                ob = g.numel() * 4
                tf = timeit(lambda: k.convex_upsample(flow, mask))
                tb = timeit(lambda: k.convex_upsample_backward(flow, mask, g))
                print(f"B={B} {H}x{W} {str(dt)[6:]:8s} {'cl  ' if fmt == torch.channels_last else 'nchw'} "
                      f"fwd {tf:6.1f}us ({(mb + ob) / tf / 1e3:5.0f} GB/s)  "
                      f"bwd {tb:6.1f}us ({(2 * mb + ob) / tb / 1e3:5.0f} GB/s)", flush=True)


if __name__ == "__main__":
    main()
