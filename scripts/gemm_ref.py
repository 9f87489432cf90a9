"""Calibration: hipBLASLt (torch.matmul) bf16 TFLOP/s on the update-block GEMM shapes."""
import torch

dev = torch.device("cuda")


def t(fn, reps=50):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


for name, M, N, K in [("zr", 22816, 256, 1920), ("q", 22816, 128, 1920), ("heads", 22816, 512, 1152),
                      ("convc2", 22816, 192, 2304), ("conv", 22816, 128, 2304), ("big", 8192, 8192, 8192),
                      ("zr_x4", 91264, 256, 1920)]:
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    us = t(lambda: a @ b)
    print(f"{name:7s} M={M} N={N} K={K}: {us:8.1f} us  {2 * M * N * K / us / 1e6:7.0f} TF", flush=True)
