"""HBM write / copy bandwidth probe: how fast can a kernel write a buffer the size of the 1080p
dense correlation volume (32400 x 43035 bf16 = 2.79 GB)?  torch fill_ (write only) and copy_
(read + write) against the corr_volume_bf16 kernel's ~1.18 ms build (profiles/)."""
import torch


def timeit(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def main():
    for n in (32400 * 43035, 22816 * 8 * 3790 // 8):
        x = torch.empty(n, dtype=torch.bfloat16, device="cuda")
        y = torch.empty_like(x)
        gb = n * 2 / 1e9
        tf = timeit(lambda: x.fill_(1.0))
        tc = timeit(lambda: y.copy_(x))
        print(f"{gb:6.2f} GB bf16: fill {tf:7.3f} ms ({gb / tf:5.2f} TB/s write)   "
              f"copy {tc:7.3f} ms ({2 * gb / tc:5.2f} TB/s read+write)", flush=True)
        del x, y


if __name__ == "__main__":
    main()
