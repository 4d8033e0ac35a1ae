#!/usr/bin/env python3
"""Config-5 bound probe: DSD M=131072 K=N=4096 at several densities vs a
plain fill of the same output bytes (write-bandwidth ceiling)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def timeit(fn, iters=50):
    import torch
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    s = torch.cuda.Event(enable_timing=True)
    e = torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    import torch
    import bench
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    m = 131072
    out = torch.empty(m * 4096, dtype=torch.float16, device=dev)
    print("fill_ 1 GiB fp16: %.1f us" % timeit(lambda: out.fill_(0)))
    print("zero_ 1 GiB fp16: %.1f us" % timeit(lambda: out.zero_()))
    for d in (0.0001, 0.02, 0.1):
        prob = bench.Problem(m, 4096, 4096, d, "f16", 0, dev)
        fn = prob.launcher()
        t = timeit(fn)
        print("dsd density %.4f nb %d: %.1f us  %.2f TB/s algorithmic" %
              (d, prob.nb, t, prob.bytes / t / 1e6))
        del prob


if __name__ == "__main__":
    main()
