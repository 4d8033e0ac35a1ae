#!/usr/bin/env python3
"""Dense GEMM anchor: torch.matmul (hipBLASLt) f16/bf16 TFLOP/s on this GPU,
random normal data, so the kernel's roofline fraction can be read against
what the vendor GEMM reaches under the same clocks/power. Prints JSON."""
import json
import torch


def run(m, n, k, dtype, iters=50):
    a = torch.randn(m, k, dtype=dtype, device="cuda")
    b = torch.randn(k, n, dtype=dtype, device="cuda")
    for _ in range(5):
        c = a @ b
    torch.cuda.synchronize()
    best = []
    for _ in range(5):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            c = a @ b
        e.record()
        torch.cuda.synchronize()
        best.append(s.elapsed_time(e) / iters * 1e3)
    us = sorted(best)[len(best) // 2]
    return {"m": m, "n": n, "k": k, "dtype": str(dtype).split(".")[-1],
            "us": round(us, 2), "tflops": round(2 * m * n * k / us / 1e6, 1)}


if __name__ == "__main__":
    out = []
    for dt in (torch.float16, torch.bfloat16):
        for s in ((4096, 4096, 4096), (4096, 4096, 2048), (8192, 8192, 8192)):
            out.append(run(*s, dt))
    print(json.dumps(out))
