"""Write-bandwidth ceiling for config 5's output: fill_ / zero_ / copy_ of a
131072 x 4096 fp16 tensor (1.07 GB), timed with events (median of 20)."""
import json
import torch


def t(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    out = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        out.append(a.elapsed_time(b) * 1e3)
    return sorted(out)[n // 2]


x = torch.empty(131072 * 4096, dtype=torch.float16, device="cuda")
y = torch.empty_like(x)
nb = x.numel() * 2
r = {}
for name, fn in (("fill", lambda: x.fill_(1.0)), ("zero", lambda: x.zero_()),
                 ("copy", lambda: y.copy_(x))):
    us = t(fn)
    r[name] = {"us": round(us, 1), "write_TBps": round(nb / us / 1e6, 2)}
print(json.dumps(r))
