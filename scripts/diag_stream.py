"""Does a process-wide non-blocking HIP stream change the speed of
null-stream launches? One workload per process: `python diag_stream.py
WORKLOAD none|stream|stream_after` (WORKLOAD: panel, moe, sdd_dds, headline)."""
import ctypes, json, os, sys, types
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.chdir(ROOT)
import torch, bench
wl, mode = sys.argv[1], sys.argv[2]
dev = torch.device("cuda", 0)
hip = ctypes.CDLL("libamdhip64.so")
if mode == "stream":  # a non-blocking stream before the operands
    s = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
args = types.SimpleNamespace(seed=0, k=4096, n=4096, m=4096, dtype="f16")
if wl == "panel":
    prob = bench.dsd_panel(args, 1, 0, dev, 0.02, m_total=131072, seed_off=5)
elif wl == "moe":
    prob = bench.MoeProblem("bf16", 0, dev)
elif wl == "sdd_dds":
    prob = bench.PairProblem(4096, 0.2, "f16", 0, dev)
else:
    prob = bench.dsd_panel(args, 1, 0, dev, 0.5, m_total=4096)
if mode == "stream_after":  # ... after the operands, before the first launch
    s = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
fn = prob.launcher()
steps = 20 if wl == "moe" else 100
out = [round(bench.time_steps(fn, steps, steps, 1) * 1000 / steps, 2) for _ in range(3)]
print(json.dumps({"workload": wl, "mode": mode, "us": out}))
