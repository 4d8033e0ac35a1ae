"""Config-5 launch speed in a fresh process after different one-time
actions (diagnosis of a 198 vs 217 us first-use difference)."""
import ctypes, json, os, sys, types
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.chdir(ROOT)
import torch, bench
mode = sys.argv[1]
dev = torch.device("cuda", 0)
args = types.SimpleNamespace(seed=0, k=4096, n=4096, m=4096, dtype="f16")
prob = bench.dsd_panel(args, 1, 0, dev, 0.02, m_total=131072, seed_off=5)
ca, cb, cc = prob.A._c(), prob.B._c(), prob.C._c()
hip = ctypes.CDLL("libamdhip64.so")
if mode == "stream":
    s = ctypes.c_void_p()
    assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
elif mode == "torchstream":
    s = torch.cuda.Stream()
elif mode == "malloc":
    ptr = ctypes.c_void_p()
    assert hip.hipMalloc(ctypes.byref(ptr), ctypes.c_size_t(16)) == 0
stream = torch.cuda.current_stream().cuda_stream
L = ctypes.CDLL(os.path.abspath("sputnik_amd/libsputnik.so"))
fn = L.sputnik_dsd_ex
fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
a = (ctypes.byref(ca), 0, ctypes.byref(cb), 0, ctypes.byref(cc), 0, ctypes.c_void_p(stream))
out = []
for _ in range(3):
    out.append(round(bench.time_steps(lambda: fn(*a), 100, 100, 1) * 10, 2))
print(json.dumps({"mode": mode, "us": out}))
