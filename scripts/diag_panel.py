import ctypes, json, os, sys, time, types
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.chdir(ROOT)
import torch, bench
dev = torch.device("cuda", 0)
args = types.SimpleNamespace(seed=0, k=4096, n=4096, m=4096, dtype="f16")
prob = bench.dsd_panel(args, 1, 0, dev, 0.02, m_total=131072, seed_off=5)
ca, cb, cc = prob.A._c(), prob.B._c(), prob.C._c()
stream = torch.cuda.current_stream().cuda_stream
order = sys.argv[1:] or ["build/exp/r05.so", "sputnik_amd/libsputnik.so", "build/exp/r05.so", "sputnik_amd/libsputnik.so"]
res = []
for path in order:
    L = ctypes.CDLL(os.path.abspath(path))
    fn = L.sputnik_dsd_ex
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p]
    a = (ctypes.byref(ca), 0, ctypes.byref(cb), 0, ctypes.byref(cc), 0, ctypes.c_void_p(stream))
    f = lambda: fn(*a)
    ms = bench.time_steps(f, 100, 100, 1)
    res.append((path, round(ms * 10, 2)))
print(json.dumps(res))
