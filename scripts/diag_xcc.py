"""blockIdx -> physical XCD (XCC_ID) of a 256-workgroup launch on torch's
current stream, in a fresh process with or without a non-blocking stream
created after the operands (the process-history effect of DESIGN 0e):
`python diag_xcc.py none|stream_after|stream_before`."""
import ctypes, json, os, sys, types
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.chdir(ROOT)
import torch, bench
mode = sys.argv[1]
dev = torch.device("cuda", 0)
hip = ctypes.CDLL("libamdhip64.so")
if mode == "stream_before":
    s = ctypes.c_void_p(); assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
args = types.SimpleNamespace(seed=0, k=4096, n=4096, m=4096, dtype="f16")
prob = bench.dsd_panel(args, 1, 0, dev, 0.5, m_total=4096)
if mode == "stream_after":
    s = ctypes.c_void_p(); assert hip.hipStreamCreateWithFlags(ctypes.byref(s), 1) == 0
L = ctypes.CDLL(os.path.join(ROOT, "microbench", "xcc", "libxcc_map.so"))
out = torch.zeros(256, dtype=torch.int32, device=dev)
stream = torch.cuda.current_stream().cuda_stream
maps = []
fn = prob.launcher()
for i in range(4):
    assert L.xcc_map(ctypes.c_void_p(out.data_ptr()), 256, ctypes.c_void_p(stream)) == 0
    torch.cuda.synchronize()
    x = out.cpu().tolist()
    rot = sorted(set((x[b] - b) % 8 for b in range(256)))
    maps.append({"first16": x[:16], "rotations": rot})
    fn()  # a headline launch between probes
    torch.cuda.synchronize()
print(json.dumps({"mode": mode, "maps": maps}))
