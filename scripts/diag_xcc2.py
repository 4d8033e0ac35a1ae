"""Does the blockIdx -> XCD rotation advance with the grid size of the
launches in between? Probes (256 workgroups) interleaved with odd-sized
grids on the same stream, and on a second stream."""
import ctypes, json, os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
import torch
dev = torch.device("cuda", 0)
L = ctypes.CDLL(os.path.join(ROOT, "microbench", "xcc", "libxcc_map.so"))
out = torch.zeros(256, dtype=torch.int32, device=dev)
junk = torch.zeros(256, dtype=torch.int32, device=dev)
def probe(stream):
    assert L.xcc_map(ctypes.c_void_p(out.data_ptr()), 256, ctypes.c_void_p(stream)) == 0
    torch.cuda.synchronize()
    x = out.cpu().tolist()
    return sorted(set((x[b] - b) % 8 for b in range(256)))
s0 = torch.cuda.current_stream().cuda_stream
res = {"start": probe(s0)}
for g in (1, 3, 5, 7, 8, 13):
    assert L.xcc_map(ctypes.c_void_p(junk.data_ptr()), g, ctypes.c_void_p(s0)) == 0
    res[f"after_grid_{g}"] = probe(s0)
s1 = torch.cuda.Stream()
res["other_stream"] = probe(s1.cuda_stream)
res["back"] = probe(s0)
print(json.dumps(res))
