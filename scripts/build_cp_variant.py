#!/usr/bin/env python3
"""Experiment library: libsputnik with cache-policy bits on the 4-wave
kernel's LDS-DMA loads (buffer_load ... lds). Renders gen_dsd4w.py, appends
the bits to every such load of the chosen macros, compiles dsd4w.hip against
that body and links it with the tree's other objects (build/sputnik_amd).
Usage: build_cp_variant.py NAME "BITS" [MACRO_SUBSTR]   -> build/exp/NAME.so
BITS = STORE:<bits> instead: the output stores' nt becomes <bits> (empty:
plain). BITS = PLAINPUB: the pair / K-split partial publishes lose their sc1
bit (the lines stay in the XCD's L2; same-XCD pairs only -- an experiment)."""
import importlib.util
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "sputnik_amd", "csrc")


def main():
    name, bits = sys.argv[1], sys.argv[2]
    only = sys.argv[3] if len(sys.argv) > 3 else ""
    spec = importlib.util.spec_from_file_location("gen", os.path.join(CSRC, "gen_dsd4w.py"))
    gen = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(gen)
    out, cur, n = [], "", 0
    for line in gen.render().split("\n"):
        if line.startswith("#define "):
            cur = line.split()[1]
        if bits.startswith("STORE:"):  # output stores: "offen nt" -> "offen <rest>"
            if "buffer_store_dwordx4" in line and " offen nt\\n" in line and only in cur:
                line = line.replace(" offen nt\\n", (" offen " + bits[6:]).rstrip() + "\\n")
                n += 1
        elif bits == "PLAINPUB":  # partial publishes without sc1 (kept in L2)
            if ("buffer_store_dwordx4 a[" in line and " sc1\\n" in line and only in cur
                    and "_KS" not in cur):  # (K-split chunks sit on other XCDs)
                line = line.replace(" sc1\\n", "\\n")
                n += 1
        elif ("buffer_load" in line and line.endswith(' lds\\n" \\') and only in cur):
            line = line.replace(" lds\\n", " " + bits + " lds\\n")
            n += 1
        out.append(line)
    d = os.path.join(ROOT, "build", "exp", name)
    os.makedirs(d, exist_ok=True)
    for f in os.listdir(CSRC):
        if f.endswith((".h", ".hip")):
            with open(os.path.join(CSRC, f)) as src, open(os.path.join(d, f), "w") as dst:
                dst.write(src.read())
    with open(os.path.join(d, "dsd4w_asm.inc"), "w") as f:
        f.write("\n".join(out))
    hipcc = "/opt/rocm/bin/hipcc"
    obj = os.path.join(d, "dsd4w.o")
    subprocess.run([hipcc, "-std=c++17", "-O3", "-fPIC", "--offload-arch=gfx950",
                    "-I" + os.path.join(ROOT, "include"), "-Wno-unused-function",
                    "-c", os.path.join(d, "dsd4w.hip"), "-o", obj], check=True)
    b = os.path.join(ROOT, "build", "sputnik_amd")
    objs = [os.path.join(b, f + ".o") for f in ("block_gemm", "metadata", "layout", "dispatch", "c_api")]
    subprocess.run([hipcc, "--offload-arch=gfx950", "-shared", "-fPIC", "-o",
                    os.path.join(ROOT, "build", "exp", name + ".so"), obj] + objs, check=True)
    print(name, "loads modified:", n)


if __name__ == "__main__":
    main()
