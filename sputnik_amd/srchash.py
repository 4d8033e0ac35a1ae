"""Hash of the sources libsputnik.so is built from.

The Makefile compiles it into the library (sputnik_build_hash()); bench.py
and smoke() recompute it over the tree they run in, so a stale binary is
reported instead of silently measured. Usage: python -m sputnik_amd.srchash
"""

import hashlib
import os
import sys

_HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(_HERE)


def source_files(root=ROOT):
    out = []
    csrc = os.path.join(root, "sputnik_amd", "csrc")
    for name in sorted(os.listdir(csrc)):
        if name.endswith((".h", ".hip", ".cpp", ".inc", ".py")):
            out.append(os.path.join("sputnik_amd", "csrc", name))
    out.append(os.path.join("sputnik_amd", "Makefile"))
    inc = os.path.join(root, "include")
    for d, _, files in sorted(os.walk(inc)):
        for name in sorted(files):
            if name.endswith(".h"):
                out.append(os.path.relpath(os.path.join(d, name), root))
    return sorted(out)


def source_hash(root=ROOT) -> str:
    h = hashlib.sha256()
    for rel in source_files(root):
        h.update(rel.replace(os.sep, "/").encode())
        h.update(b"\0")
        with open(os.path.join(root, rel), "rb") as f:
            h.update(f.read())
        h.update(b"\0")
    return h.hexdigest()[:16]


if __name__ == "__main__":
    sys.stdout.write(source_hash(sys.argv[1] if len(sys.argv) > 1 else ROOT))
