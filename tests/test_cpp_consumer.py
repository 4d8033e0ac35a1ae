"""The C++ drop-in boundary exercised by a C++ caller: examples/
cpp_consumer.cpp uses only the reference's public API (`sputnik/sputnik.h`:
BlockMatrix / Matrix, Matmul, MatmulEx, Transpose, RowIndices, the
Allocate* helpers, hipError_t codes) and links libsputnik.so, as MegaBlocks'
extension would. Built by `make -C sputnik_amd` (build()); the GPU test runs
it and the CPU test checks that it resolves the library's C++ symbols."""

import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "build", "bin", "cpp_consumer")


def test_consumer_links_against_the_cpp_api():
    assert os.path.exists(BIN), "build it: make -C sputnik_amd"
    out = subprocess.run(["ldd", BIN], capture_output=True, text=True,
                         check=True).stdout
    line = [l for l in out.splitlines() if "libsputnik.so" in l]
    assert line and "not found" not in line[0], out
    syms = subprocess.run(["nm", "-D", "--undefined-only", BIN],
                          capture_output=True, text=True, check=True).stdout
    for s in ("_ZN7sputnik5block6MatmulENS0_11BlockMatrixEbNS0_6MatrixEbS2_P12ihipStream_t",
              "_ZN7sputnik5block8MatmulExENS0_11BlockMatrixEbNS0_6MatrixEbS2_P12ihipStream_t",
              "_ZN7sputnik5block6MatmulENS0_6MatrixEbS1_bNS0_11BlockMatrixEP12ihipStream_t",
              "_ZN7sputnik5block9TransposeENS0_11BlockMatrixEP12ihipStream_t",
              "_ZN7sputnik5block10RowIndicesENS0_11BlockMatrixEPsP12ihipStream_t"):
        assert s in syms, s


@pytest.mark.gpu
def test_cpp_consumer_runs():
    assert os.path.exists(BIN), "build it: make -C sputnik_amd"
    r = subprocess.run([BIN], capture_output=True, text=True, timeout=120)
    print(r.stdout, r.stderr)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout
