"""CPU: the C-ABI library loads, exports every symbol include/*.h declares,
and its host-only entry points (ABI layout, acceptance rules) behave like the
reference. No compute call is made (no GPU here)."""

import ctypes
import os
import re

import pytest

import sputnik_amd as sp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_c_symbols():
    src = open(os.path.join(ROOT, "include", "sputnik_amd.h")).read()
    return sorted(set(re.findall(r"\b(sputnik_[a-z_0-9]+)\s*\(", src)))


def test_library_exports_every_declared_symbol():
    L = sp.lib()
    names = declared_c_symbols()
    assert len(names) >= 12
    for n in names:
        assert hasattr(L, n), n


def test_cpp_api_symbols_exported():
    """The C++ overload set of the reference (dsd.h, dds.h, sdd.h, ssd.h,
    sds.h, dss.h, row_indices.h, transpose.h) with hipStream_t in place of
    cudaStream_t."""
    import subprocess
    out = subprocess.run(["nm", "-D", "--defined-only", sp.LIB_PATH],
                         capture_output=True, text=True, check=True).stdout
    want = [
        "_ZN7sputnik5block6MatmulENS0_11BlockMatrixEbNS0_6MatrixEbS2_P12ihipStream_t",
        "_ZN7sputnik5block8MatmulExENS0_11BlockMatrixEbNS0_6MatrixEbS2_P12ihipStream_t",
        "_ZN7sputnik5block6MatmulENS0_6MatrixEbNS0_11BlockMatrixEbS1_P12ihipStream_t",
        "_ZN7sputnik5block8MatmulExENS0_6MatrixEbNS0_11BlockMatrixEbS1_P12ihipStream_t",
        "_ZN7sputnik5block6MatmulENS0_6MatrixEbS1_bNS0_11BlockMatrixEP12ihipStream_t",
        "_ZN7sputnik5block10RowIndicesENS0_11BlockMatrixEPsP12ihipStream_t",
        "_ZN7sputnik5block9TransposeENS0_11BlockMatrixEP12ihipStream_t",
        # bitmask.h:10
        "_ZN7sputnik5block7BitmaskENS0_11BlockMatrixEP12ihipStream_t",
        # SSD (ssd.h:10-22) and SDS (sds.h:10-22)
        "_ZN7sputnik5block6MatmulENS0_11BlockMatrixEbNS0_6MatrixEbS1_P12ihipStream_t",
        "_ZN7sputnik5block8MatmulExENS0_11BlockMatrixEbNS0_6MatrixEbS1_P12ihipStream_t",
        "_ZN7sputnik5block6MatmulENS0_6MatrixEbNS0_11BlockMatrixEbS2_P12ihipStream_t",
        "_ZN7sputnik5block8MatmulExENS0_6MatrixEbNS0_11BlockMatrixEbS2_P12ihipStream_t",
        # DSS (dss.h:10-22)
        "_ZN7sputnik5block6MatmulENS0_11BlockMatrixEbS1_bNS0_6MatrixEP12ihipStream_t",
        "_ZN7sputnik5block8MatmulExENS0_11BlockMatrixEbS1_bNS0_6MatrixEP12ihipStream_t",
    ]
    for w in want:
        assert w in out, w


def test_abi_layout():
    L = sp.lib()
    assert L.sputnik_abi_block_matrix_size() == 88
    assert L.sputnik_abi_matrix_size() == 16
    expected = [0, 4, 8, 12, 16, 24, 32, 40, 48, 56, 64, 72, 80]
    assert [L.sputnik_abi_block_matrix_offset(i) for i in range(13)] == expected
    assert ctypes.sizeof(sp._CBlockMatrix) == 88
    assert ctypes.sizeof(sp._CMatrix) == 16
    fields = [f[0] for f in sp._CBlockMatrix._fields_]
    assert [getattr(sp._CBlockMatrix, f).offset for f in fields] == expected


class _T:
    """Stand-in for a device tensor: only data_ptr() is read by the host
    checks; nothing is dereferenced."""

    def __init__(self, addr=0x1000):
        self.addr = addr

    def data_ptr(self):
        return self.addr


def bm(rows, cols, nblocks, block=128, **kw):
    return sp.BlockMatrix(rows, cols, block, nblocks * block * block, _T(),
                          _T(), _T(), **kw)


def dm(rows, cols):
    return sp.Matrix(rows, cols, _T())


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_can_implement_dsd(ta, tb):
    m, k, n = 256, 384, 72
    a = bm(*((k, m) if ta else (m, k)), 3,
           **({"offsets_t": _T(), "indices_t": _T(), "block_offsets": _T()}
              if ta else {}))
    b = dm(*((n, k) if tb else (k, n)))
    assert sp.can_implement("dsd", a, ta, b, tb, dm(m, n))
    assert not sp.can_implement("dsd", a, ta, b, tb, dm(m, n + 8))  # shape
    assert not sp.can_implement("dsd", a, ta, dm(*((12, k) if tb else (k, 12))),
                                tb, dm(m, 12))                      # n % 8
    a64 = bm(*((k, m) if ta else (m, k)), 3, block=64)
    assert not sp.can_implement("dsd", a64, ta, b, tb, dm(m, n))


def test_can_implement_needs_transposed_metadata():
    a = bm(384, 256, 3)  # stored [K][M]
    assert not sp.can_implement("dsd", a, True, dm(384, 64), False, dm(256, 64))
    assert sp.can_implement("dsd", a, False, dm(256, 64), False, dm(384, 64))


@pytest.mark.parametrize("ta,tb", [(0, 0), (0, 1), (1, 0), (1, 1)])
def test_can_implement_dds_sdd(ta, tb):
    m, k, n = 40, 256, 384
    meta = {} if tb else {"offsets_t": _T(), "indices_t": _T(),
                          "block_offsets": _T()}
    b = bm(*((n, k) if tb else (k, n)), 2, **meta)
    a = dm(*((k, m) if ta else (m, k)))
    assert sp.can_implement("dds", a, ta, b, tb, dm(m, n))
    m = 256
    c = bm(m, n, 2, row_indices=_T())
    a = dm(*((8, m) if ta else (m, 8)))
    bb = dm(*((n, 8) if tb else (8, n)))
    assert sp.can_implement("sdd", a, ta, bb, tb, c)
    c_noidx = bm(m, n, 2)
    assert not sp.can_implement("sdd", a, ta, bb, tb, c_noidx)


def test_version():
    assert "gfx950" in sp.version()


def test_build_hash_matches_sources():
    """The library in the tree was built from the sources in the tree."""
    from sputnik_amd import srchash
    assert sp.build_hash() == srchash.source_hash()


@pytest.mark.parametrize("trans", [False, True])
def test_bitmask_bytes(trans):
    """reference bitmask.h:16-23 / bit_matrix.h:14-17: rows of ceil(cols/64)
    uint64 words, over the transposed orientation when offsets_t is set."""
    a = bm(3 * 128, 70 * 128, 5, **({"offsets_t": _T()} if trans else {}))
    rows, cols = (70, 3) if trans else (3, 70)
    words = (cols + 63) // 64
    assert sp.lib().sputnik_bitmask_bytes(ctypes.byref(a._c())) == rows * words * 8


def test_dsd4w_asm_matches_generator():
    """sputnik_amd/csrc/dsd4w_asm.inc is generated by gen_dsd4w.py (the Makefile
    regenerates it when the generator changes); the committed copy must be
    exactly the generator's output."""
    import importlib.util
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    gen = os.path.join(root, "sputnik_amd", "csrc", "gen_dsd4w.py")
    spec = importlib.util.spec_from_file_location("gen_dsd4w", gen)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    with open(os.path.join(root, "sputnik_amd", "csrc", "dsd4w_asm.inc")) as f:
        assert f.read() == mod.render()


def test_tuning_knobs_host_only():
    """The unsupported tuning knobs (sputnik_tuning_get / _set, dispatch.cpp
    kKnobs): defaults, set returns the previous value, range and name checks
    change nothing, select_dsd_kernel is the "dsd4w" knob."""
    import os as _os
    defaults = {"pairs": 1, "pair_xcd2": 3, "split": 1, "split_min_bn": 128,
                "dsd4w": 1, "grouped_sdd": 1, "grouped_min_per_cu": 4,
                "tall": 1, "tall_persistent": 1, "dds_xcd2": 3,
                "sdd4w_max_ld": 16384, "pair_fault": 0, "sdd_ksplit": 1,
                "sdd_ksplit_min_k": 6144, "sdd_order": 1, "tall4w": 1,
                "tall_flush_w": 4, "tall_odd_share": 120,
                "min_handoff": 2, "xcd_rows": 1, "sdd_krot": 0, "sdd_spread": 2, "sdd_bt_min_mib": 256, "sdd_tail_min_k": 8192}
    for name, v in defaults.items():
        if "SPUTNIK_AMD_" + name.upper() not in _os.environ:
            assert sp.tuning(name) == v, name
    prev = sp.tuning("pairs", 0)
    try:
        assert sp.tuning("pairs") == 0
        with pytest.raises(KeyError):
            sp.tuning("pairs", 7)          # out of range: unchanged
        assert sp.tuning("pairs") == 0
    finally:
        assert sp.tuning("pairs", prev) == 0
    with pytest.raises(KeyError):
        sp.tuning("no_such_knob")
    prev = sp.select_dsd_kernel(5)
    try:
        assert sp.tuning("dsd4w") == 5
    finally:
        sp.select_dsd_kernel(prev)
    L = sp.lib()
    L.sputnik_debug_pair_fault(1)
    assert sp.tuning("pair_fault") == 1
    L.sputnik_debug_pair_fault(0)
    assert sp.tuning("pair_fault") == 0
