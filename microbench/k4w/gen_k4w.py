"""Generates the hand-scheduled k-loop of the 4-wave DSD kernel (experiment).

One workgroup of 4 waves (one per SIMD) owns a 128 x 512 output tile; wave w
owns columns [128 w, 128 w + 128) as 8 x 8 accumulators of
v_mfma_f32_16x16x32_{f16,bf16} held in a[0:255]. Per 32-deep k-step a wave
issues 64 MFMAs and, in their gaps, the 24 LDS fragment reads of the next
step (16 ds_read_b64_tr_b16 for its D columns, 8 ds_read_b128 for the S
rows) and the 10 LDS-DMA instructions of the step three ahead (2 for its
share of the shared S image, 8 for its private D image).

Register map (all fixed, declared as clobbers):
  a[0:255]   accumulators, acc(m, n) = a[4 (8 m + n) : +3]
  v[128:159] S fragments, set 0    v[160:191] D fragments, set 0
  v[192:223] S fragments, set 1    v[224:255] D fragments, set 1
  s[40:43] S-block descriptor, s[44:47] D descriptor, s48..s79 loop state.
LDS: S slots 4 x 8 KiB at [0, 32K); wave w's D slots 4 x 8 KiB at
32K + 32K w. Staging for the epilogue: 128 rows x 1040 B.

Usage: python gen_k4w.py OUT.inc [dtype f16|bf16]
"""
import sys

FS = (128, 192)
FD = (160, 224)
SLOT = 8192


def mfma(dt, m, n, s):
    a = 4 * (8 * m + n)
    return (f"v_mfma_f32_16x16x32_{dt} a[{a}:{a + 3}], v[{FD[s] + 4 * n}:{FD[s] + 4 * n + 3}], "
            f"v[{FS[s] + 4 * m}:{FS[s] + 4 * m + 3}], a[{a}:{a + 3}]")


def d_reads(slot, s):
    out = []
    for n in range(8):
        b = FD[s] + 4 * n
        out.append(f"ds_read_b64_tr_b16 v[{b}:{b + 1}], %[vrd{n}] offset:{slot * SLOT}")
        out.append(f"ds_read_b64_tr_b16 v[{b + 2}:{b + 3}], %[vrd{n}] offset:{slot * SLOT + 1024}")
    return out


def s_reads(slot, s):
    out = []
    for m in range(8):
        b = FS[s] + 4 * m
        out.append(f"ds_read_b128 v[{b}:{b + 3}], %[vrs] offset:{slot * SLOT + m * 1024}")
    return out


def dmas(slot, opt=None):
    """(m0 setup, load) pairs of one step's 10 DMAs into ring slot `slot`."""
    opt = opt or {}
    sd = "s[80:83]" if opt.get("s_fixed") else "s[40:43]"
    dd = "s[84:87]" if opt.get("d_fixed") else "s[44:47]"
    out = []
    for q in range(2):
        if opt.get("s_linear"):
            out.append((f"s_add_u32 m0, s62, {slot * SLOT + q * 1024}",
                        f"buffer_load_dwordx4 %[vsl], {sd}, {'0' if q == 0 else 's73'} offen lds"))
            continue
        out.append((f"s_add_u32 m0, s62, {slot * SLOT + q * 1024}",
                    f"buffer_load_dwordx4 %[vs], {sd}, {'0' if q == 0 else 's72'} offen lds"))
    for q in range(8):
        out.append((f"s_add_u32 m0, s63, {slot * SLOT + q * 1024}",
                    f"buffer_load_dwordx4 %[vd{(q >> 1) & 1}], {dd}, s{64 + q} offen lds"))
    return out


ADVANCE = ["s_add_u32 s40, s40, 64", "s_addc_u32 s41, s41, 0",
           "s_add_u32 s44, s44, s53", "s_addc_u32 s45, s45, 0"]

# Next block's descriptors (S entry s57 + 1 clamped to s74; D k-block s58),
# then s58 <- the k-block loaded by the index prefetch (s59 >> s60).
SWITCH = ["s_add_u32 s57, s57, 1", "s_min_u32 s57, s57, s74",
          "s_lshl_b32 s76, s57, 15", "s_lshr_b32 s77, s57, 17",
          "s_add_u32 s40, s48, s76", "s_addc_u32 s41, s49, s77",
          "s_mul_i32 s76, s58, s52", "s_mul_hi_u32 s77, s58, s52",
          "s_add_u32 s44, s50, s76", "s_addc_u32 s45, s51, s77",
          "s_lshr_b32 s58, s59, s60", "s_and_b32 s58, s58, 0xffff"]

# Scalar load of the k-block of entry min(s56, s74) into s59 (shift in s60).
IDX_LOAD = ["s_min_u32 s78, s56, s74", "s_add_u32 s56, s56, 1",
            "s_lshl_b32 s79, s78, 1", "s_and_b32 s60, s79, 2",
            "s_lshl_b32 s60, s60, 3", "s_and_b32 s79, s79, 0xfffffffc",
            "s_add_u32 s76, s54, s79", "s_addc_u32 s77, s55, 0",
            "s_load_dword s59, s[76:77], 0x0"]

DMA_POS = [3, 9, 15, 21, 27, 33, 39, 45, 51, 57]

# Experiment variants (ablations / placements); 0 is the kernel.
VARIANTS = {
    0: {},
    1: {"no_dma": True},
    2: {"no_reads": True},
    3: {"no_dma": True, "no_reads": True, "no_barrier": True},
    4: {"dma_pos": list(range(30, 50, 2))},
    5: {"barrier_at": 40, "s_reads_at": 41},
    6: {"dma_pos": [3, 7, 11, 15, 19, 23, 27, 31, 35, 39]},
    7: {"no_barrier": True},
    8: {"no_d_reads": True},
    9: {"no_s_reads": True},
    10: {"no_s_dma": True},
    11: {"no_d_dma": True},
    12: {"no_vmcnt": True},
    13: {"no_lgkm": True},
    14: {"s_fixed": True},
    15: {"dma_pos": [1, 2, 9, 15, 21, 27, 33, 39, 45, 51]},
    16: {"dma_pos": [45, 51, 3, 9, 15, 21, 27, 33, 39, 57]},
    17: {"s_fixed": True, "d_fixed": True},
    18: {"s_linear": True},
    19: {"s_linear": True, "s_fixed": True},
}


def step(dt, H, opt):
    """Loop step H of a block: MFMAs on set H%2, reads of step i+1 from slot
    (H+1)%4 into the other set, DMA of step i+3 into slot (H+3)%4."""
    cur = H % 2
    nxt = 1 - cur
    gaps = [[] for _ in range(64)]
    if H == 0:
        gaps[0] += IDX_LOAD
    if not opt.get("no_vmcnt"):
        gaps[1].append("s_waitcnt vmcnt(10)")
    if H == 1:
        gaps[1] += SWITCH
    if not opt.get("no_reads") and not opt.get("no_d_reads"):
        dr = d_reads((H + 1) % 4, nxt)
        for i, ins in enumerate(dr):
            gaps[2 + i].append(ins)
    if not opt.get("no_barrier"):
        gaps[opt.get("barrier_at", 18)].append("s_barrier")
    if not opt.get("no_reads") and not opt.get("no_s_reads"):
        sr = s_reads((H + 1) % 4, nxt)
        for i, ins in enumerate(sr):
            gaps[opt.get("s_reads_at", 19) + i].append(ins)
    for j, ((m0, ld), k) in enumerate(zip(dmas((H + 3) % 4, opt), opt.get("dma_pos", DMA_POS))):
        gaps[k - 1].append(m0)
        skip = (opt.get("no_dma") or (opt.get("no_s_dma") and j < 2)
                or (opt.get("no_d_dma") and j >= 2))
        if not skip:
            gaps[k].append(ld)
    gaps[58] += ADVANCE if H != 0 else []
    gaps[63].append("s_waitcnt lgkmcnt(0)" if not opt.get("no_lgkm") else "s_nop 0")
    out = []
    idx = 0
    for m in range(8):
        for n in range(8):
            out.append(mfma(dt, m, n, cur))
            out += gaps[idx]
            idx += 1
    return out


def prologue():
    out = [
        # descriptor constants, loop state
        "s_mov_b32 s42, 0x7fffffff", "s_mov_b32 s43, 0x00020000",
        "s_mov_b32 s46, 0x7fffffff", "s_mov_b32 s47, 0x00020000",
        "s_mov_b32 s48, %[sdlo]", "s_mov_b32 s49, %[sdhi]",
        "s_mov_b32 s50, %[dtlo]", "s_mov_b32 s51, %[dthi]",
        "s_mov_b32 s52, %[k128]", "s_mov_b32 s53, %[k32]",
        "s_mov_b32 s54, %[ixlo]", "s_mov_b32 s55, %[ixhi]",
        "s_add_u32 s56, %[e0], 2", "s_mov_b32 s57, %[e0]",
        "s_mov_b32 s58, %[kb1]", "s_mov_b32 s61, %[nblk]",
        "s_mov_b32 s62, %[ms]", "s_mov_b32 s63, %[md]",
        "s_mov_b32 s72, 4096", "s_mov_b32 s74, %[elast]", "s_mov_b32 s73, 1024",
        "s_mov_b32 s64, 0",
    ]
    for q in range(1, 8):
        out.append(f"s_mul_i32 s{64 + q}, %[k4], {q}")
    # block 0 descriptors
    out += ["s_lshl_b32 s76, s57, 15", "s_lshr_b32 s77, s57, 17",
            "s_add_u32 s40, s48, s76", "s_addc_u32 s41, s49, s77",
            "s_mul_i32 s76, %[kb0], s52", "s_mul_hi_u32 s77, %[kb0], s52",
            "s_add_u32 s44, s50, s76", "s_addc_u32 s45, s51, s77",
            "s_mov_b64 s[80:81], s[40:41]", "s_mov_b64 s[82:83], s[42:43]",
            "s_mov_b64 s[84:85], s[44:45]", "s_mov_b64 s[86:87], s[46:47]"]
    for slot in range(3):
        for m0, ld in dmas(slot):
            out += [m0, "s_nop 0", ld]
        out += ADVANCE
    for i in range(256):
        out.append(f"v_accvgpr_write_b32 a{i}, 0")
    out += ["s_waitcnt vmcnt(20)", "s_barrier"]
    out += d_reads(0, 0) + s_reads(0, 0)
    out.append("s_waitcnt lgkmcnt(0)")
    return out


def epilogue():
    out = ["s_waitcnt vmcnt(0)", "s_barrier", "s_nop 7", "s_nop 7", "s_nop 7"]
    t = 0
    for m in range(8):
        for n in range(8):
            a = 4 * (8 * m + n)
            v = 128 + 8 * (t % 8)
            t += 1
            out += [f"v_accvgpr_read_b32 v{v + i}, a{a + i}" for i in range(4)]
            out += [f"v_cvt_pk_f16_f32 v{v + 4}, v{v}, v{v + 1}",
                    f"v_cvt_pk_f16_f32 v{v + 5}, v{v + 2}, v{v + 3}"]
            base = "%[vw0]" if m < 4 else "%[vw1]"
            off = (16 * (m % 4)) * 1040 + 32 * n
            out.append(f"ds_write_b64 {base}, v[{v + 4}:{v + 5}] offset:{off}")
    out.append("s_waitcnt lgkmcnt(0)")
    return out


def build(dt, opt):
    body = prologue()
    body += ["s_memtime %[t0]", "s_memrealtime %[r0]", "s_waitcnt lgkmcnt(0)"]
    body.append("L_loop_%=:")
    for H in range(4):
        body += step(dt, H, opt)
    body += ["s_sub_u32 s61, s61, 1", "s_cmp_lg_u32 s61, 0",
             "s_cbranch_scc1 L_loop_%="]
    body += ["s_memtime %[t1]", "s_memrealtime %[r1]", "s_waitcnt lgkmcnt(0)"]
    body += epilogue()
    return body


def main():
    out = sys.argv[1]
    with open(out, "w") as f:
        f.write("// generated by gen_k4w.py -- do not edit\n")
        for v, opt in VARIANTS.items():
            for dt in ("f16", "bf16"):
                if dt == "bf16" and v != 0:
                    continue
                body = build(dt, opt)
                if dt == "bf16":
                    body = [b.replace("v_cvt_pk_f16_f32", "v_cvt_pk_bf16_f32")
                            for b in body]
                f.write(f"#define K4W_ASM_{dt.upper()}_V{v} \\\n")
                for ins in body:
                    f.write(f'  "{ins}\\n" \\\n')
                f.write("  \"\"\n\n")
        f.write(f"#define K4W_NVARIANTS {len(VARIANTS)}\n")
        clob = ([f'"a{i}"' for i in range(256)] + [f'"v{i}"' for i in range(128, 256)]
                + [f'"s{i}"' for i in range(40, 88)] + ['"scc"', '"memory"'])
        f.write("#define K4W_CLOBBERS " + ", ".join(clob) + "\n")


if __name__ == "__main__":
    main()
