"""Generates dsd4w_asm.inc: the hand-scheduled body of the 4-wave DSD kernel
(dsd4w.hip). Run by the Makefile; the output is committed too, and
tests/test_abi.py checks that it matches this generator.

Why a generator: the k-loop interleaves, per 32-deep k-step and wave, 64
v_mfma_f32_16x16x32_{f16,bf16} with 24 LDS fragment reads and 10 LDS-DMA
instructions on fixed registers. hipcc cannot be made to keep that schedule
(at 8 waves x 256 VGPRs every change of the step structure spilled, DESIGN
§3.1), so the whole body -- prologue, k-loop, pair publish, pair collect and
the accumulator -> fp16/bf16 staging -- is ONE inline-asm statement with
literal registers, and the HIP code around it only computes operands and
copies the staged tile out.

Tile: one workgroup = 4 waves (one per SIMD) owns a 128 x 512 output tile of
DSD C = A . B (A's 128-row block-row times a 512-column panel of B); wave w
owns columns [128 w, 128 w + 128) as 8 x 8 accumulators of 16 x 16 (fp32, in
a[0:255]). The MFMA computes the tile transposed (B fragment as the A
operand), so a lane's 4 accumulator values are 4 consecutive columns of one
output row -- the layout of the 8-wave kernel (block_gemm.h mfma_step), so the
two kernels' products are bit-identical on unpaired rows.

Per k-step (32 deep), each wave:
  * 64 MFMAs on fragment set (step % 2);
  * in their gaps: 16 ds_read_b64_tr_b16 (its 8 D fragments of step + 1,
    from its private D image) and 8 ds_read_b128 (the 8 S fragments, from
    the S image all four waves share) into the other set;
  * 10 LDS-DMA (buffer_load_dwordx4 ... lds) of step + 3: 8 KiB of its own D
    image and 2 KiB of the shared S image;
  * one s_barrier (the S image of step + 1 is written by all waves).
LDS (160 KiB): S ring 4 x 8 KiB at [0, 32K); wave w's D ring 4 x 8 KiB at
32K + 32K w. Images and swizzles are block_gemm.h's (kc_key / tr_key):
S [128 rows][32 k] with 16-byte chunk c ^ ((row >> 1) & 3), D [32 k][128 cols]
with 32-byte sector s ^ tr_key(k), both applied on the DMA source address.

Register map (literal, declared as clobbers):
  a[0:255]                accumulators, acc(m, n) = a[4 (8 m + n) : +3]
  v[128:159] / v[160:191] S / D fragments, set 0
  v[192:223] / v[224:255] S / D fragments, set 1
  v[96:127]               epilogue / poll temporaries
  s[40:43] S-block buffer descriptor, s[44:47] D descriptor,
  s[84:87] pair-partial descriptor, s56..s79, s94..s99 loop state.
Everything read-only comes in as an operand (%[name]); %[flags] packs the
workgroup's role bits: 0 collect (pair consumer), 1 specialized last block
allowed, 2 test fault (producer skips its flag), 3 last wave (raises the
flag), 4 wave 0 (counts a time-out), 5 split-mode first chunk (no tile of
its own: ends after publishing).

Sparse-row segments (pair balancing, dispatch.cpp PreparePairs): a virtual
entry x in [0, ntot) is the CSR entry x + (x < n1 ? b1 : b2m) (b2m = b2 - n1).
A pair producer runs the heavy row's head [0, n1) and publishes its fp32
partial when `remaining blocks == flushrem` (= n2), then its own row; a
consumer (collect != 0) adds the published partial in the epilogue.

Usage: python gen_dsd4w.py OUT.inc
"""
import sys

FS = (128, 192)
FD = (160, 224)
SLOT = 8192
DMA_POS = [3, 9, 15, 21, 27, 33, 39, 45, 51, 57]
READS_AT = 2    # own image's reads from here, then the barrier, then the shared image's
NAN_F16 = "0x7e007e00"
NAN_BF16 = "0x7fc07fc0"
WAIT_TICKS = 20000000   # s_memrealtime (100 MHz): 0.2 s (block_gemm.h kPairWaitTicks)


def mfma(dt, m, n, s, zero_c=False):
    a = 4 * (8 * m + n)
    c = "0" if zero_c else f"a[{a}:{a + 3}]"
    return (f"v_mfma_f32_16x16x32_{dt} a[{a}:{a + 3}], "
            f"v[{FD[s] + 4 * n}:{FD[s] + 4 * n + 3}], "
            f"v[{FS[s] + 4 * m}:{FS[s] + 4 * m + 3}], {c}")


def d_reads(slot, s, into=None):
    """The 8 transposed fragments of a [32 k][128] image in ring slot
    `slot` (by default into the A-operand set; SDD TT: the B-operand set)."""
    out = []
    for n in range(8):
        b = (into or FD)[s] + 4 * n
        out.append(f"ds_read_b64_tr_b16 v[{b}:{b + 1}], %[vrd{n}] offset:{slot * SLOT}")
        out.append(f"ds_read_b64_tr_b16 v[{b + 2}:{b + 3}], %[vrd{n}] "
                   f"offset:{slot * SLOT + 1024}")
    return out


def t_reads(slot, s):
    """DSD TN: the 8 row-tile fragments, transposed, from the shared [32 k]
    [128 m] slice into the B-operand set."""
    out = []
    for m in range(8):
        b = FS[s] + 4 * m
        out.append(f"ds_read_b64_tr_b16 v[{b}:{b + 1}], %[vrt{m}] offset:{slot * SLOT}")
        out.append(f"ds_read_b64_tr_b16 v[{b + 2}:{b + 3}], %[vrt{m}] "
                   f"offset:{slot * SLOT + 1024}")
    return out


def s_reads(slot, s):
    return [f"ds_read_b128 v[{FS[s] + 4 * m}:{FS[s] + 4 * m + 3}], %[vrs] "
            f"offset:{slot * SLOT + m * 1024}" for m in range(8)]


def dmas(slot):
    """(m0 setup, load) pairs of one step's 10 LDS-DMAs into ring slot `slot`:
    2 x 1 KiB of the shared S image (16 rows each), 8 x 1 KiB of the wave's D
    image (4 k-rows each)."""
    out = []
    for q in range(2):
        out.append((f"s_add_u32 m0, %[ms], {slot * SLOT + q * 1024}",
                    f"buffer_load_dwordx4 %[vs], s[40:43], {'0' if q == 0 else 's72'} "
                    f"offen lds"))
    for q in range(8):
        out.append((f"s_add_u32 m0, %[md], {slot * SLOT + q * 1024}",
                    f"buffer_load_dwordx4 %[vd{(q >> 1) & 1}], s[44:47], s{64 + q} "
                    f"offen lds"))
    return out


# The fed block advances one k-step: S by 64 B (32 k of a 256-B row), D by
# 32 rows.
# DDS (`VARIANT["dds"]`, see build): the shared image is the sparse block's
# [32 k][128 n] slice (8 KiB contiguous: S advances 32 rows of 256 B) and
# the wave's image [128 m][32 k] of the dense rows (D advances 64 B).
VARIANT = {"dds": False, "ds": False, "sdd": False, "nt": False, "tt": False,
           "bar2": False, "tn": False, "ddstt": False, "il": False, "ks": False,
           "tp": False}
# "ks": SDD K-split (ksplit_path): the epilogue of a chunk of a group's K.
# "tp": tall DSD NN, persistent (tall_flush): a workgroup's blocks come from
# per-lane tables (%[vent]: lane x = CSR entry | panel << 24 of virtual block
# x, %[vent2] of block 64 + x; %[vtile] / %[vtile2]: row | panel << 16 |
# last-of-tile << 31) and every tile is stored as soon as its last block is
# done.
# "il": the plain per-wave epilogue stores each 16-row batch as soon as it is
# staged (on with "bar2"; alone: _W4).
# DDS TT ("ddstt", with "ds"): B's rows (storage order) are the shared image
# in double slots as in DSD; A stored [k][m] gives each wave a per-step [32 k]
# [128 m] slice as DSD's B, read transposed into the B operand (%[vrt<m>]),
# and the shared rows go to the A operand with ds_read_b128 (%[vrk*]).
# DSD TN ("tn", per-step images): A^T in column order (A's transposed
# metadata), so the shared image is the sparse block's [32 k][128 m] slice as
# in DDS, read transposed into the B-operand set (%[vrt<m>]); B's [32 k][128
# n] slice per wave as in DSD NN.
# "bar2" (double-slot mode with a double-slot SHARED image: DSD, SDD NN / NT):
# one s_barrier every other step. The shared double slot of steps (S0, S0 +
# 1) is first read in step S0 - 1 (odd), after that step's barrier (every
# wave's DMA of it waited before); its second half is read in step S0 from
# the same, already synchronized slot; it is refilled after the barrier of
# step S0 + 1 (odd), which no wave passes before every wave has finished
# step S0. The wave's own images need no barrier.
# SDD TT ("tt", with "sdd" and "ds"): A stored [k][m], so the shared image is
# the per-step [32 k][128 m] slice of A (rows lda apart: %[s16] = 4 lda
# between its two DMAs, S advances %[sk32] = 32 lda per step and %[sk128] per
# k-block), read transposed into the MFMA's B-operand set; B stored [n][k]:
# the wave's image in double slots as in NT. The DDS ring structure with the
# operand sets exchanged.
# SDD NT / DSD NT ("nt", with "ds"; SDD also "sdd"): B stored [n][k], so the
# wave's image is k-contiguous too: both images in double slots, both read with ds_read_b128
# (the wave's B rows into the MFMA's A-operand set, %[vrk0] / %[vrk1] =
# half-0 / half-1 addresses), and every DMA is a double-slot one, on odd
# steps.
# SDD (grouped, NN): the shared image is the row panel of A, so entry x (=
# k-block x: no index list) starts 256 B into its rows, not at a stored
# block; the 16-row soffset is 16 lda (%[s16]).


def col_order():
    """DDS / DSD TN in column order (the sparse operand's transposed
    metadata: storage block per entry through s_block_offsets); DDS NT reads
    B's rows in storage order like DSD."""
    if VARIANT["ddstt"]:
        return False
    return ((VARIANT["dds"] and not VARIANT["nt"])
            or ((VARIANT["tn"] or VARIANT["tt"]) and not VARIANT["sdd"]))


def a_rows_t():
    """SDD TT / TN: the shared image is A's [32 k][128 m] slice (rows lda
    apart): S advances %[sk32] per step and %[sk128] per k-block."""
    return (VARIANT["tt"] or VARIANT["tn"]) and VARIANT["sdd"]


def s_block_shift():
    """(high, low) shifts of S's byte offset from the entry in s76."""
    return (24, 8) if VARIANT["sdd"] else (17, 15)


def advance():
    s = ("%[sk32]" if a_rows_t() else
         8192 if VARIANT["dds"] or VARIANT["tn"] else 64)
    return [f"s_add_u32 s40, s40, {s}", "s_addc_u32 s41, s41, 0",
            "s_add_u32 s44, s44, %[k32]", "s_addc_u32 s45, s45, 0"]


def entry_of(xreg, out_reg):
    """out_reg = absolute CSR entry of virtual entry xreg (scc clobbered).
    (tp: lane xreg of %[vent]; the lane select written by SALU just before
    needs 4 wait states.)"""
    if VARIANT["tp"]:  # (128 entries: lanes of %[vent] then of %[vent2])
        tmp = "s77" if out_reg == "s76" else "s76"
        return ["s_nop 3", f"v_readlane_b32 {out_reg}, %[vent], {xreg}",
                f"v_readlane_b32 {tmp}, %[vent2], {xreg}", f"s_cmp_lt_u32 {xreg}, 64",
                f"s_cselect_b32 {out_reg}, {out_reg}, {tmp}",
                f"s_and_b32 {out_reg}, {out_reg}, 0xffffff"]
    return [f"s_cmp_lt_u32 {xreg}, %[n1]",
            f"s_cselect_b32 {out_reg}, %[b1], %[b2m]",
            f"s_add_u32 {out_reg}, {out_reg}, {xreg}"]


# Switch the fed block to the next virtual entry (s57 + 1, clamped to the
# last): S block = its entry (storage order), D rows = 128 x its k-block
# (s58, loaded a block ahead); then s58 <- the k-block the index prefetch
# brought in (s59 >> s60).
# (DDS: the S block is the storage block of the entry, s_block_offsets[e],
# kept in s63 and prefetched into s62 like the k-block.)
def switch():
    if col_order():
        blk = ["s_lshr_b32 s77, s63, 17", "s_lshl_b32 s76, s63, 15"]
    elif a_rows_t():
        blk = (["s_add_u32 s57, s57, 1", "s_min_u32 s57, s57, %[xlast]"]
               + entry_of("s57", "s78")
               + ["s_mul_hi_u32 s77, s78, %[sk128]", "s_mul_i32 s76, s78, %[sk128]"])
    else:
        hi, lo = s_block_shift()
        blk = (["s_add_u32 s57, s57, 1", "s_min_u32 s57, s57, %[xlast]"]
               + entry_of("s57", "s76")
               + [f"s_lshr_b32 s77, s76, {hi}", f"s_lshl_b32 s76, s76, {lo}"])
    out = blk + ["s_add_u32 s40, %[sdlo], s76", "s_addc_u32 s41, %[sdhi], s77",
                 "s_mul_i32 s76, s58, %[k128]", "s_mul_hi_u32 s77, s58, %[k128]",
                 "s_add_u32 s44, %[dtlo], s76", "s_addc_u32 s45, %[dthi], s77"]
    if VARIANT["tp"]:  # + the block's panel: 512 columns = 1 KiB
        out += ["v_readlane_b32 s79, %[vent], s57", "v_readlane_b32 s78, %[vent2], s57",
                "s_cmp_lt_u32 s57, 64", "s_cselect_b32 s79, s79, s78",
                "s_lshr_b32 s79, s79, 24",
                "s_lshl_b32 s79, s79, 10", "s_add_u32 s44, s44, s79",
                "s_addc_u32 s45, s45, 0"]
    out += ["s_lshr_b32 s58, s59, s60", "s_and_b32 s58, s58, 0xffff"]
    if col_order():
        out.append("s_mov_b32 s63, s62")
    return out

# Scalar load of the k-block (int16) of virtual entry min(s56, xlast) into
# s59 (its half in s60), one block ahead of the SWITCH that uses it.
def idx_load():
    if VARIANT["sdd"]:  # k-block of virtual entry x is its entry (x, or
        # x rotated: dsd4w.hip sdd_krot)
        return (["s_min_u32 s78, s56, %[xlast]", "s_add_u32 s56, s56, 1"]
                + entry_of("s78", "s59") + ["s_mov_b32 s60, 0"])
    out = ["s_min_u32 s78, s56, %[xlast]", "s_add_u32 s56, s56, 1"] + entry_of("s78", "s79")
    if col_order():
        out += ["s_lshl_b32 s74, s79, 2", "s_add_u32 s74, %[bolo], s74",
                "s_addc_u32 s75, %[bohi], 0", "s_load_dword s62, s[74:75], 0x0"]
    # the entry's byte address, then its aligned dword and the half within
    # it (the list may start 2 bytes into a dword: a scalar load drops the
    # low address bits, block_gemm.h scalar_load_short)
    return out + ["s_lshl_b32 s79, s79, 1",
                  "s_add_u32 s76, %[ixlo], s79", "s_addc_u32 s77, %[ixhi], 0",
                  "s_and_b32 s60, s76, 2", "s_lshl_b32 s60, s60, 3",
                  "s_and_b32 s76, s76, 0xfffffffc",
                  "s_load_dword s59, s[76:77], 0x0"]


def step(dt, H, zero_c=False, last=0, cvt=None):
    if VARIANT["ds"]:
        assert not last
        return step_ds(dt, H, zero_c)
    """Step H of a block: MFMAs on set H % 2; reads of step + 1 from slot
    (H + 1) % 4 into the other set; DMA of step + 3 into slot (H + 3) % 4
    (H = 0: the fed block's last step; H = 1..3: steps 0..2 of the next
    block, switched to at H = 1).
    last = H (1..3): step H of the launch's last block (per-wave epilogue
    only): no DMA (there is no next block); step 2 waits for step 3's DMA
    with vmcnt(0) (nothing younger in flight); step 3 reads nothing, meets
    no barrier, and converts + stages each accumulator two MFMAs after its
    final update (the per-wave staging region is the wave's own D ring,
    whose last reads and DMAs are done)."""
    cur, nxt = H % 2, 1 - H % 2
    gaps = [[] for _ in range(64)]
    if H == 0:
        gaps[0] += idx_load()
    if last != 3:
        # own DMA of step + 1 landed (step + 2's 10 may still fly)
        gaps[1].append("s_waitcnt vmcnt(0)" if last == 2 else "s_waitcnt vmcnt(10)")
    if H == 1 and not last:
        gaps[1] += switch()
    if last != 3:
        # the wave's own image first, then (after the barrier) the shared one:
        # DSD D (tr) / S (b128), DDS the other way round
        own, shared = d_reads((H + 1) % 4, nxt), s_reads((H + 1) % 4, nxt)
        if VARIANT["dds"]:
            own, shared = shared, own
        if VARIANT["tn"] and VARIANT["dds"]:
            # DDS TN: A^T's [32 k][128 m] slice per wave, read transposed
            # into the B operand (%[vrt<m>] on the wave's own ring); the
            # shared sparse slice into the A operand as in DDS NN
            own, shared = t_reads((H + 1) % 4, nxt), d_reads((H + 1) % 4, nxt)
        elif VARIANT["tn"]:
            shared = t_reads((H + 1) % 4, nxt)
        for i, ins in enumerate(own):
            gaps[READS_AT + i].append(ins)
        # every wave's S DMA of step + 1 landed (each waited above) / every
        # wave done reading the slot refilled below (its reads were waited at
        # the end of step - 2)
        gaps[READS_AT + len(own)].append("s_barrier")
        for i, ins in enumerate(shared):
            gaps[READS_AT + len(own) + 1 + i].append(ins)
    if not last:
        for (m0, ld), k in zip(dmas((H + 3) % 4), DMA_POS):
            gaps[k - 1].append(m0)
            gaps[k].append(ld)
        if H != 0:
            gaps[58] += advance()
    if last == 3:
        for i in range(2, 64):
            gaps[i] += convert(cvt, i - 2)
    else:
        gaps[63].append("s_waitcnt lgkmcnt(0)")
    out = []
    for i in range(64):
        out.append(mfma(dt, i // 8, i % 8, cur, zero_c))
        out += gaps[i]
    return out


# ---- double-slot mode (VARIANT["ds"]) -----------------------------------
# The k-contiguous image (DSD: the shared S image, rows of the stored block;
# DDS: each wave's rows of A) is loaded as 128-byte row pieces covering two
# k-steps at once: a 128-B piece is a whole cache line, where the 64-B piece
# of a 32-deep step is half of one and the L1 (32 KiB, refilled faster than
# the next step comes back to the line) fetches every line twice (TCP->TCC
# read requests r04l: DSD 1.3x, DDS 1.95x the algorithmic L2->L1 bytes). Its
# ring becomes two double slots [128 rows][128 B] (16 KiB, chunk c of row r
# at c ^ ((r >> 1) & 7): 16-B fragment reads stay bank-conflict free), filled
# on odd steps for the next block-half; the other image keeps its 4 x 8 KiB
# ring. LDS per wave and in total are unchanged.
DS_SLOT = 16384


def per_step_dmas(slot):
    """(m0, load) pairs of the per-step image's DMAs into ring slot `slot`:
    DSD the wave's D image (8 x 4 k-rows), DDS / SDD TT the shared S slice
    (2 x 4 k-rows of this wave's 8); SDD NT none."""
    if VARIANT["nt"]:
        return []
    if (VARIANT["dds"] or VARIANT["tt"]) and not VARIANT["ddstt"]:
        return [(f"s_add_u32 m0, %[ms], {slot * SLOT + q * 1024}",
                 f"buffer_load_dwordx4 %[vs], s[40:43], {'0' if q == 0 else 's72'} "
                 f"offen lds") for q in range(2)]
    return [(f"s_add_u32 m0, %[md], {slot * SLOT + q * 1024}",
             f"buffer_load_dwordx4 %[vd{(q >> 1) & 1}], s[44:47], s{64 + q} offen lds")
            for q in range(8)]


def own_ds_dmas(d):
    return [(f"s_add_u32 m0, %[md], {d * DS_SLOT + q * 1024}",
             f"buffer_load_dwordx4 %[vd{q & 1}], s[44:47], s{64 + (q >> 1)} offen lds")
            for q in range(16)]


def ds_dmas(d):
    """(m0, load) pairs filling double slot d with 8-row x 128-B pieces: DSD
    this wave's 32 rows of the shared S image (rows 32 w + 16 p + 8 q + l / 8:
    %[vs<q>], soffset p x 16 rows), DDS the wave's 128 rows of A (rows 16 p +
    8 q + l / 8: %[vd<q>], soffset s<64 + p> = p x 16 rows). (SDD NT: the
    shared one here, the wave's own in own_ds_dmas.)"""
    if (col_order() or VARIANT["tt"]) and not VARIANT["ddstt"]:
        return own_ds_dmas(d)
    return [(f"s_add_u32 m0, %[ms], {d * DS_SLOT + (2 * p + q) * 1024}",
             f"buffer_load_dwordx4 {'%[vs]' if q == 0 else '%[vs1]'}, s[40:43], "
             f"{'0' if p == 0 else 's72'} offen lds")
            for p in range(2) for q in range(2)]


def s_reads_ds(d, half, s):
    """The 8 row-tile fragments (ds_read_b128) of step half `half` of double
    slot d: chunk g + 4 half of the 128-B row, i.e. the half-0 lane address
    with bit 6 flipped (%[vrs1] = %[vrs] ^ 64)."""
    v = "%[vrs]" if half == 0 else "%[vrs1]"
    return [f"ds_read_b128 v[{FS[s] + 4 * m}:{FS[s] + 4 * m + 3}], {v} "
            f"offset:{d * DS_SLOT + m * 2048}" for m in range(8)]


def advance_per_step():
    if VARIANT["nt"]:
        return []
    if VARIANT["ddstt"]:
        return ["s_add_u32 s44, s44, %[k32]", "s_addc_u32 s45, s45, 0"]
    if VARIANT["tt"]:  # (DSD TT: the stored block's next 32 k-rows)
        s = "%[sk32]" if VARIANT["sdd"] else 8192
        return [f"s_add_u32 s40, s40, {s}", "s_addc_u32 s41, s41, 0"]
    return (["s_add_u32 s40, s40, 8192", "s_addc_u32 s41, s41, 0"] if VARIANT["dds"]
            else ["s_add_u32 s44, s44, %[k32]", "s_addc_u32 s45, s45, 0"])


def advance_ds():
    if VARIANT["ddstt"]:
        return ["s_add_u32 s40, s40, 128", "s_addc_u32 s41, s41, 0"]
    if VARIANT["nt"]:
        return ["s_add_u32 s40, s40, 128", "s_addc_u32 s41, s41, 0",
                "s_add_u32 s44, s44, 128", "s_addc_u32 s45, s45, 0"]
    return (["s_add_u32 s44, s44, 128", "s_addc_u32 s45, s45, 0"]
            if VARIANT["dds"] or VARIANT["tt"]
            else ["s_add_u32 s40, s40, 128", "s_addc_u32 s41, s41, 0"])


def ds_counts():
    """DMA instructions a wave issues in an (odd, even) step."""
    if VARIANT["nt"]:
        return (20, 0)
    if VARIANT["ddstt"]:
        return (12, 8)
    return (18, 2) if VARIANT["dds"] or VARIANT["tt"] else (12, 8)


def own_reads_kc(d, half, s):
    """SDD NT: the wave's 8 column-tile fragments (ds_read_b128 of its B
    rows) into the A-operand set."""
    v = "%[vrk0]" if half == 0 else "%[vrk1]"
    return [f"ds_read_b128 v[{FD[s] + 4 * n}:{FD[s] + 4 * n + 3}], {v} "
            f"offset:{d * DS_SLOT + n * 2048}" for n in range(8)]


def step_ds(dt, H, zero_c=False, wait=None, stores=(), flag=False, pre=(),
            no_dma=False, no_reads=False):
    """Step H of a block in double-slot mode: as step(), with the per-step
    image's DMAs of step + 3 every step and the double slot of steps + 3 and
    + 4 on odd H (fed steps 0-1 / 2-3 of a block). At gap 1 every DMA of
    step - 2 has landed (in-order vmcnt: step - 1's may fly), which covers
    both images of step + 1. The shared double slot of DSD is refilled only
    after this step's barrier: its previous steps were read up to the step
    before (every wave has finished that step once all passed the barrier).
    (Early publish, publish_sequence: `wait` overrides the gap-1 count,
    `stores` adds (gap, instruction) pairs after the gap's own work, `flag`
    raises the pair flag after the barrier, `pre` (gap, instruction) pairs
    before it. Consumer last block, consumer_last_block: `no_dma` drops the
    step's DMAs (they would feed steps past the row's end), `no_reads` its
    fragment reads (the step after does not exist), `wait` -1 no wait.)"""
    dds = VARIANT["dds"]
    cur, nxt = H % 2, 1 - H % 2
    gaps = [[] for _ in range(64)]
    if H == 0:
        gaps[0] += idx_load()
    n_odd, n_even = ds_counts()
    for g, ins in pre:
        gaps[g].append(ins)
    w = wait if wait is not None else (n_odd if (H - 1) % 2 == 1 else n_even)
    if w >= 0:
        gaps[1].append(f"s_waitcnt vmcnt({w})")
    if H == 1:
        gaps[1] += switch()
    s1 = (H + 1) % 4
    kc = s_reads_ds(s1 // 2, s1 % 2, nxt)
    if VARIANT["ddstt"]:
        own, shared = t_reads(s1, nxt), own_reads_kc(s1 // 2, s1 % 2, nxt)
    elif VARIANT["nt"]:
        own, shared = own_reads_kc(s1 // 2, s1 % 2, nxt), kc
        if dds:  # DDS NT: A operand (FD) from the shared image (B's rows,
            # %[vrk*]), B operand (FS) from the wave's rows of A (%[vrs*])
            own, shared = shared, own
    elif VARIANT["tt"]:
        own, shared = own_reads_kc(s1 // 2, s1 % 2, nxt), d_reads(s1, nxt, FS)
    else:
        tr = d_reads(s1, nxt)
        own, shared = (kc, tr) if dds else (tr, kc)
    if no_reads:
        own, shared = [], []
    for i, ins in enumerate(own):
        gaps[READS_AT + i].append(ins)
    bar = READS_AT + len(own)
    if not (VARIANT["bar2"] and not dds and not VARIANT["tt"] and H % 2 == 0):
        gaps[bar].append("s_barrier")
        if flag:
            gaps[bar] += raise_flag("e")
    for i, ins in enumerate(shared):
        gaps[bar + 1 + i].append(ins)
    fed = (H + 3) % 4
    if VARIANT["nt"]:
        # the wave's own double slot anywhere, the shared one after the
        # barrier (gap 10)
        pos_per, pos_ds = [], [51, 54, 57, 60]
    elif (dds or VARIANT["tt"]) and not VARIANT["ddstt"]:
        pos_per, pos_ds = [3, 9], [13 + 3 * i for i in range(16)]
    else:
        pos_per, pos_ds = [3, 9, 15, 21, 27, 33, 39, 45], [30, 36, 42, 48]
    placed = list(zip(per_step_dmas(fed), pos_per))
    if H % 2 == 1:
        placed += list(zip(ds_dmas(fed // 2), pos_ds))
        if VARIANT["nt"]:
            placed += list(zip(own_ds_dmas(fed // 2), [3 + 3 * i for i in range(16)]))
    if no_dma:
        placed = []
    for (m0, ld), k in placed:
        gaps[k - 1].append(m0)
        gaps[k].append(ld)
    adv = 61 if VARIANT["nt"] else 59   # after the step's last DMA
    if H != 0:
        gaps[adv] += advance_per_step()
    if H == 1:
        gaps[adv] += advance_ds()
    for g, ins in stores:
        gaps[g].append(ins)
    gaps[63].append("s_waitcnt lgkmcnt(0)")
    out = []
    for i in range(64):
        out.append(mfma(dt, i // 8, i % 8, cur, zero_c))
        out += gaps[i]
    return out


def raise_flag(tag=""):
    """The last wave's lane 0 stores this launch's epoch into the pair flag
    (sc1), unless the test fault bit is set (publish's tail)."""
    return ["s_bitcmp1_b32 %[flags], 3", f"s_cbranch_scc0 L_noflag{tag}_%=",
            "s_bitcmp1_b32 %[flags], 2", f"s_cbranch_scc1 L_noflag{tag}_%=",
            "s_mov_b64 s[78:79], exec", "s_mov_b64 exec, 1",
            "v_mov_b32 v96, 0", "v_mov_b32 v97, %[epoch]",
            "global_store_dword v96, v97, %[flag] sc1",
            "s_mov_b64 exec, s[78:79]",
            f"L_noflag{tag}_%=:"]


def _is_vmem(ins):
    return ins.startswith(("buffer_load", "buffer_store", "global_"))


def publish_sequence(dt):
    """Early publish (double-slot variants; a pair producer whose own row
    follows its head, %[pubat] = n2 + 1): the head's last block's step 3
    stores every accumulator tile of the head partial as soon as its last
    MFMA is 8 slots behind (sc1, from the AGPRs, per-lane address v[96 +
    i / 4] = %[vpl] + 4 KiB (i / 4)), the rest in the gaps of the next
    block's step 0 before that step's zero-C MFMAs overwrite them; the
    k-loop runs on meanwhile. vmcnt counts loads, stores and LDS-DMA
    together in issue order (MI355X_MICROARCH.md, s_waitcnt), so each step's
    wait is recounted here over the actual instruction stream: all but the
    operations younger than the last DMA of the step two back. The first
    step whose wait leaves no store younger than that DMA has every store of
    the wave complete; after its barrier (every wave passed its own wait)
    the last wave raises the flag. Returns (instructions, rejoin label)."""
    n_odd, n_even = ds_counts()
    k1 = 63 - n_odd  # stores in step 3 (vmcnt counts to 63)

    def store(i):
        return (f"buffer_store_dwordx4 a[{4 * i}:{4 * i + 3}], v{96 + i // 4}, s[84:87], 0 "
                f"offen offset:{(i % 4) * 1024} sc1")
    pre = [(2 + j // 3, f"v_add_u32 v{96 + j}, {j * 4096}, %[vpl]") for j in range(16)]
    specs = [dict(H=3, stores=[(i + 8, store(i)) for i in range(k1)], pre=pre),
             dict(H=0, zero_c=True, stores=[(2 + j, store(k1 + j)) for j in range(64 - k1)])]
    for H in (1, 2, 3, 0, 1):
        specs.append(dict(H=H))
    steps = []
    for j, sp in enumerate(specs):
        ins = step_ds(dt, sp["H"], sp.get("zero_c", False), wait=None if j == 0 else 999,
                      stores=sp.get("stores", ()), pre=sp.get("pre", ()))
        steps.append(ins)
    # recount the waits of steps 1.. (step 0's is the loop's own)
    out_steps = [steps[0]]
    flag_at = None
    for j in range(1, len(specs)):
        # the youngest DMA at or before step j - 2 (a step may issue none:
        # NT's even steps); everything issued after it may still fly
        younger = []
        for t in range(j - 1, -1, -1):
            dmas_t = [k for k, x in enumerate(steps[t]) if x.startswith("buffer_load")
                      and x.endswith("lds")]
            if t <= j - 2 and dmas_t:
                younger = [x for x in steps[t][dmas_t[-1] + 1:] if _is_vmem(x)] + younger
                break
            younger = [x for x in steps[t] if _is_vmem(x)] + younger
        w = len(younger)
        assert w <= 63, w
        stores_younger = any(x.startswith("buffer_store") for x in younger)
        sp = specs[j]
        flag = not stores_younger
        ins = step_ds(dt, sp["H"], sp.get("zero_c", False), wait=w,
                      stores=sp.get("stores", ()), flag=flag)
        steps[j] = ins
        out_steps.append(ins)
        if flag:
            flag_at = j
            break
    # the flag must be up before the producer's own row can end (its first
    # block ends with the sequence's first step 3)
    assert flag_at is not None and flag_at <= 4, flag_at
    body = []
    for j, ins in enumerate(out_steps):
        body += ins
        if j == 0:
            body.append("s_sub_u32 s61, s61, 1")
        elif specs[j]["H"] == 3:
            body += ["s_sub_u32 s61, s61, 1", "s_cmp_lg_u32 s61, 0",
                     "s_cbranch_scc0 L_exit_%="]
    nxt = (specs[flag_at]["H"] + 1) % 4
    return body, {0: "L_loop_%=", 1: "L_mid_%=", 2: "L_s2_%=", 3: "L_s3_%="}[nxt]


def _pload(f):
    """sc1 load of the pair partial's fragment f (1 KiB per wave) into slot
    f % 32 = v[96 + 4 (f % 32)] (soffset s78 = 4 KiB (f / 4), set first)."""
    v = 96 + 4 * (f % 32)
    return [f"s_mov_b32 s78, {(f // 4) * 4096}",
            f"buffer_load_dwordx4 v[{v}:{v + 3}], %[vpl], s[84:87], s78 offen "
            f"offset:{(f % 4) * 1024} sc1"]


def publish_last(dt, stamps=False):
    """A producer with nothing after its head (a pair producer whose own row
    is empty, a split-mode first chunk; %[publast] = 1): the head's last step
    stores the partial's tiles 0-55 as each is final (sc1, 8 MFMA slots
    behind, as publish_sequence), tiles 56-63 follow the step, then every
    store drained, one barrier, and the last wave's flag -- the flag goes up
    about a step after the last MFMA instead of after a 256 KiB publish."""
    def store(i):
        return (f"buffer_store_dwordx4 a[{4 * i}:{4 * i + 3}], v{96 + i // 4}, s[84:87], 0 "
                f"offen offset:{(i % 4) * 1024} sc1")
    pre = [(2 + j // 3, f"v_add_u32 v{96 + j}, {j * 4096}, %[vpl]") for j in range(16)]
    out = ["s_memrealtime %[r3]", "s_waitcnt lgkmcnt(0)"] if stamps else []
    out += step_ds(dt, 3, stores=[(i + 8, store(i)) for i in range(56)], pre=pre)
    out += ["s_nop 7", "s_nop 7", "s_nop 7"]
    out += [store(i) for i in range(56, 64)]
    out += ["s_waitcnt vmcnt(0)", "s_barrier"] + raise_flag("l")
    if stamps:
        out += ["s_memrealtime %[r4]", "s_waitcnt lgkmcnt(0)"]
    out += ["s_sub_u32 s61, s61, 1"]
    return out


def consumer_last_block(dt):
    """Pair consumer, double-slot variants (%[clbf] = 2, %[clbc] = 1 for a
    consumer of at least 3 blocks, 0 otherwise): the flag is loaded (sc1)
    when the penultimate block starts; when the last block starts that load
    is four steps old (a counted wait), and if the producer has published,
    the last block runs here: its steps 1-3 issue no DMA (each would feed a
    step past the row's end), step 3 no fragment reads, and the partial's
    fragments 0-7 (step 1, into v[96:127], free during the k-loop) and 8-23
    (step 3, into fragment set 0, v[128:191], free once step 2's MFMAs are 8
    slots behind) are loaded (sc1, after the matched poll, as the hand-off
    table requires) while the MFMAs run. The epilogue (epilogue_collect_pre)
    then needs no poll and no DMA drain. Otherwise the normal last block and
    the polling epilogue run. Returns (flag-load code, check code, last
    block)."""
    flag_load = ["v_mov_b32 v96, 0", "global_load_dword v97, v96, %[flag] sc1"]
    # VMEM ops issued after the flag load: the penultimate block's DMAs
    n_odd, n_even = ds_counts()
    k = 2 * (n_odd + n_even)
    check = [f"s_waitcnt vmcnt({k})", "v_readfirstlane_b32 s98, v97",
             "s_cmp_eq_u32 s98, %[epoch]", "s_cbranch_scc0 L_loop_%="]
    loads1 = []
    for f in range(8):
        loads1 += [(4 + 2 * f, x) for x in _pload(f)]
    loads3 = []
    for f in range(8, 24):
        loads3 += [(8 + 2 * (f - 8), x) for x in _pload(f)]
    body = step_ds(dt, 0)
    # step 1 waits for step 3 of the penultimate block (step 0's DMAs fly)
    body += step_ds(dt, 1, wait=n_even, stores=loads1, no_dma=True)
    # step 2 needs step 0's DMAs: every DMA is older than step 1's 8 loads
    body += step_ds(dt, 2, wait=8, no_dma=True)
    # step 3 reads nothing: no wait
    body += step_ds(dt, 3, wait=-1, stores=loads3, no_dma=True, no_reads=True)
    return flag_load, check, body


def epilogue_collect_pre(cvt):
    """Epilogue of a consumer that ran consumer_last_block: fragments 0-23
    of the partial are in v[96:191] (in flight or landed), 24-31 are loaded
    now into v[192:223]; tile i adds slot i % 32 and refills it with
    fragment i + 32; temporaries v[224:255]. Only these loads are in flight
    (the block issued no DMA), in issue order f = 0, 1, ... 63, so tile i
    waits for vmcnt(min(31, 63 - i)) as epilogue_body. Staging and the sums
    are epilogue_body's (acc + partial, the same fp32 additions)."""
    out = []
    for f in range(24, 32):
        out += _pload(f)
    for i in range(64):
        t = 224 + 8 * (i % 4)
        out += [f"v_accvgpr_read_b32 v{t + j}, a{4 * i + j}" for j in range(4)]
        out.append(f"s_waitcnt vmcnt({min(31, 63 - i)})")
        p = 96 + 4 * (i % 32)
        out += [f"v_add_f32 v{t + j}, v{t + j}, v{p + j}" for j in range(4)]
        if i + 32 < 64:
            out += _pload(i + 32)
        out += [f"{cvt} v{t + 4}, v{t}, v{t + 1}", f"{cvt} v{t + 5}, v{t + 2}, v{t + 3}",
                f"ds_write_b64 %[vws{i % 8}], v[{t + 4}:{t + 5}] offset:{4096 * (i // 8)}"]
    return out


def prologue_ds():
    """Block 0: per-step slot 0, double slot 0 (steps 0-1), per-step slot 1;
    wait for the first two; barrier; step 0's reads; per-step slot 2 and
    double slot 1 (steps 2-3). The first loop step (H = 0) then waits with
    the count of an odd step (slot 1 and double slot 0 landed)."""
    out = prologue_setup()

    def issue(pairs):
        r = []
        for m0, ld in pairs:
            r += [m0, "s_nop 0", ld]
        return r
    own_ds = own_ds_dmas if VARIANT["nt"] else (lambda d: [])
    out += issue(per_step_dmas(0)) + advance_per_step()
    out += issue(ds_dmas(0)) + issue(own_ds(0)) + advance_ds()
    out += issue(per_step_dmas(1)) + advance_per_step()
    out += [f"s_waitcnt vmcnt({ds_counts()[1]})", "s_barrier"]
    if VARIANT["ddstt"]:
        out += t_reads(0, 0) + own_reads_kc(0, 0, 0)
    elif VARIANT["nt"]:
        out += own_reads_kc(0, 0, 0) + s_reads_ds(0, 0, 0)
    elif VARIANT["tt"]:
        out += own_reads_kc(0, 0, 0) + d_reads(0, 0, FS)
    else:
        out += d_reads(0, 0) + s_reads_ds(0, 0, 0)
    out += issue(per_step_dmas(2)) + advance_per_step()
    out += issue(ds_dmas(1)) + issue(own_ds(1))
    out.append("s_waitcnt lgkmcnt(0)")
    return out


def convert(cvt, i):
    """Accumulator i (m = i / 8, n = i % 8) -> fp16 / bf16 pairs -> the
    wave's staging region (per-wave layout, see epilogue_body)."""
    t = 96 + 8 * (i % 4)
    m, n = i // 8, i % 8
    out = [f"v_accvgpr_read_b32 v{t + j}, a{4 * i + j}" for j in range(4)]
    out += [f"{cvt} v{t + 4}, v{t}, v{t + 1}", f"{cvt} v{t + 5}, v{t + 2}, v{t + 3}",
            f"ds_write_b64 %[vws{n}], v[{t + 4}:{t + 5}] offset:{4096 * m}"]
    return out


def prologue():
    if VARIANT["ds"]:
        return prologue_ds()
    out = prologue_setup()
    # steps 0 and 1, wait for step 0 only, then step 2's DMA issued behind
    # the step-0 fragment reads: the CU's TA serializes the 30 DMAs of every
    # wave, and only step 0 is needed before the first MFMA
    for slot in range(2):
        for m0, ld in dmas(slot):
            out += [m0, "s_nop 0", ld]
        out += advance()
    # (no accumulator zeroing: the first step's MFMAs take C = 0)
    out += ["s_waitcnt vmcnt(10)", "s_barrier"]
    out += d_reads(0, 0) + (t_reads(0, 0) if VARIANT["tn"] else s_reads(0, 0))
    for m0, ld in dmas(2):
        out += [m0, "s_nop 0", ld]
    out += advance()
    out.append("s_waitcnt lgkmcnt(0)")
    return out


def prologue_setup():
    """Descriptors, loop state, soffsets and block 0's S / D bases."""
    out = ["s_mov_b32 s42, 0x7fffffff", "s_mov_b32 s43, 0x00020000",
           "s_mov_b32 s46, 0x7fffffff", "s_mov_b32 s47, 0x00020000",
           "s_mov_b32 s84, %[pdlo]", "s_mov_b32 s85, %[pdhi]",
           "s_mov_b32 s86, 0x7fffffff", "s_mov_b32 s87, 0x00020000",
           "s_mov_b32 s56, 2", "s_mov_b32 s57, 0",
           "s_mov_b32 s58, %[kb1]", "s_mov_b32 s61, %[ntot]",
           "s_mov_b32 s72, " + ("%[s16]" if VARIANT["sdd"] else
                                f"{1024 if col_order() else 4096}"),
           "s_mov_b32 s64, 0"]
    out += [f"s_mul_i32 s{64 + q}, %[k4], {q}" for q in range(1, 8)]
    # block 0: virtual entry 0, k-block kb0 (DDS: storage block bo0; s63 =
    # entry 1's, bo1)
    if col_order():
        out += ["s_lshr_b32 s77, %[bo0], 17", "s_lshl_b32 s76, %[bo0], 15",
                "s_mov_b32 s63, %[bo1]"]
    elif a_rows_t():  # entry 0's k-block of the panel
        out += entry_of("s57", "s78") + ["s_mul_hi_u32 s77, s78, %[sk128]",
                                         "s_mul_i32 s76, s78, %[sk128]"]
    else:
        hi, lo = s_block_shift()
        out += entry_of("s57", "s76")
        out += [f"s_lshr_b32 s77, s76, {hi}", f"s_lshl_b32 s76, s76, {lo}"]
    out += ["s_add_u32 s40, %[sdlo], s76", "s_addc_u32 s41, %[sdhi], s77",
            "s_mul_i32 s76, %[kb0], %[k128]", "s_mul_hi_u32 s77, %[kb0], %[k128]",
            "s_add_u32 s44, %[dtlo], s76", "s_addc_u32 s45, %[dthi], s77"]
    if VARIANT["tp"]:
        out += ["v_readlane_b32 s79, %[vent], 0", "s_lshr_b32 s79, s79, 24",
                "s_lshl_b32 s79, s79, 10", "s_add_u32 s44, s44, s79",
                "s_addc_u32 s45, s45, 0"]
    return out


def publish():
    """Pair producer: the head partial (fp32, write-through sc1) to its slot,
    every wave drained, one barrier, then the last wave's lane 0 raises the
    flag (sc1) with this launch's epoch (the 8-wave kernel's protocol,
    block_gemm.h publish / MI355X_MICROARCH hand-off table row 1)."""
    out = ["s_nop 7", "s_nop 7", "s_nop 7"]
    for i in range(64):
        if i % 4 == 0:
            out.append(f"s_mov_b32 s78, {(i // 4) * 4096}")
        out.append(f"buffer_store_dwordx4 a[{4 * i}:{4 * i + 3}], %[vpl], s[84:87], s78 "
                   f"offen offset:{(i % 4) * 1024} sc1")
    out += ["s_waitcnt vmcnt(0)", "s_barrier",
            "s_bitcmp1_b32 %[flags], 3", "s_cbranch_scc0 L_noflag_%=",
            "s_bitcmp1_b32 %[flags], 2", "s_cbranch_scc1 L_noflag_%=",
            "s_mov_b64 s[78:79], exec", "s_mov_b64 exec, 1",
            "v_mov_b32 v96, 0", "v_mov_b32 v97, %[epoch]",
            "global_store_dword v96, v97, %[flag] sc1",
            "s_mov_b64 exec, s[78:79]",
            "L_noflag_%=:"]
    return out


def epilogue_body(cvt, mode, wave_epi=False):
    """Accumulators -> staging image. Workgroup staging (wave_epi False):
    [128 rows][1040 B] of the whole tile (row 16 m + l % 16, columns
    128 w + 16 n + 4 (l / 16) .. + 3 at %[vw0] / %[vw1] + offset), copied out
    by the HIP code after a barrier. Per-wave staging (wave_epi): the wave's
    own 128 x 128 block in its own D ring region, [128 rows][256 B] with
    16-byte chunk c of row r at c ^ (r & 15) (%[vws<n>] + 4096 m), then the
    wave stores it itself (copy_out). mode "plain"; "collect": + the
    published partial, streamed through v[128:255] (32 fragments in flight,
    sc1 loads); "nan": NaN tile."""
    out = []

    def stage(i, src):
        m, n = i // 8, i % 8
        if wave_epi:
            return f"ds_write_b64 %[vws{n}], {src} offset:{4096 * m}"
        base = "%[vw0]" if m < 4 else "%[vw1]"
        off = 16 * (m % 4) * 1040 + 32 * n
        return f"ds_write_b64 {base}, {src} offset:{off}"

    def load(i):
        v = 128 + 4 * (i % 32)
        return [f"s_mov_b32 s78, {(i // 4) * 4096}",
                f"buffer_load_dwordx4 v[{v}:{v + 3}], %[vpl], s[84:87], s78 offen "
                f"offset:{(i % 4) * 1024} sc1"]

    if mode == "nan":
        nan = NAN_F16 if cvt.endswith("f16_f32") else NAN_BF16
        out += [f"v_mov_b32 v96, {nan}", "v_mov_b32 v97, v96"]
        out += [stage(i, "v[96:97]") for i in range(64)]
        return out
    if mode == "collect":
        for i in range(32):
            out += load(i)
    for i in range(64):
        t = 96 + 8 * (i % 4)
        a = 4 * i
        out += [f"v_accvgpr_read_b32 v{t + j}, a{a + j}" for j in range(4)]
        if mode == "collect":
            out.append(f"s_waitcnt vmcnt({min(31, 63 - i)})")
            p = 128 + 4 * (i % 32)
            out += [f"v_add_f32 v{t + j}, v{t + j}, v{p + j}" for j in range(4)]
            if i + 32 < 64:
                out += load(i + 32)
        out += [f"{cvt} v{t + 4}, v{t}, v{t + 1}", f"{cvt} v{t + 5}, v{t + 2}, v{t + 3}"]
        out.append(stage(i, f"v[{t + 4}:{t + 5}]"))
    return out


def epilogue_plain_interleaved(cvt):
    """Per-wave plain epilogue with the copy-out interleaved: after the 8
    tiles of row tile m are converted and staged, the wave reads rows 16 m ..
    16 m + 15 back (into v[128:159], free after the k-loop, two alternating
    sets) and stores them, so the stores of batch m drain while batch m + 1
    converts."""
    out = ["s_mov_b32 s84, %[cdlo]", "s_mov_b32 s85, %[cdhi]",
           "s_mov_b32 s86, 0x7fffffff", "s_mov_b32 s87, 0x00020000",
           "s_mov_b32 s78, 0"]
    for m in range(8):
        for n in range(8):
            i = 8 * m + n
            t = 96 + 8 * (i % 4)
            out += [f"v_accvgpr_read_b32 v{t + j}, a{4 * i + j}" for j in range(4)]
            out += [f"{cvt} v{t + 4}, v{t}, v{t + 1}", f"{cvt} v{t + 5}, v{t + 2}, v{t + 3}",
                    f"ds_write_b64 %[vws{n}], v[{t + 4}:{t + 5}] offset:{4096 * m}"]
        base = 128 + 16 * (m % 2)
        for j in range(4):
            out.append(f"ds_read_b128 v[{base + 4 * j}:{base + 4 * j + 3}], "
                       f"%[vrb{j}] offset:{4096 * m}")
        out.append("s_waitcnt lgkmcnt(0)")
        for j in range(4):
            out += [f"buffer_store_dwordx4 v[{base + 4 * j}:{base + 4 * j + 3}], %[vco], "
                    f"s[84:87], s78 offen nt",
                    "s_add_u32 s78, s78, %[c4]"]
        out.append("s_nop 1")
    return out


def copy_out():
    """Per-wave epilogue: the wave's staged 128 x 128 block -> C with 16-byte
    nontemporal buffer stores, 4 rows x 256 B per instruction (lane l: row
    4 i + l / 16, chunk l % 16; out-of-range columns carry an offset past
    num_records and are dropped). C descriptor in s[84:87] (the partial's is
    no longer needed), row offset 4 i ldc in s78."""
    out = ["s_waitcnt lgkmcnt(0)",
           "s_mov_b32 s84, %[cdlo]", "s_mov_b32 s85, %[cdhi]",
           "s_mov_b32 s86, 0x7fffffff", "s_mov_b32 s87, 0x00020000",
           "s_mov_b32 s78, 0"]
    for b in range(8):
        base = 96 + 16 * (b % 2)
        idx = [4 * b + j for j in range(4)]
        for j, i in enumerate(idx):
            out.append(f"ds_read_b128 v[{base + 4 * j}:{base + 4 * j + 3}], "
                       f"%[vrb{i % 4}] offset:{4096 * (i // 4)}")
        out.append("s_waitcnt lgkmcnt(0)")
        for j, i in enumerate(idx):
            out += [f"buffer_store_dwordx4 v[{base + 4 * j}:{base + 4 * j + 3}], %[vco], "
                    f"s[84:87], s78 offen nt",
                    "s_add_u32 s78, s78, %[c4]"]
        out.append("s_nop 1")
    return out


def poll():
    """Consumer: wait (bounded, s_memrealtime) for the producer's flag =
    this launch's epoch; every wave polls for itself (each adds only its own
    part of the partial). On time-out wave 0 counts the error and the tile
    becomes NaN."""
    return ["s_memrealtime s[96:97]", "s_waitcnt lgkmcnt(0)",
            "L_poll_%=:",
            "v_mov_b32 v96, 0",
            "global_load_dword v97, v96, %[flag] sc1",
            "s_waitcnt vmcnt(0)", "s_nop 0",
            "v_readfirstlane_b32 s98, v97",
            "s_cmp_eq_u32 s98, %[epoch]", "s_cbranch_scc1 L_got_%=",
            "s_sleep 1",
            "s_memrealtime s[98:99]", "s_waitcnt lgkmcnt(0)",
            "s_sub_u32 s98, s98, s96", "s_subb_u32 s99, s99, s97",
            "s_cmp_lg_u32 s99, 0", "s_cbranch_scc1 L_timeout_%=",
            f"s_cmp_lt_u32 s98, {WAIT_TICKS}", "s_cbranch_scc1 L_poll_%=",
            "L_timeout_%=:",
            "s_bitcmp1_b32 %[flags], 4", "s_cbranch_scc0 L_nan_%=",
            "s_mov_b64 s[78:79], exec", "s_mov_b64 exec, 1",
            "v_mov_b32 v96, 0", "v_mov_b32 v97, 1",
            "global_atomic_add v96, v97, %[err]",
            "s_waitcnt vmcnt(0)",
            "s_mov_b64 exec, s[78:79]",
            "s_branch L_nan_%="]


TP_NO_STORES = [False]  # (experiment variant _W2_TP_NS: the flush without its stores)


def tall_flush(cvt, dt, stamps=False):
    """tp: the tile of the block just finished (%[vtile] lane s74 in s75:
    row, panel) is complete. Its 128 x 128 block per wave goes out through
    the one ring slot free at this point -- per-step slot 3 of the wave's D
    ring (8 KiB at 24 KiB: step 3's data, read during step 2; the next
    block's steps 0-2 are in flight into slots 0-2, step 3's DMA is issued in
    its step 0) -- in four rounds of 32 rows: accumulators -> fp16 / bf16 ->
    the per-wave staging layout (epilogue_body), then read back as 4 rows x
    256 B per store (copy_out). Fragment set 1 (v[192:255]: step 3's, done;
    step 0 reads step 1's into it only after this) holds the read-back
    rows. Then drain and restart the next tile's first block from zero (or
    end)."""
    out = ["L_tflush_%=:"]
    if stamps:  # (timeline: %[r3] += flush time, %[r4] += the next two steps')
        out += ["s_memrealtime s[96:97]", "s_waitcnt lgkmcnt(0)"]
    out += ["s_nop 7", "s_nop 7", "s_nop 7",
           "s_and_b32 s76, s75, 0xffff",
           "s_mul_i32 s84, s76, %[crow]", "s_mul_hi_u32 s85, s76, %[crow]",
           "s_add_u32 s84, s84, %[cdlo]", "s_addc_u32 s85, s85, %[cdhi]",
           "s_lshr_b32 s77, s75, 16", "s_and_b32 s77, s77, 0xff",
           "s_lshl_b32 s77, s77, 10",
           "s_add_u32 s84, s84, s77", "s_addc_u32 s85, s85, 0",
           "s_mov_b32 s86, 0x7fffffff", "s_mov_b32 s87, 0x00020000"]
    win = 3 * SLOT
    for k in range(4):
        for m in (2 * k, 2 * k + 1):
            for n in range(8):
                i = 8 * m + n
                t = 96 + 8 * (i % 4)
                out += [f"v_accvgpr_read_b32 v{t + j}, a{4 * i + j}" for j in range(4)]
                out += [f"{cvt} v{t + 4}, v{t}, v{t + 1}", f"{cvt} v{t + 5}, v{t + 2}, v{t + 3}",
                        f"ds_write_b64 %[vws{n}], v[{t + 4}:{t + 5}] "
                        f"offset:{win + 4096 * (m - 2 * k)}"]
        out += ["s_waitcnt lgkmcnt(0)", f"s_mul_i32 s78, %[c4], {8 * k}"]
        for b in (2 * k, 2 * k + 1):
            base = 192 + 16 * (b % 2)
            for j in range(4):
                out.append(f"ds_read_b128 v[{base + 4 * j}:{base + 4 * j + 3}], "
                           f"%[vrb{j}] offset:{win + 4096 * (b - 2 * k)}")
            out.append("s_waitcnt lgkmcnt(0)")
            if TP_NO_STORES[0]:
                continue
            for j in range(4):
                out += [f"buffer_store_dwordx4 v[{base + 4 * j}:{base + 4 * j + 3}], %[vco], "
                        f"s[84:87], s78 offen nt",
                        "s_add_u32 s78, s78, %[c4]"]
    # The next block's steps 0 and 1 run with their waits recounted over
    # the instruction stream (as publish_sequence): the DMAs they wait for
    # are older than these stores, which may still fly; step 2 waits for
    # step 0's DMAs, younger than the stores, with the loop's own count.
    if stamps:  # s88 += this flush, s89 += the next two steps (s96: their start)
        out += ["s_memrealtime s[98:99]", "s_waitcnt lgkmcnt(0)",
                "s_sub_u32 s96, s98, s96", "s_add_u32 s88, s88, s96",
                "s_mov_b32 s96, s98"]
    out += ["s_cmp_eq_u32 s61, 0", "s_cbranch_scc1 L_fin_%="]
    ctx = [step_ds(dt, 2), step_ds(dt, 3) + out]

    def younger_than_dma_of(t, steps):
        dm = [k for k, x in enumerate(steps[t]) if x.startswith("buffer_load")
              and x.endswith("lds")]
        ops = [x for x in steps[t][dm[-1] + 1:] if _is_vmem(x)]
        for u in range(t + 1, len(steps)):
            ops += [x for x in steps[u] if _is_vmem(x)]
        return len(ops)
    w0 = younger_than_dma_of(0, ctx)
    s0 = step_ds(dt, 0, zero_c=True, wait=w0)
    w1 = younger_than_dma_of(1, ctx + [s0])
    s1 = step_ds(dt, 1, wait=w1)
    # then one of the workgroup's zero chunks (%[vzero] lane s90, s90 <
    # %[nzero]; else 32 dummy stores dropped by a zero-size descriptor, so
    # the counts below hold either way): the empty rows' HBM writes overlap
    # the k-loop instead of following it; steps 2 and 3 recounted too
    z = ["s_cmp_lt_u32 s90, %[nzero]", "s_cselect_b32 s86, 0x7fffffff, 0",
         "s_min_u32 s77, s90, 63", "s_add_u32 s90, s90, 1", "s_nop 3",
         "v_readlane_b32 s76, %[vzero], s77",
         "s_and_b32 s77, s76, 0xffff",
         "s_mul_i32 s84, s77, %[crow]", "s_mul_hi_u32 s85, s77, %[crow]",
         "s_add_u32 s84, s84, %[cdlo]", "s_addc_u32 s85, s85, %[cdhi]",
         "s_lshr_b32 s77, s76, 16", "s_lshl_b32 s77, s77, 10",
         "s_add_u32 s84, s84, s77", "s_addc_u32 s85, s85, 0",
         "s_mov_b32 s87, 0x00020000", "s_mov_b32 s78, 0"]
    z += [f"v_mov_b32 v{96 + j}, 0" for j in range(4)]
    for _ in range(32):
        z += ["buffer_store_dwordx4 v[96:99], %[vco], s[84:87], s78 offen nt",
              "s_add_u32 s78, s78, %[c4]"]
    w2 = younger_than_dma_of(2, ctx + [s0, s1 + z])
    s2 = step_ds(dt, 2, wait=w2)
    w3 = younger_than_dma_of(3, ctx + [s0, s1 + z, s2])
    s3 = step_ds(dt, 3, wait=w3)
    assert max(w0, w1, w2, w3) <= 63, (w0, w1, w2, w3)
    tail = []
    if stamps:
        tail = ["s_memrealtime s[98:99]", "s_waitcnt lgkmcnt(0)",
                "s_sub_u32 s98, s98, s96", "s_add_u32 s89, s89, s98"]
    return out + s0 + s1 + z + s2 + s3 + tail + ["s_branch L_blkend_%="]


KS_CHUNKS = (2, 4, 8)


def ksplit_path(cvt, S, g, stamps=False):
    """SDD K-split epilogue (VARIANT "ks", dsd4w.hip): the S workgroups of a
    group each ran K-chunk c of the same 128 x 512 tile; chunk g owns rows
    [128 g / S, 128 (g + 1) / S) of every wave's block, i.e. accumulator
    tiles [64 g / S, 64 (g + 1) / S) (row tile m = i / 8). Each wave stores
    its other tiles (fp32, sc1) to the workgroup's slot (%[pdlo] = the
    group's S slots of 256 KiB, chunk h at h * 256 KiB, wave w at 64 KiB w,
    tile i at 1 KiB i: soffset + offset over %[vpl]), every wave drains, one
    barrier, the last wave's lane 0 stores the epoch into flag h = g of the
    group (%[flag] + 4 g, sc1): the pair publish protocol
    (MI355X_MICROARCH.md hand-off table row 1). Then each wave polls the
    other chunks' flags itself and adds their tiles of its rows, in
    ascending chunk order after its own (a fixed order: the result does not
    depend on which chunk finished first), stages them and stores its rows.
    A wave past the group's count (flags bit 6) stores and loads nothing but
    joins the barrier."""
    T = 64 // S
    own = list(range(g * T, (g + 1) * T))
    peers = [h for h in range(S) if h != g]
    tag = f"{S}_{g}"
    out = [f"L_ks{tag}_%=:",
           "s_bitcmp1_b32 %[flags], 6", f"s_cbranch_scc1 L_ksb{tag}_%="]
    soff = None
    for i in range(64):
        if i in own:
            continue
        v = g * 262144 + (i // 4) * 4096
        if v != soff:
            out.append(f"s_mov_b32 s78, {v}")
            soff = v
        out.append(f"buffer_store_dwordx4 a[{4 * i}:{4 * i + 3}], %[vpl], s[84:87], s78 "
                   f"offen offset:{(i % 4) * 1024} sc1")
    out += [f"L_ksb{tag}_%=:", "s_waitcnt vmcnt(0)", "s_barrier",
            "s_bitcmp1_b32 %[flags], 3", f"s_cbranch_scc0 L_ksnf{tag}_%=",
            "s_bitcmp1_b32 %[flags], 2", f"s_cbranch_scc1 L_ksnf{tag}_%=",
            "s_mov_b64 s[78:79], exec", "s_mov_b64 exec, 1",
            "v_mov_b32 v96, 0", "v_mov_b32 v97, %[epoch]",
            f"global_store_dword v96, v97, %[flag] offset:{4 * g} sc1",
            "s_mov_b64 exec, s[78:79]",
            f"L_ksnf{tag}_%=:"]
    if stamps:
        out += ["s_memrealtime %[r3]", "s_waitcnt lgkmcnt(0)"]
    out += ["s_bitcmp1_b32 %[flags], 6", "s_cbranch_scc1 L_fin_%="]
    # bounded poll of the other chunks' flags (as poll())
    out += ["s_memrealtime s[96:97]", "s_waitcnt lgkmcnt(0)",
            f"L_ksp{tag}_%=:", "v_mov_b32 v96, 0"]
    out += [f"global_load_dword v{97 + k}, v96, %[flag] offset:{4 * h} sc1"
            for k, h in enumerate(peers)]
    out.append("s_waitcnt vmcnt(0)")
    for k in range(len(peers)):
        out += [f"v_readfirstlane_b32 s98, v{97 + k}", "s_cmp_eq_u32 s98, %[epoch]",
                f"s_cbranch_scc0 L_ksw{tag}_%="]
    out += [f"s_branch L_ksg{tag}_%=",
            f"L_ksw{tag}_%=:", "s_sleep 1",
            "s_memrealtime s[98:99]", "s_waitcnt lgkmcnt(0)",
            "s_sub_u32 s98, s98, s96", "s_subb_u32 s99, s99, s97",
            "s_cmp_lg_u32 s99, 0", "s_cbranch_scc1 L_timeout_%=",
            f"s_cmp_lt_u32 s98, {WAIT_TICKS}", f"s_cbranch_scc1 L_ksp{tag}_%=",
            "s_branch L_timeout_%=",
            f"L_ksg{tag}_%=:"]
    if stamps:
        out += ["s_memrealtime %[r4]", "s_waitcnt lgkmcnt(0)"]
    # the other chunks' tiles of this wave's rows: (tile, chunk) loads in
    # order, 32 in flight in v[128:255]
    loads = [(i, h) for i in own for h in peers]
    L = len(loads)

    def load(n):
        i, h = loads[n]
        v = 128 + 4 * (n % 32)
        return [f"s_mov_b32 s78, {h * 262144 + (i // 4) * 4096}",
                f"buffer_load_dwordx4 v[{v}:{v + 3}], %[vpl], s[84:87], s78 offen "
                f"offset:{(i % 4) * 1024} sc1"]
    for n in range(min(32, L)):
        out += load(n)
    n = 0
    for x, i in enumerate(own):
        t = 96 + 8 * (x % 4)
        out += [f"v_accvgpr_read_b32 v{t + j}, a{4 * i + j}" for j in range(4)]
        for _ in peers:
            issued = min(L, 32 + n)
            out.append(f"s_waitcnt vmcnt({min(63, issued - n - 1)})")
            p = 128 + 4 * (n % 32)
            out += [f"v_add_f32 v{t + j}, v{t + j}, v{p + j}" for j in range(4)]
            if n + 32 < L:
                out += load(n + 32)
            n += 1
        m, c = i // 8, i % 8
        out += [f"{cvt} v{t + 4}, v{t}, v{t + 1}", f"{cvt} v{t + 5}, v{t + 2}, v{t + 3}",
                f"ds_write_b64 %[vws{c}], v[{t + 4}:{t + 5}] offset:{4096 * m}"]
    # this chunk's rows of the staged block -> C (copy_out's batches b0..)
    b0, nb = 8 * g // S, 8 // S
    out += ["s_waitcnt lgkmcnt(0)",
            "s_mov_b32 s84, %[cdlo]", "s_mov_b32 s85, %[cdhi]",
            "s_mov_b32 s86, 0x7fffffff", "s_mov_b32 s87, 0x00020000",
            f"s_mul_i32 s78, %[c4], {4 * b0}"]
    for b in range(b0, b0 + nb):
        base = 96 + 16 * (b % 2)
        for j in range(4):
            out.append(f"ds_read_b128 v[{base + 4 * j}:{base + 4 * j + 3}], "
                       f"%[vrb{j}] offset:{4096 * b}")
        out.append("s_waitcnt lgkmcnt(0)")
        for j in range(4):
            out += [f"buffer_store_dwordx4 v[{base + 4 * j}:{base + 4 * j + 3}], %[vco], "
                    f"s[84:87], s78 offen nt",
                    "s_add_u32 s78, s78, %[c4]"]
        out.append("s_nop 1")
    out.append("s_branch L_fin_%=")
    return out


def ksplit():
    """Dispatch on %[kss] (S) and %[kch] (this workgroup's chunk), then the
    paths."""
    out = ["L_ks_%=:"]
    for S in KS_CHUNKS:
        for g in range(S):
            out += [f"s_cmp_eq_u32 %[kss], {S}", f"s_cbranch_scc0 L_ksn{S}_{g}_%=",
                    f"s_cmp_eq_u32 %[kch], {g}", f"s_cbranch_scc1 L_ks{S}_{g}_%=",
                    f"L_ksn{S}_{g}_%=:"]
    out.append("s_branch L_fin_%=")  # (never: kss is one of KS_CHUNKS here)
    return out


def build(dt, wave_epi=False, last_block=False, stamps=False, dds=False, ds=False,
          sdd=False, nt=False, tt=False, bar2=False, tn=False, ddstt=False, il=False,
          ks=False, tp=False):
    VARIANT.update(dds=dds, ds=ds, sdd=sdd, nt=nt, tt=tt, bar2=bar2, tn=tn, ddstt=ddstt,
                   il=il, ks=ks, tp=tp)
    try:
        return _build(dt, wave_epi, last_block, stamps)
    finally:
        VARIANT.update(dds=False, ds=False, sdd=False, nt=False, tt=False, bar2=False,
                       tn=False, ddstt=False, il=False, ks=False, tp=False)


def _build(dt, wave_epi, last_block, stamps):
    """stamps (experiment builds, SPUTNIK_EXP & 512): s_memrealtime into the
    outputs %[r0] (k-loop start), %[r1] (k-loop end), %[r2] (body end), %[r3]
    and %[r4] (a producer's publish start and end)."""
    cvt = f"v_cvt_pk_{dt}_f32"
    body = prologue()
    if VARIANT["tp"]:  # zero chunks done in the loop
        body.append("s_mov_b32 s90, 0")
    if stamps and VARIANT["tp"]:
        body += ["s_mov_b32 s88, 0", "s_mov_b32 s89, 0"]
    if stamps:
        body.append("s_memrealtime %[r0]")
    # the first block's step 0 is the zero-C copy below (L_first)
    body.append("s_branch L_first_%=")
    # early publish (publish_sequence): double-slot variants with pairs
    early = VARIANT["ds"] and not VARIANT["bar2"] and not VARIANT["sdd"]
    body.append("L_loop_%=:")
    body += step(dt, 0)
    body.append("L_mid_%=:")
    for H in (1, 2, 3):
        if H == 2:
            body.append("L_s2_%=:")
        if H == 3:
            if early:  # the head's last block of a producer (own row after it / none)
                body += ["s_cmp_eq_u32 s61, %[pubat]", "s_cbranch_scc1 L_pubs_%=",
                         "s_cmp_eq_u32 s61, %[publast]", "s_cbranch_scc1 L_publ_%="]
            body.append("L_s3_%=:")
        body += step(dt, H)
    if VARIANT["tp"]:
        body.append("L_blkend_%=:")
    body.append("s_sub_u32 s61, s61, 1")
    if VARIANT["tp"]:  # the block just done ends its tile: store the tile
        body += ["s_sub_u32 s74, %[ntot], s61", "s_sub_u32 s74, s74, 1", "s_nop 3",
                 "v_readlane_b32 s75, %[vtile], s74", "v_readlane_b32 s76, %[vtile2], s74",
                 "s_cmp_lt_u32 s74, 64", "s_cselect_b32 s75, s75, s76",
                 "s_bitcmp1_b32 s75, 31", "s_cbranch_scc1 L_tflush_%="]
    body += ["s_cmp_eq_u32 s61, %[flushrem]", "s_cbranch_scc1 L_pub_%="]
    if early:  # pair consumer: flag load / consumer last block
        body += ["s_cmp_eq_u32 s61, %[clbf]", "s_cbranch_scc1 L_clbf_%=",
                 "s_cmp_eq_u32 s61, %[clbc]", "s_cbranch_scc1 L_clbc_%="]
    if last_block:
        # one block left and no publish or collect after it: the
        # specialized last block (L_last)
        body += ["s_cmp_eq_u32 s61, 1", "s_cbranch_scc0 L_cont_%=",
                 "s_bitcmp1_b32 %[flags], 1", "s_cbranch_scc1 L_last_%=",
                 "L_cont_%=:"]
    body += ["s_cmp_lg_u32 s61, 0", "s_cbranch_scc1 L_loop_%=",
             "s_branch L_exit_%="]
    if last_block:
        body.append("L_last_%=:")
        if stamps:
            body.append("s_memrealtime %[r1]")
        body += step(dt, 0)
        for H in (1, 2, 3):
            body += step(dt, H, last=H, cvt=cvt)
        body += ["s_nop 7", "s_nop 7"] + convert(cvt, 62) + convert(cvt, 63)
        body.append("s_branch L_done_%=")
    if early:
        seq, rejoin = publish_sequence(dt)
        body.append("L_pubs_%=:")
        body += seq
        body.append(f"s_branch {rejoin}")
        body.append("L_publ_%=:")
        body += publish_last(dt, stamps)
        body.append("s_branch L_zero_%=")
        flag_load, check, clb = consumer_last_block(dt)
        body.append("L_clbf_%=:")
        body += flag_load
        body.append("s_branch L_loop_%=")
        body.append("L_clbc_%=:")
        body += check
        body += clb
        if stamps:
            body.append("s_memrealtime %[r1]")
        # no DMA in flight, the wave's ring reads done (step 2's lgkmcnt)
        body += ["s_nop 7", "s_nop 7"]
        body += epilogue_collect_pre(cvt)
        body.append("s_branch L_done_%=")
    body.append("L_pub_%=:")
    if stamps:
        body += ["s_memrealtime %[r3]", "s_waitcnt lgkmcnt(0)"]
    body += publish()
    if stamps:
        body += ["s_memrealtime %[r4]", "s_waitcnt lgkmcnt(0)"]
    body += ["s_cmp_eq_u32 s61, 0", "s_cbranch_scc1 L_zero_%="]
    # step 0 of a block with the accumulators restarting from zero (C = 0):
    # the launch's first step, and the first step after a pair publish
    body.append("L_first_%=:")
    body += step(dt, 0, zero_c=True)
    body.append("s_branch L_mid_%=")
    body.append("L_zero_%=:")
    # a split-mode first chunk (flags bit 5) has no tile of its own: done
    # once its partial is published
    body += ["s_bitcmp1_b32 %[flags], 5", "s_cbranch_scc1 L_fin_%="]
    body += [f"v_accvgpr_write_b32 a{i}, 0" for i in range(256)]
    body.append("L_exit_%=:")
    if stamps:
        body.append("s_memrealtime %[r1]")
    if wave_epi:
        # the wave's own DMAs (the loop's last three steps fed clamped
        # dummies) landed and its reads are done: its D ring region is free
        # (no other wave writes it), no barrier
        body += ["s_waitcnt vmcnt(0)", "s_nop 7", "s_nop 7"]
    else:
        # every DMA landed and every wave's reads are done: the LDS is free
        # for the staging image
        body += ["s_waitcnt vmcnt(0)", "s_barrier", "s_nop 7", "s_nop 7"]
    if VARIANT["ks"]:
        body += ["s_cmp_gt_u32 %[kss], 1", "s_cbranch_scc1 L_ks_%="]
    body += ["s_bitcmp1_b32 %[flags], 0", "s_cbranch_scc1 L_collect_%="]
    if VARIANT["bar2"] or VARIANT["il"]:
        # (with bar2 / il: the plain epilogue stores each 16-row batch as
        # soon as its 8 tiles are staged)
        body += epilogue_plain_interleaved(cvt)
        body.append("s_branch L_end_%=")
    else:
        body += epilogue_body(cvt, "plain", wave_epi)
        body.append("s_branch L_done_%=")
    body.append("L_collect_%=:")
    body += poll()
    body.append("L_got_%=:")
    body += epilogue_body(cvt, "collect", wave_epi)
    body.append("s_branch L_done_%=")
    if VARIANT["tp"]:
        body += tall_flush(cvt, dt, stamps)
    if VARIANT["ks"]:
        body += ksplit()
        for S in KS_CHUNKS:
            for g in range(S):
                body += ksplit_path(cvt, S, g, stamps)
    body.append("L_nan_%=:")
    body += epilogue_body(cvt, "nan", wave_epi)
    body += ["L_done_%=:"]
    body += copy_out() if wave_epi else ["s_waitcnt lgkmcnt(0)"]
    if VARIANT["bar2"] or VARIANT["il"]:
        body.append("L_end_%=:")
    body.append("L_fin_%=:")
    if stamps and VARIANT["tp"]:
        body.append("s_mov_b64 %[r3], s[88:89]")
    if stamps:
        body += ["s_memrealtime %[r2]", "s_waitcnt lgkmcnt(0)"]
    return body


def render():
    lines = ["// generated by sputnik_amd/csrc/gen_dsd4w.py -- do not edit", ""]
    for dt in ("f16", "bf16"):
        for suffix, wave_epi, last_block in (("", False, False), ("_W", True, False),
                                             ("_WL", True, True)):
            name = f"DSD4W_ASM_{dt.upper()}{suffix}"
            lines.append(f"#define {name} \\")
            lines += [f'  "{ins}\\n" \\' for ins in build(dt, wave_epi, last_block)]
            lines += ['  ""', ""]
        # the default epilogue with timeline stamps (experiment builds)
        lines.append(f"#define DSD4W_ASM_{dt.upper()}_W_T \\")
        lines += [f'  "{ins}\\n" \\' for ins in build(dt, True, False, True)]
        lines += ['  ""', ""]
        # DDS NN (the same kernel with the operand images swapped); _W2: the
        # double-slot k-contiguous image, DSD and DDS
        for name, dds, ds, sdd, nt, tt in (("_W_DDS", True, False, False, False, False),
                                           ("_W2", False, True, False, False, False),
                                           ("_W2_DDS", True, True, False, False, False),
                                           ("_W2_SDD", False, True, True, False, False),
                                           ("_W2_SDD_NT", False, True, True, True, False),
                                           ("_W2_SDD_TT", False, True, True, False, True),
                                           ("_W2_SDD_KS", False, True, True, False, False),
                                           ("_W2_NT", False, True, False, True, False),
                                           ("_W2_DDS_NT", True, True, False, True, False),
                                           ("_W2_TT", False, True, False, False, True)):
            lines.append(f"#define DSD4W_ASM_{dt.upper()}{name} \\")
            lines += [f'  "{ins}\\n" \\'
                      for ins in build(dt, True, False, False, dds, ds, sdd, nt, tt,
                                       ks=name.endswith("_KS"))]
            lines += ['  ""', ""]
        # DDS NN (double slots) with timeline stamps (experiment builds)
        lines.append(f"#define DSD4W_ASM_{dt.upper()}_W2_DDS_T \\")
        lines += [f'  "{ins}\\n" \\'
                  for ins in build(dt, True, False, True, dds=True, ds=True)]
        lines += ['  ""', ""]
        # tall DSD NN, persistent (tall_flush), with and without stamps
        lines.append(f"#define DSD4W_ASM_{dt.upper()}_W2_TP \\")
        lines += [f'  "{ins}\\n" \\' for ins in build(dt, True, ds=True, tp=True)]
        lines += ['  ""', ""]
        TP_NO_STORES[0] = True
        lines.append(f"#define DSD4W_ASM_{dt.upper()}_W2_TP_NS \\")
        lines += [f'  "{ins}\\n" \\'
                  for ins in build(dt, True, False, True, ds=True, tp=True)]
        lines += ['  ""', ""]
        TP_NO_STORES[0] = False
        lines.append(f"#define DSD4W_ASM_{dt.upper()}_W2_TP_T \\")
        lines += [f'  "{ins}\\n" \\'
                  for ins in build(dt, True, False, True, ds=True, tp=True)]
        lines += ['  ""', ""]
        # the SDD K-split with timeline stamps (experiment builds)
        lines.append(f"#define DSD4W_ASM_{dt.upper()}_W2_SDD_KS_T \\")
        lines += [f'  "{ins}\\n" \\'
                  for ins in build(dt, True, False, True, ds=True, sdd=True, ks=True)]
        lines += ['  ""', ""]
        # DSD / DDS / SDD TN (per-step images, per-wave epilogue)
        for name, dds, sdd in (("_W_TN", False, False), ("_W_DDS_TN", True, False),
                               ("_W_SDD_TN", False, True)):
            lines.append(f"#define DSD4W_ASM_{dt.upper()}{name} \\")
            lines += [f'  "{ins}\\n" \\'
                      for ins in build(dt, True, dds=dds, sdd=sdd, tn=True)]
            lines += ['  ""', ""]
        # DDS TT
        lines.append(f"#define DSD4W_ASM_{dt.upper()}_W2_DDS_TT \\")
        lines += [f'  "{ins}\\n" \\'
                  for ins in build(dt, True, dds=True, ds=True, ddstt=True)]
        lines += ['  ""', ""]
        # _W4: double slots with the interleaved plain epilogue (DSD)
        lines.append(f"#define DSD4W_ASM_{dt.upper()}_W4 \\")
        lines += [f'  "{ins}\\n" \\' for ins in build(dt, True, ds=True, il=True)]
        lines += ['  ""', ""]
        # the shipped DSD NN variants (_W2, _W4) with timeline stamps
        # (experiment builds, SPUTNIK_EXP & 512)
        for name, il in (("_W2_T", False), ("_W4_T", True)):
            lines.append(f"#define DSD4W_ASM_{dt.upper()}{name} \\")
            lines += [f'  "{ins}\\n" \\'
                      for ins in build(dt, True, False, True, ds=True, il=il)]
            lines += ['  ""', ""]
        # _W3*: double slots with a barrier every other step
        for name, sdd, nt in (("_W3", False, False), ("_W3_SDD", True, False),
                              ("_W3_SDD_NT", True, True)):
            lines.append(f"#define DSD4W_ASM_{dt.upper()}{name} \\")
            lines += [f'  "{ins}\\n" \\'
                      for ins in build(dt, True, False, False, False, True, sdd, nt,
                                       False, True)]
            lines += ['  ""', ""]
    clob = ([f'"a{i}"' for i in range(256)] + [f'"v{i}"' for i in range(96, 256)]
            + [f'"s{i}"' for i in range(40, 48)] + [f'"s{i}"' for i in range(56, 80)]
            + [f'"s{i}"' for i in range(84, 91)] + [f'"s{i}"' for i in range(96, 100)]
            + ['"scc"', '"vcc"', '"memory"'])
    lines.append("#define DSD4W_CLOBBERS " + ", ".join(clob))
    return "\n".join(lines) + "\n"


def main():
    with open(sys.argv[1], "w") as f:
        f.write(render())


if __name__ == "__main__":
    main()
