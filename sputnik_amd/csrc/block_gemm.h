// sputnik-amd: the block-sparse GEMM kernel for gfx950 (CDNA4, MI355X).
//
// One kernel template serves every product of the hot path. It computes an
// output tile O[i][j] = sum_k S[i][k] * D[k][j] of 128 x BN, where
//   S = the "row operand": one 128-row block-row of a BCSR matrix (DSD, DDS)
//       or a 128-row panel of a dense matrix (SDD),
//   D = the dense operand, a BN-wide panel,
// and writes O either straight (DSD), transposed (DDS computes C^T = B^T A^T)
// or into one 128x128 block of a BCSR output (SDD).
//
// It replaces the whole CUTLASS stack of the reference:
//   BlockGemm::operator()              block_gemm.h:749-878
//   ConfigHelper / OutputConfig        block_gemm.h:22-510
//   BlockTileAccessIterator            block_tile_access_iterator.h:23-322
//   DependentTileAccessIterator        dependent_tile_access_iterator.h:12-178
//   BlockTileOutputIterator (+epilogue) block_tile_output_iterator.h:18-230
//   swizzles                            threadblock_swizzle.h:6-69
// but is designed for CDNA4, not translated:
//   * 64-wide waves; 2 x (BN/64) waves, each owning a 64x64 sub-tile computed
//     with v_mfma_f32_16x16x32_{f16,bf16} (4x4 accumulators of 16x16).
//   * Operands stream HBM/L2 -> LDS with buffer_load_dwordx4 ... lds (LDS-DMA,
//     no VGPR staging) into a 3-stage ring of BK=64 slices, kept in flight
//     across raw s_barriers with counted vmcnt waits.
//   * Partial tiles (N, M, K not multiples of the tile) are zero-filled by the
//     buffer unit's range check (out-of-range lanes read 0), so the MFMA loop
//     never branches on bounds.
//   * Each operand is read from LDS in whichever orientation it has in HBM:
//     k-contiguous images with ds_read_b128, m/n-contiguous images with the
//     gfx950 transpose read ds_read_b64_tr_b16. Both images are XOR-swizzled
//     on the DMA source address so every read is bank-conflict free.
//   * The sparse row's (k-block, storage-block) list is staged once per tile
//     into LDS; each k-step resolves its block pointer with one LDS read and a
//     readfirstlane (wave-uniform -> SGPR buffer descriptor), so there is no
//     dependent global load on the critical path (the reference's TODO at
//     dependent_tile_access_iterator.h:146-147).
//   * Workgroup -> tile mapping is XCD-aware: the 8 XCDs each get a
//     contiguous run of tiles that share dense panels in their private L2.
#ifndef SPUTNIK_AMD_BLOCK_GEMM_H_
#define SPUTNIK_AMD_BLOCK_GEMM_H_

#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

// Ablation switches for performance experiments only (scripts/exp_build.sh);
// the shipped library is built with SPUTNIK_EXP == 0.
//   1: skip the MFMAs (keep LDS reads)   2: skip the operand DMA
//   4: no LPT row order                  8: no XCD-aware tile map
//  64: every DMA re-reads the first step's tiles (cache-resident: isolates
//      the memory system from the LDS-write / issue cost of the DMA)
// 128: per-segment cycle sums of the k-loop into GemmParams::debug
// 512: per-workgroup timeline into GemmParams::debug (scripts/exp_timeline.py)
#ifndef SPUTNIK_EXP
#define SPUTNIK_EXP 0
#endif
// Cache-policy bits (buffer aux: 1 sc0, 2 nt, 16 sc1) of the sparse-operand
// and dense-operand DMA. On an XCD every sparse block is read once (the XCD
// owns one dense panel), so it is streamed with nt by default and leaves the
// L2 to the dense panel that every workgroup of the XCD re-reads.
#ifndef SPUTNIK_S_AUX
#define SPUTNIK_S_AUX 0
#endif
#ifndef SPUTNIK_D_AUX
#define SPUTNIK_D_AUX 0
#endif
// Scalar-index configs: load the next stored block's (k-block, storage
// block) one block ahead, so the scalar-cache round trip is off the DMA
// issue path.
#ifndef SPUTNIK_IDX_PREFETCH
#define SPUTNIK_IDX_PREFETCH 0
#endif
// Fragment reads of the next step before this step's DMA issue.
#ifndef SPUTNIK_READ_FIRST
#define SPUTNIK_READ_FIRST 0
#endif
// DSD / DDS staggered pipeline unrolled by one stored block (constant ring
// slots, branch-free steady state); 0 = the generic per-step pipeline.
#ifndef SPUTNIK_BLOCK_LOOP
#define SPUTNIK_BLOCK_LOOP 1
#endif
// The same block loop for the grouped SDD (groups of 4 k-steps).
#ifndef SPUTNIK_SDD_BLOCK_LOOP
#define SPUTNIK_SDD_BLOCK_LOOP 1
#endif
// Staggered configs: static s_setprio(1) for the lagging (younger) half.
// Tall configuration: scalar index loads (see kScalarIdx).
#ifndef SPUTNIK_TALL_SIDX
#define SPUTNIK_TALL_SIDX 1
#endif
// Output stores are nontemporal (global_store ... nt): the output is written
// once and not re-read by the launch. Dense outputs (DSD / DDS / DSS):
// config 5 262 -> 236 us, DSD 4096^3 50% 63.1 -> 61.8 us (interleaved A/B,
// r02). Sparse outputs (SDD / SSD / SDS) are normally read back at once by
// the next product, see SPUTNIK_SPARSE_OUT_NT.
#ifndef SPUTNIK_OUT_NT
#define SPUTNIK_OUT_NT 1
#endif
#ifndef SPUTNIK_SPARSE_OUT_NT
#define SPUTNIK_SPARSE_OUT_NT 0
#endif
#ifndef SPUTNIK_LAG_PRIO
#define SPUTNIK_LAG_PRIO 1
#endif

namespace sputnik_amd {

constexpr int kBlock = 128;        // BCSR block edge (only 128 is supported)
constexpr int kBM = 128;           // output tile rows = one sparse block-row
constexpr int kMaxIndexChunk = 1024;  // sparse-row entries staged in LDS at once
constexpr int kLptRows = 256;      // rank block-rows in-kernel up to this many
constexpr uint32_t kOOB = 0x80000000u;      // buffer offset that reads as 0
constexpr uint32_t kNumRecords = 0x7fffffffu;

typedef short s16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef _Float16 f16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned v4u __attribute__((ext_vector_type(4)));

#define SPUTNIK_LDS(p) ((__attribute__((address_space(3))) void *)(p))
#define SPUTNIK_LDS_S4(p) ((__attribute__((address_space(3))) s16x4 *)(p))

// Kernel arguments (passed by value). Byte strides everywhere.
struct GemmParams {
  const char *s_data;          // sparse: block data; SDD: dense A'
  const int *s_offsets;        // sparse: entry range per row
  const short *s_indices;      // sparse: k-block per entry
  const int *s_block_offsets;  // sparse, column order: storage block per entry
  long long s_ld;              // SDD: row (or k-line) stride of A' in bytes
  const char *d_data;          // dense operand
  long long d_ld;              // its row (or k-line) stride in bytes
  char *c_data;                // output
  long long c_ld;              // dense output row stride in bytes
  const short *c_row_indices;  // SDD: block-row of each output block
  const int *c_offsets;        // SDD, grouped tiles: C's BCSR row offsets
  const short *c_indices;      // SDD: block-col of each output block
  int num_rows;                // sparse: #block-rows of S
  int num_jtiles;              // sparse: #BN-wide tiles of the dense extent
  int j_limit;                 // dense extent (elements) of the j dimension
  int k_limit;                 // SDD: K (elements)
  int num_tiles;               // output tiles (one-tile-per-workgroup grid)
  // Persistent launch (tall DSD / DDS, dispatch.cpp UseTall): `grid`
  // workgroups; workgroup b runs tile b, then the tiles it fetches from
  // tile_counter, back to back (persistent = 0: one tile per workgroup,
  // grid = num_tiles).
  int grid;
  int persistent;
  // Persistent launches fetch their tiles past the first `grid` from
  // tile_counter[0] (one atomic per tile, issued a tile ahead): tile = grid +
  // fetched. Each launch starts from zero and leaves zero behind: a
  // workgroup whose fetch ran past the last tile arrives on tile_counter[1],
  // and the grid's last arriver resets both words. No host-side state
  // advances per launch, so launch order, a failed launch or a second host
  // thread on the stream cannot skew the tile numbering.
  unsigned long long *tile_counter;
  // Pair balancing (staggered one-workgroup-per-CU configs, see the
  // kernel): the block-rows of each panel are paired heaviest-with-lightest;
  // the light workgroup also computes the head of the heavy row and hands it
  // over as an fp32 partial. pair == 0: one tile per workgroup, LPT order.
  int pair;
  float *pair_partials;        // (#pairs) x (128 x BN) fp32
  unsigned *pair_flags;        // #pairs; holds the epoch of the launch whose
                               // producer published last (never reset)
  unsigned pair_epoch;         // this launch's epoch (never 0)
  // Launches captured into a graph replay one set of arguments, so their
  // epoch lives on the device: pair_sync = [epoch word, arrival count] of
  // the capture's own workspace. Every workgroup reads the epoch word at
  // its start and uses (word mod 2^31) + 1; each adds 1 to the arrival count
  // as it exits, and the last one (every other workgroup has read the word)
  // resets the count and advances the word for the next replay. nullptr:
  // eager launch, the host's pair_epoch.
  unsigned *pair_sync;
  unsigned *pair_error;        // += 1 per consumer that timed out
  int pair_fault;              // test knob: producers never publish
  // Pair launches with 8 panels: XCD x (= workgroup b mod 8) takes panels
  // 2(x/2) and 2(x/2)+1 for half of the pairs instead of one panel for all
  // of them, so it streams half of S (each block used by two tiles) and
  // two D panels (host: dispatch.cpp PreparePairs). 0 off; 1 / 3 which
  // XCD of a panel pair takes the heavy half of the pairs; 2 interleaved.
  int pair_xcd2;
  // Split mode (pair_split = 2; at most half as many tiles as CUs, e.g. the
  // 512 to 2048-row panels of a strong-scaled 4096^2): grid = 2 x
  // num_tiles. The tile's row is cut into two halves of its blocks; the
  // first half's workgroup (dispatched first) publishes its fp32 partial,
  // the second half's adds it and writes the tile. (4 and 8 chunks were
  // slower at every panel height measured: each further partial costs its
  // consumer a 256 KiB collect, r03b.)
  int pair_split;
  int split_bn;                // split mode: columns per tile (512/256/128)
  unsigned long long *debug;   // SPUTNIK_EXP & 128 builds only
  // DSS (dense = sparse x sparse): op(B)'s column lists (k-block, storage
  // block) — B's transposed metadata, or its own when op(B) = B^T.
  const int *d_offsets;
  const short *d_indices;
  const int *d_block_offsets;  // nullptr: storage block = entry
  // Stored blocks of the sparse operand S (DSD: A's nonzeros / 128^2); the
  // 4-wave DSD kernel preloads an index list this short (dsd4w.hip).
  int s_blocks;
  // SDD K-split (4-wave grouped SDD NN with few groups, dispatch.cpp
  // PrepareSddKsplit): up to this many workgroups per group, each a slice of
  // K, reduced through the pair workspace (pair_partials: 256 KiB per
  // workgroup; ks_flags: one flag per workgroup, pair_epoch / pair_sync /
  // pair_error as pairs). 0 or 1: off.
  int sdd_ksplit;
  unsigned *ks_flags;
  // Grouped SDD on the 4-wave kernel, every row the same group count:
  // 0 group-major order, 1 blocks of 8 rows x 4 groups (dsd4w.hip).
  int sdd_order;
  // Tall DSD pipeline (dsd4w.hip kEpi 7): weight of a tile's store in
  // quarter blocks (the cost-balanced cut of the block sequence).
  int tall_flush_w;
  int tall_odd_share;  // ... and an odd XCD's workgroup share, percent of an even one's
  // 4-wave pair launches: the smallest hand-off (blocks) a pair makes;
  // below it the heavy row keeps its blocks (0: SPUTNIK_MIN_HANDOFF).
  int min_handoff;
  // 4-wave plain launches with 64..kLptRows rows of equal count, R % 8 == 0:
  // XCD x takes a contiguous eighth of the rows over every panel
  // (dsd4w.hip; 0: the panel-major XCD map).
  int xcd_rows;
  // 4-wave grouped SDD (not the K-split): start each group's k-walk at a
  // rotated k-block (0 off; 1 by row, 2 by group index, 3 by tile, 4 by
  // band of 8 rows; dsd4w.hip), a tuning experiment for power-of-two strides.
  int sdd_krot;
  // 4-wave grouped SDD, RB x GB block order over rows of equal count: the GB
  // groups of a round taken G / GB apart along the row instead of adjacent
  // (1; 0 adjacent), so its B columns span more of B's rows (dsd4w.hip;
  // knob sdd_spread, on for NT by default). The blocks computed are the same
  // either way: only which groups run side by side changes.
  int sdd_spread;
  // SDD tail split (knob sdd_tail; sdd_tail_rows below): the grouped 4-wave
  // launch takes C's rows [0, R0) and an 8-wave launch of one block per
  // workgroup the stored blocks of rows [R0, R), so the groups' last round
  // is not a few groups on an idle chip. tail_cus: the CUs (the round size).
  int sdd_tail;
  int tail_cus;
};

// XOR key of the m/n-contiguous image: spreads the 8 k-rows one
// ds_read_b64_tr_b16 half-wave touches over 8 distinct 32-byte bank sectors.
__device__ __forceinline__ int tr_key(int k) {
  return (k & 3) | (((k >> 3) & 1) << 2);
}
// XOR key of the k-contiguous image (rows of kChunks 16-byte chunks, i.e.
// 128-byte rows at BK=64, 64-byte rows at BK=32): makes each 16-lane
// ds_read_b128 group hit 16 distinct 16-byte slots (checked exhaustively for
// both widths by scripts/lds_banks.py).
template <int kChunks>
__device__ __forceinline__ int kc_key(int row) {
  return (row >> 1) & (kChunks - 1);
}

template <typename T>
struct MfmaTraits;
template <>
struct MfmaTraits<_Float16> {
  static __device__ __forceinline__ f32x4 mfma(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_f16(
        __builtin_bit_cast(f16x8, a), __builtin_bit_cast(f16x8, b), c, 0, 0,
        0);
  }
};
template <>
struct MfmaTraits<__bf16> {
  static __device__ __forceinline__ f32x4 mfma(s16x8 a, s16x8 b, f32x4 c) {
    return __builtin_amdgcn_mfma_f32_16x16x32_bf16(
        __builtin_bit_cast(bf16x8, a), __builtin_bit_cast(bf16x8, b), c, 0, 0,
        0);
  }
};

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const char *base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<char *>(base), 0,
                                           kNumRecords, 0x00020000);
}

// Wave-uniform loads through the scalar cache (s_load_dword): the sparse
// index list is read-only for the whole launch. An int16 entry is taken from
// its aligned dword, so any 2-byte-aligned base works.
__device__ __forceinline__ int scalar_load_short(const short *base, int e) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(base + e);
  const int v = *reinterpret_cast<const __attribute__((address_space(4))) int *>(
      a & ~uintptr_t(3));
  return ((a & 2) ? (v >> 16) : v) & 0xffff;
}
__device__ __forceinline__ int scalar_load_int(const int *base, int e) {
  return *(const __attribute__((address_space(4))) int *)(base + e);
}

template <int kAux = 0>
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, char *lds_dst,
                                      uint32_t voffset) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, SPUTNIK_LDS(lds_dst), 16,
                                           voffset, 0, 0, kAux);
}

// 16x32 operand fragment from a k-contiguous image [rows][BK] (kRowBytes =
// 2*BK per row): lane l gets row (row0 + l%16), k = 32*kk + 8*(l/16) .. +7.
template <int kRowBytes>
__device__ __forceinline__ s16x8 read_kc(const char *img, int row0, int kk,
                                         int lane) {
  const int row = row0 + (lane & 15);
  const int c = 4 * kk + (lane >> 4);
  return *reinterpret_cast<const s16x8 *>(
      img + row * kRowBytes + ((c ^ kc_key<kRowBytes / 16>(row)) << 4));
}

// Same fragment from an m/n-contiguous image [64 k][cols] (kRowBytes per
// k-row) via two transpose reads: lane l gets column (col0 + l%16) of
// k = 32*kk + 8*(l/16) + {0..3} and then + {4..7}.
//
// Issued as inline asm on purpose: hipcc cannot tell a ds_read_tr builtin
// from the LDS-DMA writes still in flight and puts an s_waitcnt vmcnt(0) in
// front of it, which would drain the whole prefetch ring every k-step. The
// caller therefore owns the lgkmcnt wait for these registers (wait_step).
template <int kRowBytes>
__device__ __forceinline__ s16x8 read_mn(const char *img, int col0, int kk,
                                         int lane) {
  const int q = (lane >> 2) & 3;
  const int p = lane & 3;
  const int g = lane >> 4;
  const int sector = col0 >> 4;
  s16x4 lo, hi;
  const int k = 32 * kk + 8 * g + q;
  // (image + lane's row/piece) is shared by every fragment of a step, the
  // swizzled sector term is loop-invariant: one add per fragment per step.
  const uint32_t row_base = (uint32_t)(uintptr_t)(
      (__attribute__((address_space(3))) const char *)(img)) +
      (uint32_t)(k * kRowBytes + (p << 3));
  const uint32_t addr = row_base + (uint32_t)((sector ^ tr_key(k)) << 5);
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(lo) : "v"(addr));
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2"
               : "=v"(hi)
               : "v"(addr), "n"(4 * kRowBytes));
  s16x8 out;
  out[0] = lo[0]; out[1] = lo[1]; out[2] = lo[2]; out[3] = lo[3];
  out[4] = hi[0]; out[5] = hi[1]; out[6] = hi[2]; out[7] = hi[3];
  return out;
}

// Maps the launch index to a tile index so that each XCD (blocks b and b+8
// share one) walks a contiguous run of tiles. Bijective for any grid size.
// The hardware deals workgroup b of a launch to XCD (b + r) mod 8, r a
// rotation set by the device's dispatch history across queues (the same r
// for every workgroup of one launch; it moves when another stream's work is
// dispatched in between -- scripts/diag_xcc*.py). The XCD
// tile maps below only need "b mod 8 = one XCD"; the speed skews (pair
// placement, the tall pipeline's odd-XCD share) need the physical XCD,
// read here from the XCC_ID hardware register.
__device__ __forceinline__ int xcd_rotation() {
  unsigned v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return ((int)(v & 7u) - (int)(blockIdx.x & 7u)) & 7;
}
// 1 for logical XCD x (b mod 8) of this launch on a physically even XCD,
// the faster half of the XCDs (~6% per block in the 4-wave
// k-loop, ~20% in the tall pipeline). The placement knobs were tuned in
// processes whose rotation was 7, where this equals x & 1 -- what they
// used to read.
__device__ __forceinline__ int fast_xcd(int x, int rot) { return ((x + rot) & 1) ^ 1; }

// SDD tail split (GemmParams::sdd_tail). The grouped SDD runs one group of
// up to 4 stored blocks of a row per workgroup, G = sum_r ceil(n_r / 4)
// groups in rounds of `cus`: with G = 2 cus + 24 (SDD 8192^3 at 50%: 536
// groups) the third round is 24 groups, as long as a full round, on an idle
// chip. When that last round holds at most cus / 4 groups, R0 = the most
// rows [0, R0) whose groups fit the full rounds (G(R0) <= G - G % cus);
// the stored blocks of rows [R0, R) -- at most cus of them, else no split --
// go to one 8-wave launch of a block per workgroup (~2/3 of a grouped round
// at K = 8192: 8192^3 50% 511 -> 454 us).
// Rows of equal count (group-major orders) are not split. Every workgroup of
// both launches computes the same R0 from C's offsets (deterministic); R0 ==
// R: no split. scratch: >= 2 kThreads / 64 + 2 ints of LDS, free.
template <int kThreads>
__device__ int sdd_tail_rows(const GemmParams &p, int *scratch, int tid) {
  constexpr int kWaves = kThreads / 64;
  const int R = p.num_rows, cus = p.tail_cus;
  const int lane = tid & 63, wave = tid >> 6;
  if (tid == 0) {
    scratch[kWaves] = 0x7fffffff;  // fewest groups in a row
    scratch[kWaves + 1] = 0;       // most groups in a row
  }
  __syncthreads();
  const int per = (R + kThreads - 1) / kThreads;
  const int r0 = min(R, tid * per), r1 = min(R, r0 + per);
  int local = 0, gmin = 0x7fffffff, gmax = 0;
  for (int r = r0; r < r1; ++r) {
    const int g = (p.c_offsets[r + 1] - p.c_offsets[r] + 3) / 4;
    local += g;
    gmin = min(gmin, g);
    gmax = max(gmax, g);
  }
  int incl = local;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int v = __shfl_up(incl, d, 64);
    if (lane >= d) incl += v;
  }
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    gmin = min(gmin, __shfl_xor(gmin, d, 64));
    gmax = max(gmax, __shfl_xor(gmax, d, 64));
  }
  if (lane == 63) scratch[wave] = incl;
  if (lane == 0) {
    atomicMin(&scratch[kWaves], gmin);
    atomicMax(&scratch[kWaves + 1], gmax);
  }
  __syncthreads();
  int before = 0, total = 0;
  for (int w = 0; w < kWaves; ++w) {
    before += w < wave ? scratch[w] : 0;
    total += scratch[w];
  }
  const bool uniform = scratch[kWaves] == scratch[kWaves + 1];
  __syncthreads();
  // (a last round of at most a quarter of the CUs: one block per workgroup
  // on the 8-wave tile takes ~2/3 of a grouped round at K = 8192, so a
  // fuller round is better left alone -- SDD 8192^3 at 30%, 84 groups past
  // two rounds: 332 -> 340 us split)
  const int rem = cus > 0 ? total % cus : 0;
  if (uniform || rem == 0 || rem > cus / 4 || total <= rem) return R;  // (block-uniform)
  // the most rows whose groups fit the full rounds: G(r) <= cap
  const int cap = total - rem;
  int cum = before + incl - local, best = -1;
  if (r0 < R && cum <= cap) best = r0;
  for (int r = r0; r < r1; ++r) {
    cum += (p.c_offsets[r + 1] - p.c_offsets[r] + 3) / 4;
    if (cum <= cap) best = r + 1;
  }
  if (tid == 0) scratch[0] = 0;
  __syncthreads();
  if (best > 0) atomicMax(&scratch[0], best);
  __syncthreads();
  const int cand = scratch[0];
  __syncthreads();  // scratch reads done
  const int tail = p.c_offsets[R] - p.c_offsets[cand];
  return tail > 0 && tail <= cus ? cand : R;
}

__device__ __forceinline__ int xcd_tile(int bid, int nwg) {
  const int xcd = bid & 7;
  const int q = nwg >> 3;
  const int r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// Tile configuration. The output tile is 128 x kBN; kWM x kWN waves each own
// a (128/kWM) x (kBN/kWN) sub-tile of 16x16 MFMA accumulators; kBK is the k
// depth of one LDS ring slot; kWGs workgroups are meant to share a CU (it
// sets the register budget through __launch_bounds__ and must match the LDS
// footprint).
template <int BN_, int WM_, int WN_, int BK_, int STAGES_, int WGS_,
          int STAGGER_ = 0, int KSPLIT_ = 1, int SPLITMODE_ = 0>
struct TileConfig {
  static constexpr int kBN = BN_, kWM = WM_, kWN = WN_, kBK = BK_;
  static constexpr int kStages = STAGES_, kWGs = WGS_;
  // The pair split mode (GemmParams::pair_split) is its own instantiation,
  // so the pair-balanced kernel's register allocation is not disturbed by it
  // (with both in one kernel, hipcc spills an accumulator in the last
  // block's steps).
  static constexpr bool kSplitMode = SPLITMODE_ != 0;
  // kKSplit = 2: two wave sets own the same kWM x kWN sub-tiles and split
  // each slot's k depth between them (set h takes k-half h); their fp32
  // accumulators are summed through LDS before the epilogue.
  static constexpr int kKSplit = KSPLIT_;
  static constexpr int kWaves = WM_ * WN_ * KSPLIT_;
  // kStagger: the two halves of the waves (wave w and w + kNW/2 share a
  // SIMD) run one barrier apart, so one half's DMA/read phase overlaps the
  // other half's MFMA phase (needs kStages >= 4; see the pipeline).
  static constexpr bool kStagger = STAGGER_ != 0;
};

// 8 waves, 64x64 each, BK=64, one workgroup per CU (first-generation DSD/DDS).
using CfgWide = TileConfig<256, 2, 4, 64, 3, 1>;
// 4 waves, 64x128 each, BK=32, two workgroups per CU: 25% fewer LDS fragment
// bytes per MFMA than CfgWide and two independent barrier domains per CU
// (the r01 default before CfgWide8S).
using CfgDual = TileConfig<256, 2, 2, 32, 3, 2>;
// 2 waves of 128x128 (one per SIMD, 512-register budget), BK=32, two
// workgroups per CU (measured slower than CfgDual: DESIGN.md §10).
using CfgQuad = TileConfig<256, 1, 2, 32, 3, 2>;
// 128x512 tile, 4 waves of 128x128, BK=32, one workgroup per CU (measured
// slower than CfgDual: DESIGN.md §10).
using CfgWide512 = TileConfig<512, 1, 4, 32, 3, 1>;
// 128x512 tile, 8 waves of 64x128, BK=32, one workgroup per CU (measured
// slower than CfgDual without cross-workgroup balancing: DESIGN.md §10).
using CfgWide8 = TileConfig<512, 2, 4, 32, 3, 1>;
// DSD/DDS default: CfgWide8 with staggered wave halves and a 4-slot ring
// (the whole 160 KiB LDS; the sparse index list is then read with scalar
// loads, not staged), pair-balanced across block-rows (dispatch.cpp).
using CfgWide8S = TileConfig<512, 2, 4, 32, 4, 1, 1>;
// The same pipeline in split mode: two workgroups per tile (few tiles), at
// 512, 256 or 128 columns per tile (8 staggered waves of 64x128 / 64x64 /
// 64x32), the widest that still fills the CUs (dispatch.cpp PreparePairs).
using CfgWide8Split = TileConfig<512, 2, 4, 32, 4, 1, 1, 1, 1>;
using CfgSplit256 = TileConfig<256, 2, 4, 32, 4, 1, 1, 1, 1>;
using CfgSplit128 = TileConfig<128, 2, 4, 32, 4, 1, 1, 1, 1>;
// SDD: one 128x128 output block per workgroup, 4 waves of 64x64, BK=64.
using CfgBlock = TileConfig<128, 2, 2, 64, 3, 1>;
// SDD, one block per workgroup with K split inside it: 8 waves in two
// staggered halves, each half a 2x2 set of 64x64 sub-tiles over its k-half of
// a 64-deep slot (two waves per SIMD where CfgBlock has one).
using CfgBlockKS = TileConfig<128, 2, 2, 64, 4, 1, 1, 2>;
// SDD, grouped: up to 4 consecutive stored blocks of one block-row per
// workgroup (shared S rows, D columns gathered per lane), on the staggered
// 128x512 pipeline of CfgWide8S.
using CfgSddGrouped = TileConfig<512, 2, 4, 32, 4, 1, 1>;
// 128x128 tile, 4 waves of 64x64, BK=32, three workgroups per CU (12 waves:
// three per SIMD to hide each wave's DMA/read issue chain).
using CfgTri = TileConfig<128, 2, 2, 32, 3, 3>;
// Same tile, two workgroups per CU.
using CfgBlock2 = TileConfig<128, 2, 2, 32, 3, 2>;

#ifndef SPUTNIK_SPARSE_CFG
#define SPUTNIK_SPARSE_CFG CfgWide8S
#endif
using CfgSparse = SPUTNIK_SPARSE_CFG;  // DSD / DDS tile configuration
using CfgSplit = CfgWide8Split;        // DSD / DDS in split mode
// DSD / DDS over tall sparse operands (more block-rows than kLptRows).
#ifndef SPUTNIK_TALL_CFG
#define SPUTNIK_TALL_CFG CfgDual
#endif
using CfgTall = SPUTNIK_TALL_CFG;
// k-split SDD (CfgBlockKS) vs CfgBlock, DSD-shaped 4096^3, interleaved A/B
// (scripts/exp_ks*.sh): 20% 54.9 -> 33.2 us, 50% 114.9 -> 74.8 us, 90%
// 216.6 -> 147.9 us, parity green on every reference SDD problem.
#ifndef SPUTNIK_SDD_CFG
#define SPUTNIK_SDD_CFG CfgBlockKS
#endif
using CfgSdd = SPUTNIK_SDD_CFG;        // SDD tile configuration (BN = 128)
// The same k split on SSD / SDS / DSS, 4096^3 fp16 (sparse inputs 50%, sparse
// output 20%; scripts/exp_ksall.sh): SSD 37.3 -> 29.9 us, SDS 35.3 -> 29.1 us,
// DSS NT 86.6 -> 62.4 us, parity green on all their reference problems.
#ifndef SPUTNIK_SS_CFG
#define SPUTNIK_SS_CFG CfgBlockKS
#endif
using CfgSs = SPUTNIK_SS_CFG;          // SSD / SDS tile configuration
#ifndef SPUTNIK_DSS_CFG
#define SPUTNIK_DSS_CFG CfgBlockKS
#endif
using CfgDss = SPUTNIK_DSS_CFG;        // DSS tile configuration

// Bounded wait for the pair hand-off: a launch can never hang on a missing
// partial. The producer never waits and always has a lower workgroup index
// than its consumer (in-order dispatch), so the bound is a guard, not part
// of the protocol: 0.2 s (s_memrealtime, 100 MHz), ~3000x the longest tile
// at 4096^2 x 4096, long enough to ride out a time-sliced preemption of the
// producer. A consumer that gives up does not use the partial: it poisons
// its tile with NaN (never a silently wrong number) and counts the event in
// GemmParams::pair_error (sputnik_pair_errors()); the per-launch epoch keeps
// a late publish from satisfying any later launch. (A consumer that instead
// recomputes the head itself was built three ways in r03 — a second pass of
// the pipeline, a cold in-kernel path, a non-inlined function — and every
// one pushed the kernel's hot path into scratch, 2-4 us per tile.)
constexpr unsigned long long kPairWaitTicks = 20000000;

// kSparseOut: sparse output block. With kSparseIn = false that is SDD (dense
// S); with kSparseIn = true, SSD / SDS (sparse S, as DSD / DDS, restricted to
// the output's nonzero blocks: one 128x128 block per workgroup). Without
// kSparseOut: DSD / DDS (sparse S, dense output).
// kSKC / kDKC: S / D are k-contiguous in memory (else m/n-contiguous).
// kOutT: write O transposed (DDS).
template <typename T, bool kSparseOut, bool kSKC, bool kDKC, bool kOutT,
          class Cfg, bool kSparseIn = false, bool kSparseD = false>
__global__ void __launch_bounds__(64 * Cfg::kWaves,
                                  Cfg::kWGs * Cfg::kWaves / 4)
    block_gemm_kernel(const GemmParams p) {
  constexpr int kBN = Cfg::kBN;
  constexpr int kBK = Cfg::kBK;
  constexpr int kStages = Cfg::kStages;
  constexpr int kWN = Cfg::kWN;
  constexpr int kNW = Cfg::kWaves;           // waves per workgroup
  constexpr int kKS = Cfg::kKSplit;
  constexpr int kTM = kBM / Cfg::kWM;        // wave sub-tile rows
  constexpr int kTN = kBN / Cfg::kWN;        // wave sub-tile cols
  constexpr int kFM = kTM / 16;              // 16x16 accumulators per wave
  constexpr int kFN = kTN / 16;
  constexpr int kKK = kBK / 32 / kKS;        // MFMA k-steps per slot and wave
  constexpr int kThreads = 64 * kNW;
  constexpr int kSBytes = kBM * kBK * 2;
  constexpr int kDBytes = kBK * kBN * 2;
  constexpr int kStageBytes = kSBytes + kDBytes;
  constexpr int kSInstr = kSBytes / 1024 / kNW;  // DMA instrs / wave / stage
  constexpr int kDInstr = kDBytes / 1024 / kNW;
  constexpr int kGroup = kSInstr + kDInstr;      // vmcnt per stage
  constexpr int kKcRow = kBK * 2;                // k-contiguous image row
  constexpr int kKcChunks = kBK / 8;
  constexpr int kKcRowsPerInstr = 64 / kKcChunks;
  constexpr int kDRowBytes = kBN * 2;            // D m/n-contiguous row
  constexpr int kDChunksPerRow = kBN / 8;
  constexpr int kDRowsPerInstr = 64 / kDChunksPerRow;
  constexpr int kStepsPerBlock = kBlock / kBK;
  constexpr int kRingBytes = kStages * kStageBytes;
  // Index list staged per chunk in LDS (smaller when three workgroups share
  // a CU); staggered configs read it with scalar loads instead.
  // The tall configuration (CfgTall, persistent, 0-3 blocks per tile at
  // config 5) reads it with scalar loads too: no staging round trip and no
  // barrier pair per tile (SPUTNIK_TALL_SIDX=0: staged).
  constexpr bool kTallCfg = std::is_same<Cfg, CfgTall>::value && !kSparseOut;
  constexpr bool kScalarIdx =
      (Cfg::kStagger || (SPUTNIK_TALL_SIDX != 0 && kTallCfg)) && !kSparseIn &&
      !kSparseD;
  constexpr int kIndexChunk = Cfg::kWGs >= 3 ? 256 : kMaxIndexChunk;
  constexpr bool kDenseS = kSparseOut && !kSparseIn;  // SDD
  static_assert(!kSparseIn || (kSparseOut &&
                               (!Cfg::kStagger || Cfg::kKSplit == 2) &&
                               kBN == kBlock),
                "SSD/SDS: one output block per workgroup, per-step pipeline");
  // DSS: D is op(B)'s column block, one 128x128 output tile per workgroup;
  // the k-list is the intersection of op(A)'s row and op(B)'s column.
  static_assert(!kSparseD || (!kSparseOut && !kOutT &&
                              (!Cfg::kStagger || Cfg::kKSplit == 2) &&
                              kBN == kBlock),
                "DSS: dense 128x128 tiles, per-step pipeline");
  constexpr int kDssMaxK = 256;  // k-blocks (K <= 32768, as the reference)
  constexpr int kIdxBytes =
      kDenseS ? (Cfg::kStagger ? 0 : 16)
              : (kScalarIdx ? (Cfg::kStagger ? 0 : 16) : kIndexChunk * 6 + 16);
  // SDD with kBN > 128: a tile is a group of up to kGrp stored blocks of one
  // block-row, found in-kernel from C's offsets (rows <= kMaxGroupRows).
  constexpr bool kGroupedSdd = kDenseS && kBN > kBlock;
  constexpr int kGrp = kBN / kBlock;
  static_assert(!Cfg::kStagger || kStages >= 4, "stagger needs 4 slots");
  static_assert(!Cfg::kStagger || kNW % 2 == 0, "halves");
  static_assert(kKS == 1 || (kKS == 2 && Cfg::kStagger && kBN == kBlock &&
                             !kGroupedSdd && kKK >= 1),
                "k split: staggered single-block tiles only");
  static_assert(kSInstr * kNW * 1024 == kSBytes, "S DMA split");
  static_assert(kDInstr * kNW * 1024 == kDBytes, "D DMA split");
  static_assert(kTM % 16 == 0 && kTN % 16 == 0 && kBK % 32 == 0, "tiles");
  static_assert(Cfg::kWGs * (kRingBytes + kIdxBytes) <= 163840, "LDS budget");

  // One LDS array (a second __shared__ object can make hipcc drain the DMA
  // ring before every ds_read): [ring | idx_kc | idx_blk | 4 scratch ints].
  __shared__ __attribute__((aligned(1024))) char lds[kRingBytes + kIdxBytes];
  short *idx_kc = reinterpret_cast<short *>(lds + kRingBytes);
  int *idx_blk = reinterpret_cast<int *>(lds + kRingBytes + kIndexChunk * 2);
  // 4 scratch ints: after the index list, or (scalar-index configs) inside
  // the ring, which is only used for them before the pipeline starts.
  int *scratch = reinterpret_cast<int *>(
      kIdxBytes >= 16 ? lds + kRingBytes + kIdxBytes - 16 : lds + 4096);

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  // SPUTNIK_EXP & 512: timeline of each workgroup (wave 0; 100 MHz clock):
  // entry, pipeline start, pipeline end, collect end, tile written, pair
  // partial published (producer), pair flag seen (consumer).
  unsigned long long tl_stamp[10] = {};
  unsigned long long tl_cycles[2] = {};  // shader clock at stamps 0 and 4
  auto tl = [&](int i) {
    if constexpr ((SPUTNIK_EXP & 512) != 0) {
      asm volatile("" ::: "memory");
      tl_stamp[i] = __builtin_amdgcn_s_memrealtime();
      if (i == 0) tl_cycles[0] = __builtin_amdgcn_s_memtime();
      if (i == 4) tl_cycles[1] = __builtin_amdgcn_s_memtime();
    }
  };
  tl(0);
  const int wsub = kKS > 1 ? wave % (Cfg::kWM * kWN) : wave;
  const int wm = wsub / kWN;
  const int wn = wsub % kWN;
  // k split: this wave's first 32-deep k-step inside a slot.
  const int kk0 = kKS > 1 ? (wave / (Cfg::kWM * kWN)) * kKK : 0;
  const int row_w = kTM * wm;  // first row / col of this wave's sub-tile
  const int col_w = kTN * wn;


  // ---- per-lane DMA offsets (relative to each step's tile base) ----------
  uint32_t s_off[kSInstr], d_off[kDInstr];
  int s_lk[kSInstr], d_lk[kDInstr];  // k of the lane's chunk (SDD k-mask)
  const long long s_stride = kDenseS ? p.s_ld : 256;
#pragma unroll
  for (int q = 0; q < kSInstr; ++q) {
    const int g = wave * kSInstr + q;
    if constexpr (kSKC) {
      const int row = kKcRowsPerInstr * g + lane / kKcChunks;
      const int c = (lane % kKcChunks) ^ kc_key<kKcChunks>(row);
      s_off[q] = (uint32_t)(row * s_stride + c * 16);
      s_lk[q] = c * 8;
    } else {
      const int k = 4 * g + (lane >> 4);
      const int pc = lane & 15;
      const int c = (((pc >> 1) ^ tr_key(k)) << 1) | (pc & 1);
      s_off[q] = (uint32_t)(k * s_stride + c * 16);
      s_lk[q] = k;
    }
  }
  // D offsets depend on the tile's dense origin j0 (range mask).
  // Grouped SDD: block j of the tile (j < grp_count) takes the D columns
  // grp_col[j] .. +127; lanes of absent blocks read zeros.
  static_assert(kGrp <= 4, "grouped SDD: at most 4 blocks per tile");
  long long grp_b0 = 0;   // SDD: first output block of the tile
  int grp_count = 1;      // SDD: blocks in the tile
  int grp_c0 = 0, grp_c1 = 0, grp_c2 = 0, grp_c3 = 0;  // D column origins
  auto grp_col = [&](int jb) {  // lane-dependent select, no private array
    return jb == 0 ? grp_c0 : jb == 1 ? grp_c1 : jb == 2 ? grp_c2 : grp_c3;
  };
  auto setup_d = [&](int j0) {
#pragma unroll
    for (int q = 0; q < kDInstr; ++q) {
      const int g = wave * kDInstr + q;
      bool ok;
      if constexpr (kDKC) {
        const int j = kKcRowsPerInstr * g + lane / kKcChunks;
        const int c = (lane % kKcChunks) ^ kc_key<kKcChunks>(j);
        int n = j0 + j;
        if constexpr (kGroupedSdd) {
          const int jb = j / kBlock;
          n = grp_col(jb) + j % kBlock;
          ok = jb < grp_count;
          d_off[q] = (uint32_t)(n * p.d_ld + c * 16);
        } else {
          d_off[q] = (uint32_t)(j * p.d_ld + c * 16);
          ok = n < p.j_limit;
        }
        d_lk[q] = c * 8;
      } else {
        const int k = kDRowsPerInstr * g + lane / kDChunksPerRow;
        const int pc = lane % kDChunksPerRow;
        const int c = (((pc >> 1) ^ tr_key(k)) << 1) | (pc & 1);
        if constexpr (kGroupedSdd) {
          const int jb = (c * 8) / kBlock;
          d_off[q] = (uint32_t)(k * p.d_ld +
                                (grp_col(jb) + (c * 8) % kBlock) * 2);
          ok = jb < grp_count;
        } else {
          d_off[q] = (uint32_t)(k * p.d_ld + c * 16);
          ok = j0 + c * 8 < p.j_limit;
        }
        d_lk[q] = k;
      }
      if (!ok) d_off[q] = kOOB;
    }
  };

  f32x4 acc[kFM][kFN];
  auto zero_acc = [&]() {
#pragma unroll
    for (int a = 0; a < kFM; ++a)
#pragma unroll
      for (int b = 0; b < kFN; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  };

  // Issue the DMA of pipeline step `step` into ring slot `slot`. Sparse S:
  // `step` counts from the first entry staged in the LDS index list.
  int srow = 0, j0 = 0;  // current tile
  // Sparse S: the entry's block bases are cached across the kStepsPerBlock
  // steps of one block, so the LDS index lookup (a serialized LDS round
  // trip before the DMA) happens once per block, not once per step.
  int cached_e = -1;
  // Scalar-index configs: entry e of the pipeline is idx_base + e, or, past
  // idx_split entries (a pair producer's second segment), idx_base2 + e -
  // idx_split.
  int idx_base = 0, idx_split = 0x7fffffff, idx_base2 = 0;
  // Index prefetch (SPUTNIK_IDX_PREFETCH): entry pf_e's values, and the end
  // of the pipeline's entry range (no load past it).
  int pf_e = -1, pf_kblk = 0, pf_blk = 0, e_end = 0;
  const char *blk_s = nullptr;
  const char *blk_d = nullptr;
  // issue() = prep() (scalar work: index lookup, tile bases) + fire() (the
  // LDS-DMA instructions), so a step can put its fragment reads between them.
  const char *s_base = nullptr;
  const char *d_base = nullptr;
  int krem = kBK;  // valid k in the prepared step (SDD tail)
  auto prep = [&](int step) {
    if constexpr ((SPUTNIK_EXP & 2) != 0) return;
    if constexpr ((SPUTNIK_EXP & 64) != 0) step = 0;
    if constexpr (kDenseS) {
      const long long k0 = (long long)step * kBK;
      krem = p.k_limit - (int)k0;
      s_base = kSKC ? p.s_data + (long long)srow * kBM * p.s_ld + k0 * 2
                    : p.s_data + k0 * p.s_ld + (long long)srow * kBM * 2;
      if constexpr (kGroupedSdd)  // columns live in the lane offsets
        d_base = kDKC ? p.d_data + k0 * 2 : p.d_data + k0 * p.d_ld;
      else
        d_base = kDKC ? p.d_data + (long long)j0 * p.d_ld + k0 * 2
                      : p.d_data + k0 * p.d_ld + (long long)j0 * 2;
    } else {
      const int e = step / kStepsPerBlock;
      const int h = step % kStepsPerBlock;
      if (e != cached_e) {
        int kblk, blk;
        if constexpr (kScalarIdx) {
          auto entry = [&](int x) {
            return x < idx_split ? idx_base + x : idx_base2 + (x - idx_split);
          };
          if constexpr (SPUTNIK_IDX_PREFETCH != 0) {
            // pf_kblk / pf_blk hold entry cached_e + 1 when it was
            // prefetched (pf_e == e); the next entry is loaded now, while
            // this block's 4 steps run.
            if (pf_e == e) {
              kblk = pf_kblk;
              blk = pf_blk;
            } else {
              const int ge = entry(e);
              kblk = scalar_load_short(p.s_indices, ge);
              blk = p.s_block_offsets != nullptr
                        ? scalar_load_int(p.s_block_offsets, ge)
                        : ge;
            }
            if (e + 1 < e_end) {
              const int gn = entry(e + 1);
              pf_kblk = scalar_load_short(p.s_indices, gn);
              pf_blk = p.s_block_offsets != nullptr
                           ? scalar_load_int(p.s_block_offsets, gn)
                           : gn;
              pf_e = e + 1;
            }
          } else {
            const int ge = entry(e);
            kblk = scalar_load_short(p.s_indices, ge);
            blk = p.s_block_offsets != nullptr
                      ? scalar_load_int(p.s_block_offsets, ge)
                      : ge;
          }
          cached_e = e;
        } else if constexpr (kSparseD) {
          cached_e = e;
          // intersection list staged by the DSS setup: S and D storage blocks
          const int *ls = reinterpret_cast<const int *>(lds + kRingBytes) +
                          kDssMaxK;
          kblk = __builtin_amdgcn_readfirstlane(ls[kDssMaxK + e]);
          blk = __builtin_amdgcn_readfirstlane(ls[e]);
        } else {
          cached_e = e;
          kblk = __builtin_amdgcn_readfirstlane((int)idx_kc[e]);
          blk = __builtin_amdgcn_readfirstlane(idx_blk[e]);
        }
        blk_s = p.s_data + (long long)blk * (kBlock * kBlock * 2);
        if constexpr (kSparseD) {  // kblk holds D's storage block
          blk_d = p.d_data + (long long)kblk * (kBlock * kBlock * 2);
        } else {
          const long long kg = (long long)kblk * kBlock;
          blk_d = kDKC ? p.d_data + (long long)j0 * p.d_ld + kg * 2
                       : p.d_data + kg * p.d_ld + (long long)j0 * 2;
        }
      }
      s_base = blk_s + (kSKC ? h * (kBK * 2) : h * (kBK * 256));
      d_base = blk_d + (kDKC ? (long long)h * (kBK * 2)
                             : (long long)h * kBK * p.d_ld);
    }
  };
  auto fire = [&](int slot) {
    if constexpr ((SPUTNIK_EXP & 2) != 0) return;
    char *slot_base = lds + slot * kStageBytes;
    const __amdgpu_buffer_rsrc_t rs = make_rsrc(s_base);
    const __amdgpu_buffer_rsrc_t rd = make_rsrc(d_base);
#pragma unroll
    for (int q = 0; q < kSInstr; ++q) {
      uint32_t off = s_off[q];
      if constexpr (kDenseS) off = s_lk[q] < krem ? off : kOOB;
      dma16<kDenseS ? 0 : SPUTNIK_S_AUX>(
          rs, slot_base + (wave * kSInstr + q) * 1024, off);
    }
#pragma unroll
    for (int q = 0; q < kDInstr; ++q) {
      uint32_t off = d_off[q];
      if constexpr (kDenseS) off = d_lk[q] < krem ? off : kOOB;
      dma16<SPUTNIK_D_AUX>(rd, slot_base + kSBytes + (wave * kDInstr + q) * 1024,
                           off);
    }
  };
  auto issue = [&](int step, int slot) {
    prep(step);
    fire(slot);
  };

  // Fragment registers of one k-step: [kk][f] for the S (a) and D (b)
  // operands, kk = 32-deep MFMA k-step inside the slot.
  struct Frags {
    s16x8 a[kKK][kFM];
    s16x8 b[kKK][kFN];
  };
  auto read_step = [&](int slot, Frags &F) {
    // Opaque slot offset: with a compile-time slot (pipeline_blocks) the
    // compiler would otherwise hoist every slot's fragment addresses out of
    // the loop and keep 4x the address registers live.
    int slot_off = slot * kStageBytes;
    asm volatile("" : "+s"(slot_off));
    const char *simg = lds + slot_off;
    const char *dimg = simg + kSBytes;
#pragma unroll
    for (int kk = 0; kk < kKK; ++kk) {
#pragma unroll
      for (int f = 0; f < kFM; ++f) {
        if constexpr (kSKC)
          F.a[kk][f] = read_kc<kKcRow>(simg, row_w + 16 * f, kk0 + kk, lane);
        else
          F.a[kk][f] = read_mn<kBM * 2>(simg, row_w + 16 * f, kk0 + kk, lane);
      }
#pragma unroll
      for (int f = 0; f < kFN; ++f) {
        if constexpr (kDKC)
          F.b[kk][f] = read_kc<kKcRow>(dimg, col_w + 16 * f, kk0 + kk, lane);
        else
          F.b[kk][f] = read_mn<kDRowBytes>(dimg, col_w + 16 * f, kk0 + kk, lane);
      }
    }
  };
  auto wait_step = [&](Frags &F) {
    __builtin_amdgcn_sched_barrier(0);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
    for (int kk = 0; kk < kKK; ++kk) {
#pragma unroll
      for (int f = 0; f < kFM; ++f) asm volatile("" : "+v"(F.a[kk][f]));
#pragma unroll
      for (int f = 0; f < kFN; ++f) asm volatile("" : "+v"(F.b[kk][f]));
    }
    __builtin_amdgcn_sched_barrier(0);
  };
  auto mfma_step = [&](Frags &F) {
    if constexpr ((SPUTNIK_EXP & 1) != 0) {
#pragma unroll
      for (int kk = 0; kk < kKK; ++kk) {
#pragma unroll
        for (int a = 0; a < kFM; ++a) asm volatile("" ::"v"(F.a[kk][a]));
#pragma unroll
        for (int b = 0; b < kFN; ++b) asm volatile("" ::"v"(F.b[kk][b]));
      }
      return;
    }
#if SPUTNIK_PRIO
    __builtin_amdgcn_s_setprio(1);
#endif
#pragma unroll
    for (int kk = 0; kk < kKK; ++kk)
#pragma unroll
      for (int a = 0; a < kFM; ++a)
#pragma unroll
        for (int b = 0; b < kFN; ++b)
          // Straight outputs compute the tile transposed (D fragment as
          // the MFMA's A operand), so a lane's 4 accumulator values are 4
          // consecutive output columns of one row: the epilogue then packs
          // them into one 8-byte LDS write. Transposed outputs (DDS) keep
          // S as the A operand: 4 consecutive rows = 4 consecutive
          // elements of an output row of C.
          acc[a][b] = kOutT ? MfmaTraits<T>::mfma(F.a[kk][a], F.b[kk][b],
                                                  acc[a][b])
                            : MfmaTraits<T>::mfma(F.b[kk][b], F.a[kk][a],
                                                  acc[a][b]);
#if SPUTNIK_PRIO
    __builtin_amdgcn_s_setprio(0);
#endif
  };

  // Software pipeline over k-steps [first, first + steps) (issue() indices).
  // Ring slot of the i-th step is i % 3. At the top of step i the fragments
  // of i are already in registers (cur); the step
  //   1. waits for its own DMA of step i+1 (counted vmcnt: i+2 stays in
  //      flight) and meets the other waves at a raw s_barrier, after which
  //      step i+1's slot is complete and step i's slot is no longer read;
  //   2. refills step i's slot with the DMA of step i+3;
  //   3. issues the LDS reads of step i+1 into `next` and, without waiting for
  //      them, the MFMAs of step i on `cur`;
  //   4. waits for `next`.
  // DMA therefore has two steps of MFMA time to land and the LDS read latency
  // hides under the MFMAs. The ring is fully drained on return.
  // ---- pair hand-off (see the pair branch below) ---------------------------
  // Partial layout: fragment (a, b) of lane l at pair slot + lane_base +
  // (a*kFN + b) KiB, one 1 KiB wave-instruction each. Hand-off without
  // fences (MI355X_MICROARCH.md, hand-off table row 1): every partial byte is
  // stored and loaded sc1 (L1 bypass, write-through), each storing wave
  // drains vmcnt before a barrier, then ONE lane stores the flag (relaxed,
  // agent scope = sc1) and the consumer polls it with sc1 loads.
  constexpr bool kPairs = kScalarIdx && !kSparseOut && Cfg::kStagger;
  constexpr int kSlotBytes = kBM * kBN * 4;
  constexpr int kSc1 = 16;  // cache-policy bits: sc1
  int pair_id = 0;
  int pair_target = 0;  // blocks per workgroup the pair schedule aims at
  unsigned pair_epoch = p.pair_epoch;
  if constexpr (kPairs) {
    // Captured launch: the epoch word was last written by the previous
    // launch's last workgroup (kernel boundary: the scalar cache starts
    // clean), so a scalar load sees it.
    if (p.pair != 0 && p.pair_sync != nullptr)
      pair_epoch = ((unsigned)scalar_load_int(
                        reinterpret_cast<const int *>(p.pair_sync), 0) &
                    0x7fffffffu) + 1u;
  }
  auto pair_rsrc = [&]() {
    return make_rsrc(reinterpret_cast<const char *>(p.pair_partials));
  };
  auto pair_lane_base = [&]() {
    return pair_id * kSlotBytes + (wave * kFM * kFN * 64 + lane) * 16;
  };
  // Called by every wave right after its MFMAs of the last head step. In a
  // staggered pipeline the lagging half reaches this barrier one barrier
  // later, so the flag is raised by the last wave (a lagging one): after its
  // barrier every wave of both halves has drained its stores.
  auto publish = [&]() {
    if constexpr (kPairs) {
      const __amdgpu_buffer_rsrc_t rp = pair_rsrc();
      const int lb = pair_lane_base();
#pragma unroll
      for (int a = 0; a < kFM; ++a)
#pragma unroll
        for (int b = 0; b < kFN; ++b)
          __builtin_amdgcn_raw_buffer_store_b128(
              __builtin_bit_cast(v4u, acc[a][b]), rp, lb,
              (a * kFN + b) * 1024, kSc1);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();
      if (wave == kNW - 1 && lane == 0 && !p.pair_fault)
        __hip_atomic_store(p.pair_flags + pair_id, pair_epoch,
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      tl(5);
      zero_acc();
    }
  };
  // Consumer side: poll for this launch's epoch, barrier, add the partial
  // (sc1 loads). The flag is never reset: a publish from an earlier launch
  // carries an older epoch, so it can never satisfy this one. Returns false
  // on timeout: the tile is NaN and the event counted in the error word.
  auto collect = [&]() -> bool {
    if constexpr (kPairs) {
      int *ok = scratch + 3;
      if (tid == 0) {
        const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
        bool got;
        while (!(got = __hip_atomic_load(p.pair_flags + pair_id,
                                         __ATOMIC_RELAXED,
                                         __HIP_MEMORY_SCOPE_AGENT) ==
                       pair_epoch) &&
               __builtin_amdgcn_s_memrealtime() - t0 < kPairWaitTicks)
          __builtin_amdgcn_s_sleep(1);
        if (!got)
          __hip_atomic_fetch_add(p.pair_error, 1u, __ATOMIC_RELAXED,
                                 __HIP_MEMORY_SCOPE_AGENT);
        *ok = got ? 1 : 0;
      }
      wait_vmcnt<0>();  // no DMA of the pipeline still lands in the ring
      __syncthreads();
      tl(6);
      const bool got = __builtin_amdgcn_readfirstlane(*ok) != 0;
      if (!got) {
        const float nan = __builtin_nanf("");
#pragma unroll
        for (int a = 0; a < kFM; ++a)
#pragma unroll
          for (int b = 0; b < kFN; ++b) acc[a][b] = f32x4{nan, nan, nan, nan};
        return false;
      }
      // The partial (sc1, as it was stored) comes in by LDS-DMA, each
      // wave's fragments into its own LDS region (above the scratch words):
      // the accumulators leave no registers for loads, and register loads
      // issued a few at a time cost one round trip per few KiB (8.5 us for
      // the 256 KiB tile). Quarters through two buffers, so one quarter is
      // in flight while the previous one is added.
      constexpr int kFrags = kFM * kFN;
      constexpr int kQ = kFrags / 4;  // fragments per quarter
      constexpr int kRegion = 2 * kQ * 1024;
      static_assert(16384 + kNW * kRegion <= kRingBytes && kFrags % 4 == 0,
                    "pair partial staging fits in the ring");
      const __amdgpu_buffer_rsrc_t rp = pair_rsrc();
      const int lb = pair_lane_base();
      char *region = lds + 16384 + wave * kRegion;
      auto fetch = [&](int q) {
        char *buf = region + (q & 1) * (kQ * 1024);
#pragma unroll
        for (int i = 0; i < kQ; ++i)
          dma16<kSc1>(rp, buf + i * 1024, (uint32_t)(lb + (q * kQ + i) * 1024));
      };
      auto add = [&](int q) {
        const f32x4 *m = reinterpret_cast<const f32x4 *>(
                             region + (q & 1) * (kQ * 1024)) + lane;
#pragma unroll
        for (int i = 0; i < kQ; ++i) {
          const int f = q * kQ + i;
          acc[f / kFN][f % kFN] += m[i * 64];
        }
        // Its buffer is refilled next: the reads must have landed.
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      };
      fetch(0);
      fetch(1);
      wait_vmcnt<kQ>();
      add(0);
      fetch(2);
      wait_vmcnt<kQ>();
      add(1);
      fetch(3);
      wait_vmcnt<kQ>();
      add(2);
      wait_vmcnt<0>();
      add(3);
    }
    return true;
  };

  // flush_at > 0: after the MFMAs of step flush_at - 1 the accumulators are
  // published (pair producer) and restarted from zero; the ring keeps
  // streaming.
  // SPUTNIK_EXP & 128: per-segment cycle sums of the k-loop (waves 0 and
  // kNW/2), read after wait_step so no stamp adds an LDS wait in the loop.
  unsigned long long seg_t[7] = {0, 0, 0, 0, 0, 0, 0};
  unsigned long long seg_sum[6] = {0, 0, 0, 0, 0, 0};
#define SEG_STAMP(n)                                          \
  do {                                                        \
    if constexpr ((SPUTNIK_EXP & 128) != 0) {                 \
      __builtin_amdgcn_sched_barrier(0);                      \
      seg_t[n] = __builtin_amdgcn_s_memtime();                \
      __builtin_amdgcn_sched_barrier(0);                      \
    }                                                         \
  } while (0)
#define SEG_ACCUM()                                           \
  do {                                                        \
    if constexpr ((SPUTNIK_EXP & 128) != 0) {                 \
      _Pragma("unroll") for (int q = 0; q < 6; ++q)           \
        seg_sum[q] += (seg_t[q] != 0 && seg_t[q + 1] > seg_t[q]) ? seg_t[q + 1] - seg_t[q] : 0; \
      seg_t[1] = seg_t[2] = seg_t[3] = 0;                     \
    }                                                         \
  } while (0)
  auto pipeline = [&](int first, int steps, int flush_at = -1) {
    if (steps <= 0) return;
    e_end = (first + steps + kStepsPerBlock - 1) / kStepsPerBlock;
    pf_e = -1;
    issue(first, 0);
    if (steps > 1) issue(first + 1, 1);
    if (steps > 2) issue(first + 2, 2);
    if (steps > 2)
      wait_vmcnt<2 * kGroup>();
    else if (steps > 1)
      wait_vmcnt<kGroup>();
    else
      wait_vmcnt<0>();
    __builtin_amdgcn_s_barrier();
    Frags f0, f1;
    read_step(0, f0);
    wait_step(f0);
    // Staggered configs: the lagging half (waves kNW/2..) passes one barrier
    // behind the leading half, and every step has two barriers, B1 before
    // the DMA/read phase and B2 before the MFMA phase, so a lagging wave's
    // B1 is a leading wave's B2: one half streams while the other computes.
    // Ordering (4-slot ring, DMA of step i+3 issued after B1(i)):
    //  - RAW: a wave reads slot i+1 after its B1(i). Leaders wait for their
    //    own DMA of step i+1 before B1(i); laggers wait for theirs before
    //    B2(i-1), which is the leaders' B1(i). So every piece of slot i+1 has
    //    landed before either half reads it.
    //  - WAR: DMA(i+3) refills slot (i+3)%4 = (i-1)%4, last read during step
    //    i-2 and drained (lgkmcnt(0)) before each wave's next barrier, which
    //    precedes both halves' B1(i).
    // Every wave executes the same number of barriers: laggers add one after
    // the prologue, leaders one after the loop.
    const bool lag = Cfg::kStagger && wave >= kNW / 2;
    if constexpr (SPUTNIK_LAG_PRIO != 0) {
      if (lag) __builtin_amdgcn_s_setprio(1);
    }
    if (lag) {
      if (steps > 2)
        wait_vmcnt<kGroup>();
      else
        wait_vmcnt<0>();
      __builtin_amdgcn_s_barrier();
    }
    int slot = 0;  // slot of step i
    auto body = [&](int i, Frags &cur, Frags &next) {
      const int nslot = slot + 1 == kStages ? 0 : slot + 1;
      SEG_STAMP(0);
      if (i + 1 < steps) {
        if (!lag) {
          if (i + 2 < steps)
            wait_vmcnt<kGroup>();
          else
            wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();
        SEG_STAMP(1);
        int dslot = slot + 3;
        if (dslot >= kStages) dslot -= kStages;
        if constexpr (SPUTNIK_READ_FIRST != 0) {
          // Scalar prep first (its scalar-cache wait then finds no LDS read
          // in flight). READ_FIRST 1: every wave reads, then fires its DMA.
          // READ_FIRST 2/3: waves alternate the two orders (by wave bit 0 /
          // bit 1), so while half of the memory-phase waves queue their DMA
          // at the TA the other half's reads are served by the LDS.
          if (i + 3 < steps) prep(first + i + 3);
          const bool rf = SPUTNIK_READ_FIRST == 1 ||
                          (SPUTNIK_READ_FIRST == 2 && (wave & 1) != 0) ||
                          (SPUTNIK_READ_FIRST == 3 && (wave & 2) != 0);
          if (rf) {
            read_step(nslot, next);
            __builtin_amdgcn_sched_barrier(0);
            if (i + 3 < steps) fire(dslot);
          } else {
            if (i + 3 < steps) fire(dslot);
            __builtin_amdgcn_sched_barrier(0);
            read_step(nslot, next);
          }
        } else {
          if (i + 3 < steps) issue(first + i + 3, dslot);
          SEG_STAMP(2);
          read_step(nslot, next);
        }
        SEG_STAMP(3);
      }
      if constexpr (Cfg::kStagger) {
        if (lag) {
          // Own DMA of step i+2 lands before the leaders read it (B1(i+1)).
          if (i + 3 < steps)
            wait_vmcnt<kGroup>();
          else if (i + 2 < steps)
            wait_vmcnt<0>();
        }
        __builtin_amdgcn_s_barrier();
      }
      SEG_STAMP(4);
      mfma_step(cur);
      SEG_STAMP(5);
      if (i + 1 < steps) wait_step(next);
      SEG_STAMP(6);
      SEG_ACCUM();
      if constexpr (kPairs) {
        if (i + 1 == flush_at) {
          publish();
        }
      }
      slot = nslot;
    };
    for (int i = 0; i < steps; i += 2) {
      body(i, f0, f1);
      if (i + 1 < steps) body(i + 1, f1, f0);
    }
    if (Cfg::kStagger && !lag) __builtin_amdgcn_s_barrier();
  };

  // ---- DSD / DDS on the staggered configs: pipeline()'s schedule unrolled
  // by one stored block (kStepsPerBlock = 4 steps = the 4 ring slots), so
  // every ring slot is a compile-time constant, a block's base addresses are
  // resolved once (its index scalar-loaded one block ahead), and the
  // steady-state loop carries no per-step branch beyond the two uniform
  // half-selection branches around the vmcnt waits (the leading and lagging
  // halves differ only there; the ordering argument is pipeline()'s). Two
  // loop copies, one per half, measured 2.4x slower: they spill the
  // accumulators. Entries
  // [e0, e0 + nblk) of the index segments; the pair producer publishes after
  // block flush_blk - 1.
  auto pipeline_blocks = [&](int e0, int nblk, int flush_blk) {
    if (nblk <= 0) return;
    auto entry = [&](int x) {
      return x < idx_split ? idx_base + x : idx_base2 + (x - idx_split);
    };
    int nk = 0, nbk = 0;  // (k-block, storage block) of the next block
    auto load_idx = [&](int e) {
      const int ge = entry(e);
      nk = scalar_load_short(p.s_indices, ge);
      nbk = p.s_block_offsets != nullptr ? scalar_load_int(p.s_block_offsets, ge)
                                         : ge;
    };
    const char *cs = nullptr, *cd = nullptr;  // bases of the block being fed
    auto take_next = [&]() {
      cs = p.s_data + (long long)nbk * (kBlock * kBlock * 2);
      const long long kg = (long long)nk * kBlock;
      cd = kDKC ? p.d_data + (long long)j0 * p.d_ld + kg * 2
                : p.d_data + kg * p.d_ld + (long long)j0 * 2;
    };
    auto fire_sub = [&](int h, int slot) {
      s_base = cs + (kSKC ? h * (kBK * 2) : h * (kBK * 256));
      d_base = cd + (kDKC ? (long long)h * (kBK * 2)
                          : (long long)h * kBK * p.d_ld);
      fire(slot);
    };
    if constexpr (kDenseS) {  // SDD: step s covers k = 32 s ..
      prep(0);
      fire(0);
      prep(1);
      fire(1);
      prep(2);
      fire(2);
    } else {
      load_idx(e0);
      take_next();
      fire_sub(0, 0);
      fire_sub(1, 1);
      fire_sub(2, 2);
      load_idx(e0 + min(1, nblk - 1));  // prefetch block 1
    }
    wait_vmcnt<2 * kGroup>();
    __builtin_amdgcn_s_barrier();
    Frags f0, f1;
    read_step(0, f0);
    wait_step(f0);
    const bool lag = wave >= kNW / 2;
    if constexpr (SPUTNIK_LAG_PRIO != 0) {
      if (lag) __builtin_amdgcn_s_setprio(1);
    }
    if (lag) {
      wait_vmcnt<kGroup>();
      __builtin_amdgcn_s_barrier();
    }
    // Step h of block b (i = 4b + h of s = 4 nblk steps): LAST marks the
    // final block, where pipeline()'s end conditions apply.
    auto step = [&](auto h_c, auto last_c, int b, Frags &cur, Frags &next) {
      const bool L = lag;
      constexpr int H = decltype(h_c)::value;
      constexpr bool LAST = decltype(last_c)::value;
      constexpr bool kHasNext = !(LAST && H == 3);        // i + 1 < s
      SEG_STAMP(0);
      if constexpr (kHasNext) {
        if (!L) {
          if constexpr (LAST && H == 2)
            wait_vmcnt<0>();
          else
            wait_vmcnt<kGroup>();
        }
        __builtin_amdgcn_s_barrier();
        SEG_STAMP(1);
        if constexpr (kDenseS) {
          if constexpr (H == 0 || !LAST) {                  // step i + 3
            prep(4 * b + H + 3);
            fire((H + 3) & 3);
          }
        } else if constexpr (H == 0) {
          fire_sub(3, 3);                                   // step i + 3
        } else if constexpr (!LAST) {
          if constexpr (H == 1) {
            take_next();
            load_idx(e0 + min(b + 2, nblk - 1));            // block b + 2
          }
          fire_sub(H - 1, H - 1);
        }
        SEG_STAMP(2);
        read_step((H + 1) & 3, next);
        SEG_STAMP(3);
      }
      if (L) {
        if constexpr (!LAST || H == 0)
          wait_vmcnt<kGroup>();
        else if constexpr (H == 1)
          wait_vmcnt<0>();
      }
      __builtin_amdgcn_s_barrier();
      SEG_STAMP(4);
      mfma_step(cur);
      SEG_STAMP(5);
      if constexpr (kHasNext) wait_step(next);
      SEG_STAMP(6);
      SEG_ACCUM();
    };
    using I0 = std::integral_constant<int, 0>;
    using I1 = std::integral_constant<int, 1>;
    using I2 = std::integral_constant<int, 2>;
    using I3 = std::integral_constant<int, 3>;
    auto run = [&]() {
      int b = 0;
      for (; b + 1 < nblk; ++b) {
        step(I0{}, std::false_type{}, b, f0, f1);
        step(I1{}, std::false_type{}, b, f1, f0);
        step(I2{}, std::false_type{}, b, f0, f1);
        step(I3{}, std::false_type{}, b, f1, f0);
        if constexpr (kPairs) {
          if (b + 1 == flush_blk) {
            publish();
          }
        }
      }
      step(I0{}, std::true_type{}, b, f0, f1);
      step(I1{}, std::true_type{}, b, f1, f0);
      step(I2{}, std::true_type{}, b, f0, f1);
      step(I3{}, std::true_type{}, b, f1, f0);
      if constexpr (kPairs) {
        if (b + 1 == flush_blk) {
          publish();
        }
      }
    };
    run();
    if (!lag) __builtin_amdgcn_s_barrier();
  };

  // Steps [s_begin, s_end) of sparse block-row `srow` whose entries start at
  // entry0 (entry e covers steps e*kStepsPerBlock ..). The (k-block, storage
  // block) list is staged into LDS in chunks of kIndexChunk entries.
  auto run_sparse = [&](int entry0, int s_begin, int s_end) {
    const bool col_order = p.s_block_offsets != nullptr;
    const int e_begin = s_begin / kStepsPerBlock;
    const int e_end = (s_end + kStepsPerBlock - 1) / kStepsPerBlock;
    for (int cb = e_begin; cb < e_end; cb += kIndexChunk) {
      const int n = min(kIndexChunk, e_end - cb);
      __syncthreads();  // ring, staging and index list no longer read
      for (int e = tid; e < n; e += kThreads) {
        const int ge = entry0 + cb + e;
        idx_kc[e] = p.s_indices[ge];
        idx_blk[e] = col_order ? p.s_block_offsets[ge] : ge;
      }
      __syncthreads();
      const int lo = max(s_begin, cb * kStepsPerBlock);
      const int hi = min(s_end, (cb + n) * kStepsPerBlock);
      cached_e = -1;
      pipeline(lo - cb * kStepsPerBlock, hi - lo);
    }
  };

  // ---- output of one finished tile: fp32 -> T, staged through LDS, 16-byte
  // coalesced stores. The tile is staged in kPasses slices of kPassJ dense
  // columns (j) when it does not fit in the ring at once (128 x 512 tiles).
  // A dense-output tile of an empty block-row is all zeros: store them
  // straight from registers (no LDS staging, no barrier), 16 B per lane.
  auto write_zero_tile = [&]() {
    constexpr int kRows = kOutT ? kBN : kBM;   // rows of the output image
    constexpr int kCols = kOutT ? kBM : kBN;
    constexpr int kChunksPerRow = kCols / 8;
    const uint4 z = {0u, 0u, 0u, 0u};
    for (int id = tid; id < kRows * kChunksPerRow; id += kThreads) {
      const int row = id / kChunksPerRow;
      const int cc = id % kChunksPerRow;
      char *dst;
      if constexpr (kOutT) {
        const int jrow = j0 + row;
        if (jrow >= p.j_limit) continue;
        dst = p.c_data + (long long)jrow * p.c_ld +
              ((long long)srow * kBM + cc * 8) * 2;
      } else {
        const int jcol = j0 + cc * 8;
        if (jcol >= p.j_limit) continue;
        dst = p.c_data + ((long long)srow * kBM + row) * p.c_ld +
              (long long)jcol * 2;
      }
      if constexpr (SPUTNIK_OUT_NT != 0)
        __builtin_nontemporal_store(__builtin_bit_cast(v4u, z), reinterpret_cast<v4u *>(dst));
      else
        *reinterpret_cast<uint4 *>(dst) = z;
    }
  };
  auto write_tile = [&](long long out_block) {
    wait_vmcnt<0>();
    __syncthreads();
    if constexpr (kKS > 1) {
      // Sum the two k-halves: the second wave set parks its fp32
      // accumulators in the upper half of the ring (the staging image below
      // stays under it), the first adds them and stages the tile.
      static_assert(kBM * (kBN * 2 + 16) <= kRingBytes / 2 &&
                        kNW / 2 * kFM * kFN * 1024 <= kRingBytes / 2,
                    "k-split exchange fits beside the staging image");
      f32x4 *xch = reinterpret_cast<f32x4 *>(lds + kRingBytes / 2) +
                   wsub * (kFM * kFN * 64) + lane;
      const bool second = wave >= kNW / 2;
      if (second) {
#pragma unroll
        for (int a = 0; a < kFM; ++a)
#pragma unroll
          for (int b = 0; b < kFN; ++b) xch[(a * kFN + b) * 64] = acc[a][b];
      }
      __syncthreads();
      if (!second) {
#pragma unroll
        for (int a = 0; a < kFM; ++a)
#pragma unroll
          for (int b = 0; b < kFN; ++b) acc[a][b] += xch[(a * kFN + b) * 64];
      }
    }
    constexpr int kStLdNT = kBN * 2 + 16;  // straight staging row
    constexpr int kStLdT = kBM * 2 + 16;   // transposed staging row
    constexpr int kPasses =
        kOutT ? ((kBN * kStLdT + kRingBytes - 1) / kRingBytes)
              : ((kBM * kStLdNT + kRingBytes - 1) / kRingBytes);
    constexpr int kPassJ = kBN / kPasses;
    static_assert(kPassJ % 16 == 0 && kPassJ * kPasses == kBN, "passes");
    constexpr int kOutRows = kOutT ? kPassJ : kBM;  // staging rows per pass
    constexpr int kOutCols = kOutT ? kBM : kPassJ;
    constexpr int kStLd = kOutCols * 2 + 16;  // padded staging row (bytes)
    static_assert(kOutRows * kStLd <= kRingBytes, "staging fits in the ring");
    char *st = lds;
#pragma unroll
    for (int pass = 0; pass < kPasses; ++pass) {
      const int jp0 = pass * kPassJ;
      if (pass > 0) __syncthreads();  // previous slice fully stored
#pragma unroll
      for (int a = 0; a < kFM; ++a) {
        if (kKS > 1 && wave >= kNW / 2) break;  // k split: first set stages
#pragma unroll
        for (int b = 0; b < kFN; ++b) {
          const int jb = col_w + 16 * b;  // wave-uniform
          if (jb < jp0 || jb >= jp0 + kPassJ) continue;
          typedef T t4 __attribute__((ext_vector_type(4)));
          t4 v;
          v[0] = (T)acc[a][b][0];
          v[1] = (T)acc[a][b][1];
          v[2] = (T)acc[a][b][2];
          v[3] = (T)acc[a][b][3];
          if constexpr (kOutT) {
            // lane: rows i..i+3 of column j -> staging row j
            const int i = row_w + 16 * a + 4 * (lane >> 4);
            const int j = jb - jp0 + (lane & 15);
            *reinterpret_cast<t4 *>(st + j * kStLd + i * 2) = v;
          } else {
            // lane: columns j..j+3 of row i (the MFMA computed O^T)
            const int i = row_w + 16 * a + (lane & 15);
            const int j = jb - jp0 + 4 * (lane >> 4);
            *reinterpret_cast<t4 *>(st + i * kStLd + j * 2) = v;
          }
        }
      }
      __syncthreads();
      constexpr int kChunksPerRow = kOutCols / 8;
      constexpr int kChunks = kOutRows * kChunksPerRow;
      for (int id = tid; id < kChunks; id += kThreads) {
        const int row = id / kChunksPerRow;
        const int cc = id % kChunksPerRow;
        const uint4 v =
            *reinterpret_cast<const uint4 *>(st + row * kStLd + cc * 16);
        char *dst;
        if constexpr (kSparseOut && kOutT) {
          // SDS: the tile is the block transposed; staging row j is row j
          // of the output block.
          dst = p.c_data + out_block * (kBlock * kBlock * 2) +
                (jp0 + row) * (kBlock * 2) + cc * 16;
        } else if constexpr (kSparseOut) {
          const int jcol = jp0 + cc * 8;  // column inside the tile
          const int jb = jcol / kBlock;
          if (jb >= grp_count) continue;
          dst = p.c_data + (grp_b0 + jb) * (kBlock * kBlock * 2) +
                row * (kBlock * 2) + (jcol % kBlock) * 2;
        } else if constexpr (kOutT) {
          const int jrow = j0 + jp0 + row;
          if (jrow >= p.j_limit) continue;
          dst = p.c_data + (long long)jrow * p.c_ld +
                ((long long)srow * kBM + cc * 8) * 2;
        } else {
          const int jcol = j0 + jp0 + cc * 8;
          if (jcol >= p.j_limit) continue;
          dst = p.c_data + ((long long)srow * kBM + row) * p.c_ld +
                (long long)jcol * 2;
        }
        if constexpr (kSparseOut ? SPUTNIK_SPARSE_OUT_NT != 0
                                 : SPUTNIK_OUT_NT != 0)
          __builtin_nontemporal_store(__builtin_bit_cast(v4u, v), reinterpret_cast<v4u *>(dst));
        else
          *reinterpret_cast<uint4 *>(dst) = v;
      }
    }
  };

  // Rows of rank ra and rb (rank 0 = most nonzeros, ties by row index), one
  // parallel pass over the offsets staged in LDS (R <= kLptRows). The ring
  // is free again on return.
  // Same ranking for R < 64 rows, barrier-free: every wave computes it on
  // its own, lane r holding row r (n_r by readlane broadcast, R steps), the
  // rank -> length table in a per-wave LDS scratch inside ring slot 3 (on
  // the staggered 4-slot configs, slot 3 is not written before every wave
  // has passed the pipeline's first barrier).
  // Returns (row of rank ra, row of rank rb) and their (first entry, count).
  struct RowPick { int row_a, row_b, e_a, n_a, e_b, n_b; };
  auto rank_rows_wave = [&](int ra, int rb) {
    const int R = p.num_rows;
    const int o0 = lane <= R ? p.s_offsets[lane] : 0;
    const int o1 = __shfl_down(o0, 1, 64);
    const int nr = lane < R ? o1 - o0 : -1;
    if constexpr ((SPUTNIK_EXP & 512) != 0) {
      asm volatile("" ::"v"(nr));
      tl(9);
    }
    // rank = rows before this one in (more blocks first, lower row first)
    // order = the number of larger unique keys n << 6 | (63 - row): the keys
    // go to a per-wave LDS table and every lane compares against all of them
    // (broadcast 16-B reads), which is ~2.5x fewer VALU operations than a
    // readlane per row.
    int *keys = reinterpret_cast<int *>(lds + 3 * kStageBytes + wave * 256);
    int *nbr = reinterpret_cast<int *>(lds + 3 * kStageBytes + 2048 +
                                       wave * 256);
    const bool live = lane < R;
    const int key = live ? (nr << 6) | (63 - lane) : -1;
    keys[lane] = key;
    int4 k4[16];  // all 64 keys (past R: -1, never larger), loads first
#pragma unroll
    for (int j = 0; j < 16; ++j)
      k4[j] = *reinterpret_cast<const int4 *>(keys + 4 * j);
    int rank = 0;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      rank += (k4[j].x > key) + (k4[j].y > key) + (k4[j].z > key) +
              (k4[j].w > key);
    const unsigned long long ba = __ballot(live && rank == ra);
    const unsigned long long bb = __ballot(live && rank == rb);
    RowPick out;
    out.row_a = __builtin_ctzll(ba);
    out.row_b = __builtin_ctzll(bb);
    out.e_a = __builtin_amdgcn_readlane(o0, out.row_a);
    out.n_a = __builtin_amdgcn_readlane(nr, out.row_a);
    out.e_b = __builtin_amdgcn_readlane(o0, out.row_b);
    out.n_b = __builtin_amdgcn_readlane(nr, out.row_b);
    // Pair target: max over i of ceil((n[rank i] + n[rank R-1-i]) / 2).
    if (live) nbr[rank] = nr;
    int v = 0;
    if (lane < (R + 1) / 2) {
      const int j = R - 1 - lane;
      v = lane == j ? nbr[lane] : (nbr[lane] + nbr[j] + 1) / 2;
    }
    // Wave max by ballots, one bit at a time from the top (v < 2^16: a row
    // holds at most 32768 blocks): SALU work, no cross-lane data movement.
    int vmax = 0;
#pragma unroll
    for (int bit = 15; bit >= 0; --bit) {
      const int cand = vmax | (1 << bit);
      if (__ballot(v >= cand) != 0) vmax = cand;
    }
    pair_target = vmax;
    return out;
  };
  auto rank_rows = [&](int ra, int rb) {
    const int R = p.num_rows;
    int *offs = reinterpret_cast<int *>(lds);
    int *n_by_rank = offs + R + 1;
    for (int r = tid; r <= R; r += kThreads) offs[r] = p.s_offsets[r];
    if (tid == 0) scratch[2] = 0;
    __syncthreads();
    for (int r = tid; r < R; r += kThreads) {
      const int nr = offs[r + 1] - offs[r];
      int rank = 0;
      for (int r2 = 0; r2 < R; ++r2) {
        const int n2 = offs[r2 + 1] - offs[r2];
        rank += (n2 > nr) | ((n2 == nr) & (r2 < r));
      }
      n_by_rank[rank] = nr;
      if (rank == ra) scratch[0] = r;
      if (rank == rb) scratch[1] = r;
    }
    __syncthreads();
    // Balanced target of the pair schedule: the largest pair mean (rank i
    // with rank R-1-i, rounded up; the middle row of odd R alone).
    for (int i = tid; i < (R + 1) / 2; i += kThreads) {
      const int j = R - 1 - i;
      const int v = i == j ? n_by_rank[i] : (n_by_rank[i] + n_by_rank[j] + 1) / 2;
      atomicMax(&scratch[2], v);
    }
    __syncthreads();
    const int row_a = __builtin_amdgcn_readfirstlane(scratch[0]);
    const int row_b = __builtin_amdgcn_readfirstlane(scratch[1]);
    pair_target = __builtin_amdgcn_readfirstlane(scratch[2]);
    // No closing barrier: the caller reads the staged offsets and then
    // synchronizes before the ring (which overlaps them) is written.
    return make_int2(row_a, row_b);
  };

  // ---- which work this workgroup does ----------------------------------
  // Every branch below only sets up (srow, j0, the index segments, the step
  // range); the pipeline is then entered from ONE call site per kernel, so
  // it is inlined and the accumulators stay in registers.
  // A persistent workgroup (p.persistent != 0) loops over its tiles here;
  // the body still enters the pipeline from one call site.
  // (Only the non-staggered DSD / DDS configs run persistent: CfgTall.)
  constexpr bool kPersist = !Cfg::kStagger && !kSparseOut && !kSparseD;
  // Split mode: the first num_tiles workgroups only publish partials
  // (recomputed from the launch, not kept live across the pipeline).
  auto split_producer = [&]() {
    return kPairs && Cfg::kSplitMode && (int)blockIdx.x < p.num_tiles;
  };
  int tile_next = blockIdx.x;
  for (int iter = 0;; ++iter) {
    // The tile after this one: fetched now, used after this tile's epilogue,
    // so the atomic's round trip hides under the tile.
    int fetched = 0;
    if constexpr (kPersist) {
      if (p.persistent != 0 && tid == 0)
        fetched = (int)atomicAdd(p.tile_counter, 1ull);
    }
    long long out_block = 0;
    int entry0 = 0, entries = 0;   // sparse S: the row's CSR entry range
    int p_first = 0, p_steps = 0;  // scalar-index pipeline range
    int p_flush = -1;              // pair producer: end of the head segment
    bool do_collect = false;       // pair consumer
    bool use_pairs = false;
    if constexpr (kPairs) use_pairs = p.pair != 0;
    tl(7);
    if (Cfg::kSplitMode) {
      // ==== split mode: two workgroups per tile (GemmParams::pair_split) ===
      // Chunk g of the tile's row is entries [g n / 2, (g+1) n / 2). Grid
      // order [chunk 0 x T] [chunk 1 x T]: every producer precedes its
      // consumer in dispatch order, as in the pair mode below.
      const int nt = p.num_tiles;
      const int g = (int)blockIdx.x >= nt ? 1 : 0;
      const int t = xcd_tile((int)blockIdx.x - g * nt, nt);
      srow = t % p.num_rows;
      j0 = (t / p.num_rows) * kBN;
      const int e_r = scalar_load_int(p.s_offsets, srow);
      const int n_r = scalar_load_int(p.s_offsets, srow + 1) - e_r;
      const int c0 = g * n_r / 2, c1 = (g + 1) * n_r / 2;
      idx_base = e_r;
      p_first = c0 * kStepsPerBlock;
      p_steps = (c1 - c0) * kStepsPerBlock;
      pair_id = t;
      if (g == 0) {
        p_flush = p_steps;
      } else {
        do_collect = true;
      }
    } else if (use_pairs) {
      // ==== pair balancing (one workgroup per CU, #tiles <= #CUs) ==========
      // A tile's length is its block-row's nonzero count, and with one tile
      // per CU the launch ends with the longest row. Within each panel the
      // rows are paired by rank, i <-> R-1-i: the heavy row (rank i, n_h
      // blocks) gives its first hb = (n_h - n_l) / 2 blocks to the light row's
      // workgroup (n_l blocks), which runs them first in the same pipeline,
      // publishes the fp32 partial and then runs its own row; the heavy
      // workgroup runs blocks [hb, n_h) and adds the partial. Both run
      // (n_h + n_l) / 2 blocks, +-1. Grid order: [light x P*(R/2)] [middle row
      // of odd R x P] [heavy x P*(R/2)], so a producer always precedes its
      // consumer in dispatch order and never waits; pairs share an XCD when
      // P*(R/2) + P*(R&1) is a multiple of 8.
      const int R = p.num_rows;
      const int half = R >> 1;
      const int n_light = p.num_jtiles * half;
      const int n_solo = p.num_jtiles * (R & 1);
      const int bid = blockIdx.x;
      int role, panel, pi;  // role 0 light, 1 middle, 2 heavy; pi = pair
      // GemmParams::pair_xcd2 (8 panels, no middle row, an even number of
      // pairs): XCD x = b mod 8 takes panels 2(x/2), 2(x/2)+1 and pairs
      // [(x mod 2) half/2, +half/2) (mode 1), [(1 - x mod 2) half/2, ..)
      // (mode 3) or x mod 2, + 2, .. (mode 2). A bijection on each role's (panel,
      // pair), so producers still precede their consumers.
      // (DSD only: measured there.)
      const bool xcd2 = !kOutT && p.pair_xcd2 != 0 && p.num_jtiles == 8 &&
                        n_solo == 0 && (half & 1) == 0;
      // (modes 1 / 3 by physical XCD: which member of each logical XCD
      // pair is fast depends on the launch's rotation, xcd_rotation)
      const int rot = xcd2 ? xcd_rotation() : 0;
      auto place = [&](int b) {
        if (xcd2) {
          const int x = b & 7, k = b >> 3;
          panel = 2 * (x >> 1) + (k & 1);
          pi = p.pair_xcd2 == 2 ? 2 * (k >> 1) + (x & 1)
             : (fast_xcd(x, rot) ^ (p.pair_xcd2 == 3 ? 1 : 0)) * (half >> 1) + (k >> 1);
        } else {
          const int t = xcd_tile(b, n_light);
          panel = t / half;
          pi = t % half;
        }
      };
      if (bid < n_light) {
        role = 0;
        place(bid);
      } else if (bid < n_light + n_solo) {
        role = 1;
        panel = bid - n_light;
        pi = half;
      } else {
        role = 2;
        place(bid - n_light - n_solo);
      }
      int2 rows;
      int e_h, n_h, e_l, n_l;
      if (Cfg::kStagger && R < 64) {
        const RowPick rp = rank_rows_wave(pi, R - 1 - pi);
        tl(8);
        rows = make_int2(rp.row_a, rp.row_b);
        e_h = rp.e_a; n_h = rp.n_a; e_l = rp.e_b; n_l = rp.n_b;
      } else {
        rows = rank_rows(pi, R - 1 - pi);
        // The offsets are still staged in LDS by rank_rows (the ring is not
        // written before the first DMA): no dependent global round trip.
        const int *offs = reinterpret_cast<const int *>(lds);
        e_h = __builtin_amdgcn_readfirstlane(offs[rows.x]);
        n_h = __builtin_amdgcn_readfirstlane(offs[rows.x + 1]) - e_h;
        e_l = __builtin_amdgcn_readfirstlane(offs[rows.y]);
        n_l = __builtin_amdgcn_readfirstlane(offs[rows.y + 1]) - e_l;
        __syncthreads();  // staged offsets / scratch read by every wave
      }
      // Hand over only what exceeds the panel's balanced target, and nothing
      // under kMinHandoff blocks: a hand-off costs each side about one
      // 256 KiB partial round trip beyond L2 (≈ 1-2 blocks of pipeline).
  #ifndef SPUTNIK_MIN_HANDOFF
  #define SPUTNIK_MIN_HANDOFF 2
  #endif
      constexpr int kMinHandoff = SPUTNIK_MIN_HANDOFF;
      // (Shifting a block from the consumer to the producer to cover the
      // consumer's collect: 50% / 90% +0 / +1%, 10% / 20% -6%; r02, not kept.)
      int hb = role == 1 ? 0 : n_h - pair_target;
      if (hb < kMinHandoff) hb = 0;
      pair_id = panel * half + pi;
      j0 = panel * kBN;
      if (role == 0) {
        srow = rows.y;
        idx_base = e_h;
        idx_split = hb;
        idx_base2 = e_l;
        p_first = 0;
        p_steps = (hb + n_l) * kStepsPerBlock;
        p_flush = hb > 0 ? hb * kStepsPerBlock : -1;
      } else {
        srow = rows.x;
        idx_base = e_h;
        p_first = hb * kStepsPerBlock;
        p_steps = (n_h - hb) * kStepsPerBlock;
        do_collect = hb > 0;
      }
    } else {
      // ==== one output tile per workgroup ===================================
      const int tile = kPersist && p.persistent != 0 ? tile_next
                       : (SPUTNIK_EXP & 8) ? (int)blockIdx.x
                                           : xcd_tile(blockIdx.x, gridDim.x);
      if constexpr (kGroupedSdd) {
        // Tile t = group t of the row-major list of groups, a block-row
        // contributing ceil(n_r / kGrp) groups of consecutive stored blocks.
        // One parallel scan of the group counts over C's offsets (each lane a
        // contiguous run of rows; wave scan by shuffles, then wave totals); the
        // grid is the host's upper bound nb/kGrp + R, so late tiles exit.
        const int R = p.num_rows;
        const int per = (R + kThreads - 1) / kThreads;
        const int r0 = min(R, tid * per), r1 = min(R, r0 + per);
        int local = 0;
        for (int r = r0; r < r1; ++r)
          local += (p.c_offsets[r + 1] - p.c_offsets[r] + kGrp - 1) / kGrp;
        int incl = local;
  #pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          const int v = __shfl_up(incl, d, 64);
          if (lane >= d) incl += v;
        }
        // Row group counts' min / max: when every row has the same count G
        // (block-rows sharing one column set, e.g. the MoE expert-diagonal),
        // tiles run group-major (t -> group t / R, row t % R), so the
        // workgroups that run together on an XCD share one D column slice in
        // its L2 instead of each streaming a different one from HBM.
        int gmin = 0x7fffffff, gmax = 0;
        for (int r = r0; r < r1; ++r) {
          const int g =
              (p.c_offsets[r + 1] - p.c_offsets[r] + kGrp - 1) / kGrp;
          gmin = min(gmin, g);
          gmax = max(gmax, g);
        }
  #pragma unroll
        for (int d = 1; d < 64; d <<= 1) {
          gmin = min(gmin, __shfl_xor(gmin, d, 64));
          gmax = max(gmax, __shfl_xor(gmax, d, 64));
        }
        int *wsum = reinterpret_cast<int *>(lds);
        if (lane == 63) {
          wsum[wave] = incl;
          wsum[kNW + wave] = gmin;
          wsum[2 * kNW + wave] = gmax;
        }
        __syncthreads();
        int before = 0, total = 0;
        for (int w2 = 0; w2 < kNW; ++w2) {
          const int v = wsum[w2];
          before += w2 < wave ? v : 0;
          total += v;
          gmin = min(gmin, wsum[kNW + w2]);
          gmax = max(gmax, wsum[2 * kNW + w2]);
        }
        int start = before + incl - local;
        const bool uniform = gmin == gmax;
        // The grid is an upper bound on the groups: the first `total`
        // workgroups take the groups, XCD-contiguous over `total` (not over
        // the grid), so no XCD's share spills into a second round while the
        // spare workgroups exit (dsd4w.hip, the same mapping).
        const int gt = (SPUTNIK_EXP & 8) ? tile
                       : (int)blockIdx.x < total ? xcd_tile(blockIdx.x, total) : total;
        if (!uniform) {
          for (int r = r0; r < r1; ++r) {
            const int g =
                (p.c_offsets[r + 1] - p.c_offsets[r] + kGrp - 1) / kGrp;
            if (gt >= start && gt < start + g) {
              scratch[0] = r;
              scratch[1] = gt - start;
            }
            start += g;
          }
        }
        __syncthreads();
        if (gt >= total) return;  // whole workgroup: no barrier pending
        int gi;
        if (uniform) {
          srow = gt % R;
          gi = gt / R;
        } else {
          srow = __builtin_amdgcn_readfirstlane(scratch[0]);
          gi = __builtin_amdgcn_readfirstlane(scratch[1]);
        }
        const int b0 = p.c_offsets[srow] + gi * kGrp;
        grp_b0 = b0;
        grp_count = min(kGrp, p.c_offsets[srow + 1] - b0);
        grp_c0 = p.c_indices[b0] * kBlock;
        if (kGrp > 1 && grp_count > 1) grp_c1 = p.c_indices[b0 + 1] * kBlock;
        if (kGrp > 2 && grp_count > 2) grp_c2 = p.c_indices[b0 + 2] * kBlock;
        if (kGrp > 3 && grp_count > 3) grp_c3 = p.c_indices[b0 + 3] * kBlock;
        __syncthreads();  // wsum / scratch reads done before the ring is used
      } else if constexpr (kSparseD) {
        // DSS tile (r, c): op(A)'s row r meets op(B)'s column c. LDS (after
        // the ring): bmap[256] = D storage block of k-block k (or -1), then
        // the intersection as S blocks [256] and D blocks [256], then count.
        const int nc = p.num_jtiles;
        srow = tile / nc;
        const int c = tile % nc;
        j0 = c * kBlock;
        int *bmap = reinterpret_cast<int *>(lds + kRingBytes);
        int *ls = bmap + kDssMaxK;
        int *ld = ls + kDssMaxK;
        int *cnt = ld + kDssMaxK;
        for (int k = tid; k < kDssMaxK; k += kThreads) bmap[k] = -1;
        __syncthreads();
        const int b0 = p.d_offsets[c], b1 = p.d_offsets[c + 1];
        for (int e = b0 + tid; e < b1; e += kThreads)
          bmap[p.d_indices[e]] =
              p.d_block_offsets != nullptr ? p.d_block_offsets[e] : e;
        __syncthreads();
        if (wave == 0) {  // order-preserving compaction of op(A)'s row
          const int a0 = p.s_offsets[srow], a1 = p.s_offsets[srow + 1];
          int pos = 0;
          for (int base = a0; base < a1; base += 64) {
            const int e = base + lane;
            const bool valid = e < a1;
            const int k = valid ? p.s_indices[e] : 0;
            const int bm = valid ? bmap[k] : -1;
            const bool hit = bm >= 0;
            const unsigned long long ball = __ballot(hit);
            if (hit) {
              const int at = pos + __popcll(ball & ((1ull << lane) - 1));
              ls[at] = p.s_block_offsets != nullptr ? p.s_block_offsets[e] : e;
              ld[at] = bm;
            }
            pos += __popcll(ball);
          }
          if (lane == 0) cnt[0] = pos;
        }
        __syncthreads();
        entries = __builtin_amdgcn_readfirstlane(cnt[0]);
      } else if constexpr (kSparseIn) {
        // SSD: block (r, c) of C is row r of op(A) times column panel c of
        // op(B). SDS computes the block transposed: row c of op(B)^T times
        // row panel r of op(A)^T.
        out_block = tile;
        grp_b0 = tile;
        const int r = p.c_row_indices[tile];
        const int c = p.c_indices[tile];
        srow = kOutT ? c : r;
        j0 = (kOutT ? r : c) * kBlock;
        entry0 = p.s_offsets[srow];
        entries = p.s_offsets[srow + 1] - entry0;
      } else if constexpr (kSparseOut) {
        int t = tile;
        if (p.sdd_tail != 0) {
          // tail launch (GemmParams::sdd_tail): workgroup b takes stored
          // block offsets[R0] + b of the rows the grouped launch left
          const int r_tail = sdd_tail_rows<kThreads>(p, reinterpret_cast<int *>(lds), tid);
          t = p.c_offsets[r_tail] + (int)blockIdx.x;
          if (r_tail == p.num_rows || t >= p.c_offsets[p.num_rows]) return;
        }
        out_block = t;
        grp_b0 = t;
        srow = p.c_row_indices[t];
        j0 = p.c_indices[t] * kBlock;
      } else {
        // Longest-processing-time order: within each dense panel, tile t takes
        // the block-row with the t-th most nonzeros (ties by row index), so
        // the workgroups dispatched last are the shortest. Snake (several
        // workgroups per CU): odd panels run ascending, so two workgroups
        // sharing a CU pair a long row with a short one. Rows are ranked in
        // LDS (R <= kLptRows; taller matrices have many more tiles than CUs and
        // keep natural order).
        const int panel = tile / p.num_rows;
        int target = tile % p.num_rows;
        if (Cfg::kWGs > 1 && (panel & 1)) target = p.num_rows - 1 - target;
        j0 = panel * kBN;
        srow = target;
        if (!(SPUTNIK_EXP & 4) && p.num_rows <= kLptRows) {
          if (Cfg::kStagger && p.num_rows < 64) {
            const RowPick rp = rank_rows_wave(target, target);
            srow = rp.row_a;
            entry0 = rp.e_a;
            entries = rp.n_a;
          } else {
            srow = rank_rows(target, target).x;
            const int *offs = reinterpret_cast<const int *>(lds);  // staged
            entry0 = __builtin_amdgcn_readfirstlane(offs[srow]);
            entries = __builtin_amdgcn_readfirstlane(offs[srow + 1]) - entry0;
            __syncthreads();  // staged offsets / scratch read by every wave
          }
        } else if constexpr (kScalarIdx) {
          entry0 = scalar_load_int(p.s_offsets, srow);
          entries = scalar_load_int(p.s_offsets, srow + 1) - entry0;
        } else {
          entry0 = p.s_offsets[srow];
          entries = p.s_offsets[srow + 1] - entry0;
        }
        idx_base = entry0;
        p_first = 0;
        p_steps = entries * kStepsPerBlock;
      }
    }
    setup_d(j0);
    zero_acc();
    tl(1);
    if constexpr (kDenseS) {
      const int nsteps = (p.k_limit + kBK - 1) / kBK;
      // Staggered (grouped) SDD: whole groups of 4 k-steps; steps past K read
      // zeros through the k mask (at most 3, none when K % 128 == 0).
      if constexpr (SPUTNIK_SDD_BLOCK_LOOP != 0 && Cfg::kStagger &&
                    kStages == 4)
        pipeline_blocks(0, (nsteps + 3) / 4, -1);
      else
        pipeline(0, nsteps);
    } else if constexpr (kScalarIdx) {
      // (Both operands k-contiguous, DSD NT / DDS NT: the unrolled loop
      // needs 12 more address registers than it has and spills; those two
      // keep the per-step pipeline.)
      cached_e = -1;
      if constexpr (SPUTNIK_BLOCK_LOOP != 0 && Cfg::kStagger &&
                    kStages == 4 && kStepsPerBlock == 4 && !(kSKC && kDKC))
        pipeline_blocks(p_first / kStepsPerBlock, p_steps / kStepsPerBlock,
                        p_flush > 0 ? p_flush / kStepsPerBlock : -1);
      else
        pipeline(p_first, p_steps, p_flush);
      tl(2);
      if constexpr (kPairs) {
        if (split_producer() && p_steps == 0) publish();  // an empty chunk
        // Both modes hand over exactly one partial: the head [0, p_first)
        // of the consumer's row (pair: the heavy row's first hb blocks;
        // split: the first half).
        if (do_collect) collect();
      }
    } else if constexpr (kSparseD) {
      cached_e = -1;
      pipeline(0, entries * kStepsPerBlock);  // list staged by the setup
    } else {
      run_sparse(entry0, 0, entries * kStepsPerBlock);
    }
    tl(3);
    bool empty = false;
    if constexpr (!kSparseOut) empty = p_steps == 0 && !do_collect;
    if constexpr (!kSparseOut && !kScalarIdx) empty = entries == 0;
    if (split_producer()) {
      // split mode: this chunk's partial is published; the tile is written
      // by its consumer
    } else if (empty) {
      write_zero_tile();
    } else {
      write_tile(out_block);
    }
    if constexpr ((SPUTNIK_EXP & 512) != 0) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      tl(4);
      if (p.debug != nullptr && wave == 0 && lane < 16) {
        // lane i < 7 writes stamp i; then the steps, the role and the row.
        unsigned long long v = 0;
  #pragma unroll
        for (int i = 0; i < 7; ++i) v = lane == i ? tl_stamp[i] : v;
        if (lane == 7)
          v = (unsigned long long)(p_steps ? p_steps : entries * kStepsPerBlock);
        if (lane == 8)
          v = (unsigned long long)(do_collect ? 2 : (p_flush > 0 ? 1 : 0));
        if (lane == 9) v = (unsigned long long)srow;
        if (lane == 10) v = (unsigned long long)pair_id;
        if (lane == 11) v = tl_stamp[7];
        if (lane == 12) v = tl_stamp[8];
        if (lane == 13) v = tl_stamp[9];
      if (lane == 14) v = tl_cycles[0];
      if (lane == 15) v = tl_cycles[1];
        p.debug[blockIdx.x * 16 + lane] = v;
      }
    }
    if constexpr ((SPUTNIK_EXP & 128) != 0) {
      if (p.debug != nullptr && lane == 0 && (wave == 0 || wave == kNW / 2)) {
        unsigned long long *o =
            p.debug + 2048 * 16 + blockIdx.x * 16 + (wave == 0 ? 0 : 8);
  #pragma unroll
        for (int q = 0; q < 6; ++q) o[q] = seg_sum[q];
      }
    }
    if (!kPersist || p.persistent == 0) break;
    // Slot iter & 1: its next write (two tiles on) comes after the barrier
    // that ends the next tile, when every wave has read it.
    if (tid == 0) scratch[iter & 1] = min(p.grid + fetched, p.num_tiles);
    __syncthreads();  // the next tile reuses the ring and the staging image
    tile_next = __builtin_amdgcn_readfirstlane(scratch[iter & 1]);
    if (tile_next >= p.num_tiles) {
      // This workgroup makes no further fetch: arrive; the last arriver
      // (every fetch of the launch is then done) resets the counter pair.
      if (tid == 0) {
        const unsigned long long d = atomicAdd(p.tile_counter + 1, 1ull);
        if (d + 1 == (unsigned long long)p.grid) {
          __hip_atomic_store(p.tile_counter, 0ull, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(p.tile_counter + 1, 0ull, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      break;
    }
  }  // tiles of a persistent workgroup
  if constexpr (kPairs) {
    if (p.pair != 0 && p.pair_sync != nullptr) {
      // Captured launch: arrive; the last arriver advances the epoch word
      // for the next replay and resets the count (GemmParams::pair_sync).
      __syncthreads();
      if (tid == 0) {
        const unsigned d = __hip_atomic_fetch_add(
            p.pair_sync + 1, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (d + 1 == gridDim.x) {
          __hip_atomic_store(p.pair_sync + 1, 0u, __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
          __hip_atomic_store(p.pair_sync, (pair_epoch & 0x7fffffffu),
                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
#undef SEG_STAMP
#undef SEG_ACCUM
}

// Host-side launch of one instantiation (defined in block_gemm.hip).
// grouped: SDD on CfgSddGrouped (params.num_tiles = the grid's upper bound);
// DSD / DDS on CfgTall (params.num_jtiles over CfgTall::kBN).
hipError_t LaunchBlockGemm(int dtype, bool sparse_out, bool s_kc, bool d_kc,
                           bool out_t, bool grouped, const GemmParams &params,
                           hipStream_t stream);
// DSS on CfgBlock: num_tiles = (M/128) x (N/128), num_jtiles = N/128.
hipError_t LaunchBlockGemmDss(int dtype, bool s_kc, bool d_kc,
                              const GemmParams &params, hipStream_t stream);
// SSD (out_t = false) / SDS (out_t = true) on CfgBlock: num_tiles = C's
// nonzero blocks.
hipError_t LaunchBlockGemmSparseIn(int dtype, bool s_kc, bool d_kc, bool out_t,
                                   const GemmParams &params,
                                   hipStream_t stream);

}  // namespace sputnik_amd

#endif  // SPUTNIK_AMD_BLOCK_GEMM_H_
