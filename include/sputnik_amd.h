/* sputnik-amd C-ABI: the FFI boundary of the block-sparse matmul hot path.
 *
 * Every entry point is extern "C", takes plain structs/pointers/ints and a
 * hipStream_t (passed as void*), and returns a hipError_t value as int
 * (0 == hipSuccess). No torch or C++ types cross this boundary. These are the
 * symbols a ctypes / cgo / JNI binding of the reference's sputnik::block API
 * would bind; INTEGRATION.md shows the bindings.
 *
 * Struct layouts are byte-identical to the C++ descriptors in
 * include/sputnik/block/arguments.h (reference sputnik/block/arguments.h:48-162):
 *   sputnik_block_matrix_t: 88 bytes, fields at 0,4,8,12,16,24,...,72,80
 *   sputnik_matrix_t:       16 bytes, fields at 0,4,8
 *
 * Error behaviour: where the reference aborts (missing transposed-metadata or
 * row-index workspace: dsd_..._tn_align8.cu:73-75, sdd_..._nn_align8.cu:75;
 * no compatible kernel: dsd/cutlass/dsd.cu:68-73) these functions return
 * hipErrorInvalidValue (1) instead; unsupported shapes/block sizes return
 * hipErrorNotSupported (801) exactly as the reference does (dsd.cu:16,
 * block_gemm.h:728-745).
 */
#ifndef SPUTNIK_AMD_H_
#define SPUTNIK_AMD_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct sputnik_block_matrix {
  int32_t rows;        /* elements */
  int32_t cols;        /* elements */
  int32_t nonzeros;    /* elements = #blocks * block_size^2 */
  int32_t block_size;  /* 16/32/64/128; only 128 is accepted by the ops */
  void *data;          /* #blocks * bs * bs values, block-major, row-major blocks */
  void *offsets;       /* int32[rows/bs + 1] (in blocks) */
  void *indices;       /* int16[#blocks] block-column */
  void *offsets_t;     /* int32[cols/bs + 1] */
  void *indices_t;     /* int16[#blocks] */
  void *block_offsets; /* int32[#blocks] */
  void *row_indices;   /* int16[#blocks] */
  void *bitmask;       /* uint64 BitMatrix words (sputnik_bitmask) */
  uint8_t create_metadata; /* C++ bool */
} sputnik_block_matrix_t;

typedef struct sputnik_matrix {
  int32_t rows;
  int32_t cols;
  void *data;
} sputnik_matrix_t;

enum {
  SPUTNIK_DTYPE_F16 = 0,
  SPUTNIK_DTYPE_BF16 = 1,
};

/* ---- DSD: C = op(A_bcsr) * op(B)   (reference sputnik/block/dsd/dsd.h:10-22) */
int sputnik_dsd(const sputnik_block_matrix_t *a, int transpose_a,
                const sputnik_matrix_t *b, int transpose_b,
                const sputnik_matrix_t *c, int dtype, void *stream);
/* MatmulEx: uses a's precomputed transposed metadata (create_metadata=false). */
int sputnik_dsd_ex(const sputnik_block_matrix_t *a, int transpose_a,
                   const sputnik_matrix_t *b, int transpose_b,
                   const sputnik_matrix_t *c, int dtype, void *stream);

/* ---- DDS: C = op(A) * op(B_bcsr)   (reference sputnik/block/dds/dds.h:10-22) */
int sputnik_dds(const sputnik_matrix_t *a, int transpose_a,
                const sputnik_block_matrix_t *b, int transpose_b,
                const sputnik_matrix_t *c, int dtype, void *stream);
int sputnik_dds_ex(const sputnik_matrix_t *a, int transpose_a,
                   const sputnik_block_matrix_t *b, int transpose_b,
                   const sputnik_matrix_t *c, int dtype, void *stream);

/* ---- SDD: C_bcsr = op(A) * op(B) at C's nonzero blocks
 *      (reference sputnik/block/sdd/sdd.h:10-15; needs c->row_indices) */
int sputnik_sdd(const sputnik_matrix_t *a, int transpose_a,
                const sputnik_matrix_t *b, int transpose_b,
                const sputnik_block_matrix_t *c, int dtype, void *stream);

/* ---- SSD: C_bcsr = op(A_bcsr) * op(B) at C's nonzero blocks
 *      (reference sputnik/block/ssd/ssd.h:10-22; needs c->row_indices, and
 *      a's transposed metadata when transpose_a) */
int sputnik_ssd(const sputnik_block_matrix_t *a, int transpose_a,
                const sputnik_matrix_t *b, int transpose_b,
                const sputnik_block_matrix_t *c, int dtype, void *stream);
int sputnik_ssd_ex(const sputnik_block_matrix_t *a, int transpose_a,
                   const sputnik_matrix_t *b, int transpose_b,
                   const sputnik_block_matrix_t *c, int dtype, void *stream);

/* ---- SDS: C_bcsr = op(A) * op(B_bcsr) at C's nonzero blocks
 *      (reference sputnik/block/sds/sds.h:10-22; needs c->row_indices, and
 *      b's transposed metadata when !transpose_b) */
int sputnik_sds(const sputnik_matrix_t *a, int transpose_a,
                const sputnik_block_matrix_t *b, int transpose_b,
                const sputnik_block_matrix_t *c, int dtype, void *stream);
int sputnik_sds_ex(const sputnik_matrix_t *a, int transpose_a,
                   const sputnik_block_matrix_t *b, int transpose_b,
                   const sputnik_block_matrix_t *c, int dtype, void *stream);

/* ---- DSS: C = op(A_bcsr) * op(B_bcsr), dense
 *      (reference sputnik/block/dss/dss.h:10-22; K <= 32768; a's transposed
 *      metadata when transpose_a, b's when !transpose_b; no bitmask needed) */
int sputnik_dss(const sputnik_block_matrix_t *a, int transpose_a,
                const sputnik_block_matrix_t *b, int transpose_b,
                const sputnik_matrix_t *c, int dtype, void *stream);
int sputnik_dss_ex(const sputnik_block_matrix_t *a, int transpose_a,
                   const sputnik_block_matrix_t *b, int transpose_b,
                   const sputnik_matrix_t *c, int dtype, void *stream);

/* ---- Metadata builders */
/* reference sputnik/block/row_indices/row_indices.h:10 */
int sputnik_row_indices(const sputnik_block_matrix_t *a, int16_t *row_indices,
                        void *stream);
/* reference sputnik/block/transpose/transpose.h:10 (device, bit-identical) */
int sputnik_transpose(const sputnik_block_matrix_t *a, void *stream);

/* reference sputnik/block/bitmask/bitmask.h:10 (device, bit-identical
 * BitMatrix layout: rows of ceil(cols/64) uint64 words). Orientation as the
 * reference: over the transposed order when m->offsets_t is set. */
int sputnik_bitmask(const sputnik_block_matrix_t *m, void *stream);
/* Bytes of m's bitmask workspace (reference AllocateBitmaskBuffers,
 * bitmask.h:16-23; host-only). */
size_t sputnik_bitmask_bytes(const sputnik_block_matrix_t *m);

/* ---- Device topology builders (no host round trip) */
/* Block mask (uint8 [block_rows][block_cols] row-major, nonzero = present)
 * -> BCSR offsets int32[block_rows+1] and ascending int16 indices, the
 * reference's mask -> CSR scan (sputnik/matrix_utils.cu:254-289, pad_rows_to
 * = 1). `indices` must hold the mask's nonzero count (block_rows*block_cols
 * bounds it); block_cols <= 32768. */
int sputnik_mask_to_bcsr(const uint8_t *mask, int block_rows, int block_cols,
                         int32_t *offsets, int16_t *indices, void *stream);
/* MegaBlocks dMoE topology: padded_bins int32[num_experts] = cumulative
 * per-expert token counts, each padded to a multiple of 128. Block-row r
 * belongs to expert e = #{e : padded_bins[e] <= 128 r} (clamped to the last
 * expert) and holds block-columns [e*blocks_per_expert, (e+1)*...).
 * offsets int32[block_rows+1], indices int16[block_rows*blocks_per_expert]. */
int sputnik_expert_topology(const int32_t *padded_bins, int num_experts,
                            int block_rows, int blocks_per_expert,
                            int32_t *offsets, int16_t *indices, void *stream);

/* ---- Host-only queries (no GPU work; safe without a device) */
/* 1 when the reference would accept the problem (same rules as
 * can_launch_* + ValidMatmul), 0 otherwise. op: 0=DSD 1=DDS 2=SDD. */
int sputnik_can_implement(int op, const void *a, int transpose_a,
                          const void *b, int transpose_b, const void *c);
/* sizeof / offsetof of the descriptors, for ABI checks by bindings. */
size_t sputnik_abi_block_matrix_size(void);
size_t sputnik_abi_block_matrix_offset(int field);
size_t sputnik_abi_matrix_size(void);
const char *sputnik_version(void);
/* Hash of the sources the library was built from (bench.py compares it
 * with the tree it runs in). */
const char *sputnik_build_hash(void);

/* ---- Diagnostics (need a device) */
/* SDD tile plan: 1 = grouped 128x512 tiles (>= 4 blocks per CU), 2 = the
 * grouped tiles with each group's K split over 2-8 workgroups (SDD NN, few
 * groups: one workgroup per CU), 0 = one k-split 128x128 block per
 * workgroup, -1 = the problem is rejected. (Decides as a launch on the null
 * stream would, allocating nothing.) */
int sputnik_sdd_plan(const sputnik_matrix_t *a, int transpose_a,
                     const sputnik_matrix_t *b, int transpose_b,
                     const sputnik_block_matrix_t *c);
/* The SDD kernel behind that plan: 0 = the 8-wave k-split block tile,
 * 1 = grouped tiles on the 8-wave kernel, 2 = the 4-wave K-split, 3 =
 * grouped tiles on the 4-wave kernel, 4 = (NT / TT over a B past the
 * MALL) B transposed into a library buffer, then grouped tiles on the
 * 4-wave kernel (eager launches; a stream being captured keeps 3), -1 =
 * rejected. */
int sputnik_sdd_kernel(const sputnik_matrix_t *a, int transpose_a,
                       const sputnik_matrix_t *b, int transpose_b,
                       const sputnik_block_matrix_t *c);
/* DDS kernel plan of a problem launched on `stream` (no launch, nothing
 * allocated): 0 = the 8-wave 128x512 tile, 1 = the 4-wave kernel, 2 = the
 * tall configuration, 3 = split mode (8-wave), -1 = rejected. */
int sputnik_dds_plan(const sputnik_matrix_t *a, int transpose_a,
                     const sputnik_block_matrix_t *b, int transpose_b,
                     const sputnik_matrix_t *c, hipStream_t stream);
/* DSD kernel plan of a problem launched on `stream` (no launch; makes the
 * launch's workspace decisions): 0 = the 8-wave 128x512 tile, 1 = the
 * 4-wave hand-scheduled kernel, 2 = the tall configuration, 3 = split mode,
 * 4 = the tall pipeline (4-wave, persistent, NN), -1 = the problem is
 * rejected. */
int sputnik_dsd_plan(const sputnik_block_matrix_t *a, int transpose_a,
                     const sputnik_matrix_t *b, int transpose_b,
                     const sputnik_matrix_t *c, hipStream_t stream);
/* Number of pair hand-offs on the current device whose consumer workgroup
 * timed out waiting for its partial (a bounded 0.2 s wait) since the last
 * call; such a consumer's output tile is written as NaN, never as a partial
 * sum. Callers that share the GPU with other work can poll this after a
 * launch to detect the (otherwise unobserved) event. Clears the counts.
 * Synchronizes the device. -1 on a HIP error. */
int sputnik_pair_errors(void);
/* Workspaces made for launches captured into graphs on the current device
 * (pair-balancing workspaces + persistent tile counters). A captured launch
 * gets one per (capture, capturing stream). Once the captured graph and
 * every executable made from it are destroyed, its workspace is re-used by
 * the next capture that needs one, and this call frees the ones still
 * unused (the only place the library frees them: no free ever runs inside
 * a launch). A graph must not be replayed concurrently with a second
 * instantiation of the same capture. Host-only query. */
int sputnik_capture_workspaces(void);

/* ---- Test hooks and tuning knobs: UNSUPPORTED.
 * For the library's own tests and same-process A/B experiments; a correct
 * caller never needs them, names and ranges may change between versions,
 * and every setting is process-wide. */
/* Test hook: when on, pair producers never publish (forces the timeout).
 * Same as sputnik_tuning_set("pair_fault", on). */
void sputnik_debug_pair_fault(int on);
/* Kernel choice for DSD / DDS (every transpose) and the grouped SDD: 1 =
 * the 4-wave hand-scheduled kernel where it applies and pays (the default),
 * 2..7 = wherever it applies, whatever the density, with the DSD NN variant
 * kEpi = mode - 2 (0 workgroup epilogue, 1 per-wave, 2 per-wave +
 * specialized last block, 3 double slots, 4 double slots + barrier every
 * other step + interleaved copy-out, 5 double slots + interleaved copy-out;
 * DDS NN runs kEpi 1 for modes 2-4 and kEpi 3 for 5-7, the grouped SDD the
 * barrier-every-other-step variant for mode 6 and double slots otherwise,
 * the transposed DSD / DDS launches the one variant they have), 0 = the
 * 8-wave kernel everywhere, -1 = query only. Returns the previous choice.
 * Same as the knob "dsd4w". */
int sputnik_select_dsd_kernel(int four_wave);
/* Tuning knobs, each initialised from its environment variable
 * SPUTNIK_AMD_<NAME> (upper case) or its default: "pairs" (1), "pair_xcd2"
 * (3), "split" (1), "split_min_bn" (128), "dsd4w" (1), "grouped_sdd" (1),
 * "grouped_min_per_cu" (4), "tall" (1), "tall_persistent" (1), "dds_xcd2"
 * (3), "sdd4w_max_ld" (16384), "pair_fault" (0), "sdd_ksplit" (1: off;
 * 2-8 the most K-split chunks -- its chunks wait on each other, so only
 * where the launch has the device to itself),
 * "sdd_ksplit_min_k" (6144), "sdd_order" (1),
 * "tall4w" (1: the tall DSD NN pipeline), "tall_flush_w" (4: a tile
 * store's weight in quarter blocks for the pipeline's work split),
 * "tall_odd_share" (120: an odd XCD's workgroup share in percent of an even
 * one's). An environment value that does not parse or is out of range
 * means the default. get returns the value,
 * set the previous value; both return INT_MIN for an unknown name, set also
 * for a value out of the knob's range (nothing changes then). */
int sputnik_tuning_get(const char *name);
int sputnik_tuning_set(const char *name, int value);

#ifdef __cplusplus
}  /* extern "C" */
#endif

#endif  /* SPUTNIK_AMD_H_ */
