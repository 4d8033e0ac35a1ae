// sputnik-amd: extern "C" boundary (declared in include/sputnik_amd.h).
//
// Each function converts the plain-C descriptors to the C++ ones (identical
// layout, checked below) and runs the same host path as the C++ API, but
// returns an error code in every case where the reference would abort.
#include <cstddef>
#include <cstring>

#include "api_internal.h"
#include "sputnik/sputnik.h"
#include "metadata.h"
#include "sputnik_amd.h"

using sputnik::block::BlockMatrix;
using sputnik::block::BlockSize;
using sputnik::block::Matrix;

static_assert(sizeof(BlockMatrix) == 88, "BlockMatrix ABI");
static_assert(sizeof(sputnik_block_matrix_t) == 88, "C BlockMatrix ABI");
static_assert(offsetof(BlockMatrix, block_size) == 12, "ABI");
static_assert(offsetof(BlockMatrix, data) == 16, "ABI");
static_assert(offsetof(BlockMatrix, row_indices) == 64, "ABI");
static_assert(offsetof(BlockMatrix, bitmask) == 72, "ABI");
static_assert(offsetof(BlockMatrix, create_metadata) == 80, "ABI");
static_assert(offsetof(sputnik_block_matrix_t, create_metadata) == 80, "ABI");
static_assert(offsetof(sputnik_block_matrix_t, row_indices) == 64, "ABI");
static_assert(sizeof(Matrix) == 16 && sizeof(sputnik_matrix_t) == 16, "ABI");
static_assert(offsetof(Matrix, data) == 8, "ABI");

namespace {

BlockMatrix ToCpp(const sputnik_block_matrix_t *m) {
  BlockMatrix out(m->rows, m->cols, static_cast<BlockSize>(m->block_size),
                  m->nonzeros, m->data, m->offsets, m->indices, m->offsets_t,
                  m->indices_t, m->block_offsets, m->bitmask);
  out.row_indices = m->row_indices;
  out.create_metadata = m->create_metadata != 0;
  return out;
}

Matrix ToCpp(const sputnik_matrix_t *m) {
  return Matrix(m->rows, m->cols, m->data);
}

int Code(hipError_t launch, int status_code) {
  return status_code != 0 ? status_code : static_cast<int>(launch);
}

}  // namespace


extern "C" {

int sputnik_dsd(const sputnik_block_matrix_t *a, int transpose_a,
                const sputnik_matrix_t *b, int transpose_b,
                const sputnik_matrix_t *c, int dtype, void *stream) {
  if (!a || !b || !c) return hipErrorInvalidValue;
  const BlockMatrix ca = ToCpp(a);
  sputnik_amd::Status st;
  const hipError_t e = sputnik_amd::RunDsd(
      ca, transpose_a != 0, ToCpp(b), transpose_b != 0, ToCpp(c), dtype,
      ca.create_metadata, static_cast<hipStream_t>(stream), &st);
  return Code(e, sputnik_amd::StatusCode(st));
}

int sputnik_dsd_ex(const sputnik_block_matrix_t *a, int transpose_a,
                   const sputnik_matrix_t *b, int transpose_b,
                   const sputnik_matrix_t *c, int dtype, void *stream) {
  if (!a || !b || !c) return hipErrorInvalidValue;
  sputnik_amd::Status st;
  const hipError_t e = sputnik_amd::RunDsd(
      ToCpp(a), transpose_a != 0, ToCpp(b), transpose_b != 0, ToCpp(c), dtype,
      false, static_cast<hipStream_t>(stream), &st);
  return Code(e, sputnik_amd::StatusCode(st));
}

int sputnik_dds(const sputnik_matrix_t *a, int transpose_a,
                const sputnik_block_matrix_t *b, int transpose_b,
                const sputnik_matrix_t *c, int dtype, void *stream) {
  if (!a || !b || !c) return hipErrorInvalidValue;
  const BlockMatrix cb = ToCpp(b);
  sputnik_amd::Status st;
  const hipError_t e = sputnik_amd::RunDds(
      ToCpp(a), transpose_a != 0, cb, transpose_b != 0, ToCpp(c), dtype,
      cb.create_metadata, static_cast<hipStream_t>(stream), &st);
  return Code(e, sputnik_amd::StatusCode(st));
}

int sputnik_dds_ex(const sputnik_matrix_t *a, int transpose_a,
                   const sputnik_block_matrix_t *b, int transpose_b,
                   const sputnik_matrix_t *c, int dtype, void *stream) {
  if (!a || !b || !c) return hipErrorInvalidValue;
  sputnik_amd::Status st;
  const hipError_t e = sputnik_amd::RunDds(
      ToCpp(a), transpose_a != 0, ToCpp(b), transpose_b != 0, ToCpp(c), dtype,
      false, static_cast<hipStream_t>(stream), &st);
  return Code(e, sputnik_amd::StatusCode(st));
}

int sputnik_sdd(const sputnik_matrix_t *a, int transpose_a,
                const sputnik_matrix_t *b, int transpose_b,
                const sputnik_block_matrix_t *c, int dtype, void *stream) {
  if (!a || !b || !c) return hipErrorInvalidValue;
  sputnik_amd::Status st;
  const hipError_t e = sputnik_amd::RunSdd(
      ToCpp(a), transpose_a != 0, ToCpp(b), transpose_b != 0, ToCpp(c), dtype,
      static_cast<hipStream_t>(stream), &st);
  return Code(e, sputnik_amd::StatusCode(st));
}

static int SparseInOut(bool ssd, bool ex, const void *a, int ta,
                       const void *b, int tb,
                       const sputnik_block_matrix_t *c, int dtype,
                       void *stream) {
  if (!a || !b || !c) return hipErrorInvalidValue;
  sputnik_amd::Status st;
  hipError_t e;
  if (ssd) {
    BlockMatrix ca = ToCpp(static_cast<const sputnik_block_matrix_t *>(a));
    if (ex) ca.create_metadata = false;
    e = sputnik_amd::RunSsd(ca, ta != 0,
                            ToCpp(static_cast<const sputnik_matrix_t *>(b)),
                            tb != 0, ToCpp(c), dtype, ca.create_metadata,
                            static_cast<hipStream_t>(stream), &st);
  } else {
    BlockMatrix cb = ToCpp(static_cast<const sputnik_block_matrix_t *>(b));
    if (ex) cb.create_metadata = false;
    e = sputnik_amd::RunSds(ToCpp(static_cast<const sputnik_matrix_t *>(a)),
                            ta != 0, cb, tb != 0, ToCpp(c), dtype,
                            cb.create_metadata,
                            static_cast<hipStream_t>(stream), &st);
  }
  return Code(e, sputnik_amd::StatusCode(st));
}

int sputnik_ssd(const sputnik_block_matrix_t *a, int transpose_a,
                const sputnik_matrix_t *b, int transpose_b,
                const sputnik_block_matrix_t *c, int dtype, void *stream) {
  return SparseInOut(true, false, a, transpose_a, b, transpose_b, c, dtype,
                     stream);
}

int sputnik_ssd_ex(const sputnik_block_matrix_t *a, int transpose_a,
                   const sputnik_matrix_t *b, int transpose_b,
                   const sputnik_block_matrix_t *c, int dtype, void *stream) {
  return SparseInOut(true, true, a, transpose_a, b, transpose_b, c, dtype,
                     stream);
}

int sputnik_sds(const sputnik_matrix_t *a, int transpose_a,
                const sputnik_block_matrix_t *b, int transpose_b,
                const sputnik_block_matrix_t *c, int dtype, void *stream) {
  return SparseInOut(false, false, a, transpose_a, b, transpose_b, c, dtype,
                     stream);
}

int sputnik_sds_ex(const sputnik_matrix_t *a, int transpose_a,
                   const sputnik_block_matrix_t *b, int transpose_b,
                   const sputnik_block_matrix_t *c, int dtype, void *stream) {
  return SparseInOut(false, true, a, transpose_a, b, transpose_b, c, dtype,
                     stream);
}

static int DssEntry(bool ex, const sputnik_block_matrix_t *a, int ta,
                    const sputnik_block_matrix_t *b, int tb,
                    const sputnik_matrix_t *c, int dtype, void *stream) {
  if (!a || !b || !c) return hipErrorInvalidValue;
  BlockMatrix ca = ToCpp(a), cb = ToCpp(b);
  if (ex) ca.create_metadata = cb.create_metadata = false;
  sputnik_amd::Status st;
  const hipError_t e = sputnik_amd::RunDss(
      ca, ta != 0, cb, tb != 0, ToCpp(c), dtype, ca.create_metadata,
      cb.create_metadata, static_cast<hipStream_t>(stream), &st);
  return Code(e, sputnik_amd::StatusCode(st));
}

int sputnik_dss(const sputnik_block_matrix_t *a, int transpose_a,
                const sputnik_block_matrix_t *b, int transpose_b,
                const sputnik_matrix_t *c, int dtype, void *stream) {
  return DssEntry(false, a, transpose_a, b, transpose_b, c, dtype, stream);
}

int sputnik_dss_ex(const sputnik_block_matrix_t *a, int transpose_a,
                   const sputnik_block_matrix_t *b, int transpose_b,
                   const sputnik_matrix_t *c, int dtype, void *stream) {
  return DssEntry(true, a, transpose_a, b, transpose_b, c, dtype, stream);
}

int sputnik_row_indices(const sputnik_block_matrix_t *a, int16_t *row_indices,
                        void *stream) {
  if (!a || (!row_indices && a->nonzeros > 0)) return hipErrorInvalidValue;
  return sputnik::block::RowIndices(ToCpp(a), row_indices,
                                    static_cast<hipStream_t>(stream));
}

int sputnik_transpose(const sputnik_block_matrix_t *a, void *stream) {
  // A matrix without nonzero blocks has empty (possibly null) per-block
  // workspaces; only offsets_t must exist.
  if (!a || !a->offsets_t || !a->offsets) return hipErrorInvalidValue;
  if (a->nonzeros > 0 && (!a->indices_t || !a->block_offsets || !a->indices))
    return hipErrorInvalidValue;
  if (a->block_size != 128 && a->block_size != 64 && a->block_size != 32 &&
      a->block_size != 16)
    return hipErrorNotSupported;
  return sputnik::block::Transpose(ToCpp(a), static_cast<hipStream_t>(stream));
}

int sputnik_bitmask(const sputnik_block_matrix_t *m, void *stream) {
  if (!m || !m->bitmask) return hipErrorInvalidValue;
  const bool trans = m->offsets_t != nullptr;
  if ((trans ? !m->offsets_t : !m->offsets) ||
      (m->nonzeros > 0 && !(trans ? m->indices_t : m->indices)))
    return hipErrorInvalidValue;
  if (m->block_size != 128 && m->block_size != 64 && m->block_size != 32 &&
      m->block_size != 16)
    return hipErrorNotSupported;
  return sputnik::block::Bitmask(ToCpp(m), static_cast<hipStream_t>(stream));
}

size_t sputnik_bitmask_bytes(const sputnik_block_matrix_t *m) {
  if (!m) return 0;
  const int b = m->block_size;
  if (b != 128 && b != 64 && b != 32 && b != 16) return 0;
  const bool trans = m->offsets_t != nullptr;
  return sputnik::block::BitMatrix::SizeInBytes(
      (trans ? m->cols : m->rows) / b, (trans ? m->rows : m->cols) / b);
}

int sputnik_mask_to_bcsr(const uint8_t *mask, int block_rows, int block_cols,
                         int32_t *offsets, int16_t *indices, void *stream) {
  if (!offsets || (block_rows > 0 && block_cols > 0 && (!mask || !indices)))
    return hipErrorInvalidValue;
  return sputnik_amd::LaunchMaskToBcsr(block_rows, block_cols, mask, offsets,
                                       indices,
                                       static_cast<hipStream_t>(stream));
}

int sputnik_expert_topology(const int32_t *padded_bins, int num_experts,
                            int block_rows, int blocks_per_expert,
                            int32_t *offsets, int16_t *indices, void *stream) {
  if (!padded_bins || !offsets || (block_rows > 0 && !indices))
    return hipErrorInvalidValue;
  return sputnik_amd::LaunchExpertTopology(
      padded_bins, num_experts, block_rows, blocks_per_expert, offsets,
      indices, static_cast<hipStream_t>(stream));
}

int sputnik_can_implement(int op, const void *a, int transpose_a,
                          const void *b, int transpose_b, const void *c) {
  return sputnik_amd::CanImplement(op, a, transpose_a != 0, b,
                                   transpose_b != 0, c)
             ? 1
             : 0;
}

int sputnik_sdd_plan(const sputnik_matrix_t *a, int transpose_a,
                     const sputnik_matrix_t *b, int transpose_b,
                     const sputnik_block_matrix_t *c) {
  if (!a || !b || !c) return -1;
  const Matrix ca = ToCpp(a), cb = ToCpp(b);
  const BlockMatrix cc = ToCpp(c);
  return sputnik_amd::SddPlan(&ca, transpose_a != 0, &cb, transpose_b != 0,
                              &cc);
}

int sputnik_sdd_kernel(const sputnik_matrix_t *a, int transpose_a,
                       const sputnik_matrix_t *b, int transpose_b,
                       const sputnik_block_matrix_t *c) {
  if (!a || !b || !c) return -1;
  const Matrix ca = ToCpp(a), cb = ToCpp(b);
  const BlockMatrix cc = ToCpp(c);
  return sputnik_amd::SddKernel(&ca, transpose_a != 0, &cb, transpose_b != 0,
                                &cc);
}

int sputnik_dds_plan(const sputnik_matrix_t *a, int transpose_a,
                     const sputnik_block_matrix_t *b, int transpose_b,
                     const sputnik_matrix_t *c, hipStream_t stream) {
  if (!a || !b || !c) return -1;
  const Matrix ca = ToCpp(a), cc = ToCpp(c);
  const BlockMatrix cb = ToCpp(b);
  return sputnik_amd::DdsPlan(&ca, transpose_a != 0, &cb, transpose_b != 0, &cc,
                              stream);
}

int sputnik_dsd_plan(const sputnik_block_matrix_t *a, int transpose_a,
                     const sputnik_matrix_t *b, int transpose_b,
                     const sputnik_matrix_t *c, hipStream_t stream) {
  if (!a || !b || !c) return -1;
  const BlockMatrix ca = ToCpp(a);
  const Matrix cb = ToCpp(b), cc = ToCpp(c);
  return sputnik_amd::DsdPlan(&ca, transpose_a != 0, &cb, transpose_b != 0, &cc,
                              stream);
}

int sputnik_pair_errors(void) { return sputnik_amd::PairErrors(); }

void sputnik_debug_pair_fault(int on) { sputnik_amd::SetPairFault(on); }

int sputnik_capture_workspaces(void) {
  return sputnik_amd::CaptureWorkspaces();
}

int sputnik_select_dsd_kernel(int four_wave) {
  return sputnik_amd::SelectDsdKernel(four_wave);
}

int sputnik_tuning_get(const char *name) { return sputnik_amd::TuningGet(name); }

int sputnik_tuning_set(const char *name, int value) {
  return sputnik_amd::TuningSet(name, value);
}

size_t sputnik_abi_block_matrix_size(void) { return sizeof(BlockMatrix); }

size_t sputnik_abi_block_matrix_offset(int field) {
  switch (field) {
    case 0: return offsetof(BlockMatrix, rows);
    case 1: return offsetof(BlockMatrix, cols);
    case 2: return offsetof(BlockMatrix, nonzeros);
    case 3: return offsetof(BlockMatrix, block_size);
    case 4: return offsetof(BlockMatrix, data);
    case 5: return offsetof(BlockMatrix, offsets);
    case 6: return offsetof(BlockMatrix, indices);
    case 7: return offsetof(BlockMatrix, offsets_t);
    case 8: return offsetof(BlockMatrix, indices_t);
    case 9: return offsetof(BlockMatrix, block_offsets);
    case 10: return offsetof(BlockMatrix, row_indices);
    case 11: return offsetof(BlockMatrix, bitmask);
    case 12: return offsetof(BlockMatrix, create_metadata);
    default: return (size_t)-1;
  }
}

size_t sputnik_abi_matrix_size(void) { return sizeof(Matrix); }

#ifndef SPUTNIK_BUILD_HASH
#define SPUTNIK_BUILD_HASH "unknown"
#endif
const char *sputnik_version(void) { return "sputnik-amd 0.2 (gfx950)"; }
const char *sputnik_build_hash(void) { return SPUTNIK_BUILD_HASH; }

}  // extern "C"
