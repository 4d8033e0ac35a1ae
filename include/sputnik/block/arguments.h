// sputnik-amd: operand descriptors of the sputnik::block API, restated for HIP.
//
// Drop-in contract: the structs below keep the exact field
// order, sizes and by-value passing of the reference descriptors so that a
// caller written against the reference headers recompiles unchanged against
// these. Replaces:
//   BlockSize / AsInt / AsBlockSize     reference sputnik/block/arguments.h:13-46
//   BlockMatrix (BCSR descriptor)       reference sputnik/block/arguments.h:48-153
//   Matrix (dense row-major descriptor) reference sputnik/block/arguments.h:155-162
//   MatmulShape / ValidMatmul           reference sputnik/block/arguments.h:164-231
//   Allocate/Free{Transpose,RowIndices}Buffers  arguments.h:233-269
// The only intended difference is the runtime: hipMalloc/hipFree instead of the
// CUDA runtime. Everything here is host-side and header-only.
#ifndef SPUTNIK_BLOCK_ARGUMENTS_H_
#define SPUTNIK_BLOCK_ARGUMENTS_H_

#include <cstddef>
#include <cstdio>
#include <cstdlib>

#include <hip/hip_runtime_api.h>

#include "sputnik/logging.h"

namespace sputnik {
namespace block {

// Block edge length of a BCSR matrix. Only k128 reaches a kernel.
enum class BlockSize {
  kNone = 0,
  k16 = 16,
  k32 = 32,
  k64 = 64,
  k128 = 128,
};

inline int AsInt(BlockSize b) {
  switch (b) {
    case BlockSize::k16:
    case BlockSize::k32:
    case BlockSize::k64:
    case BlockSize::k128:
      return static_cast<int>(b);
    default:
      return 0;
  }
}

// Aborts on an edge length that is not a supported block size, like the
// reference (arguments.h:34-46).
inline BlockSize AsBlockSize(int b) {
  switch (b) {
    case 16: return BlockSize::k16;
    case 32: return BlockSize::k32;
    case 64: return BlockSize::k64;
    case 128: return BlockSize::k128;
    default: break;
  }
  SPUTNIK_LOG(FATAL) << "Invalid block size.";
  return BlockSize::kNone;
}

// Block compressed sparse row matrix.
//
//   rows, cols, nonzeros  — in ELEMENTS (nonzeros = #blocks * b * b).
//   data                  — #blocks blocks of b*b values, block-major; each block
//                           row-major and contiguous at data + i*b*b.
//   offsets               — int32[rows/b + 1], block-row starts, in blocks.
//   indices               — int16[#blocks], block-column of each stored block.
//   offsets_t, indices_t,
//   block_offsets         — metadata of the transposed iteration order
//                           (CSC offsets, block-row per block in column order,
//                           storage index per block in column order).
//   row_indices           — int16[#blocks], block-row of each stored block
//                           (sparse outputs).
//   bitmask               — uint64 bit matrix of the block pattern, filled by
//                           Bitmask() (block/bitmask/bitmask.h); DSS does not
//                           need it here (it intersects rows and columns in
//                           LDS) but reference DSS callers allocate it.
//   create_metadata       — Matmul builds the transposed metadata when true;
//                           MatmulEx clears it so precomputed metadata is used.
struct BlockMatrix {
  int rows, cols, nonzeros;
  BlockSize block_size;

  void *data;
  void *offsets;
  void *indices;

  void *offsets_t;
  void *indices_t;
  void *block_offsets;

  void *row_indices;

  void *bitmask;

  bool create_metadata = true;

  BlockMatrix(int rows_, int cols_, BlockSize block_size_, int nonzeros_,
              void const *data_, void const *offsets_, void const *indices_)
      : rows(rows_), cols(cols_), nonzeros(nonzeros_),
        block_size(block_size_),
        data(const_cast<void *>(data_)),
        offsets(const_cast<void *>(offsets_)),
        indices(const_cast<void *>(indices_)),
        offsets_t(nullptr), indices_t(nullptr), block_offsets(nullptr),
        row_indices(nullptr), bitmask(nullptr) {}

  BlockMatrix(int rows_, int cols_, BlockSize block_size_, int nonzeros_,
              void const *data_, void const *offsets_, void const *indices_,
              void const *row_indices_)
      : BlockMatrix(rows_, cols_, block_size_, nonzeros_, data_, offsets_,
                    indices_) {
    row_indices = const_cast<void *>(row_indices_);
  }

  BlockMatrix(int rows_, int cols_, BlockSize block_size_, int nonzeros_,
              void const *data_, void const *offsets_, void const *indices_,
              void const *offsets_t_, void const *indices_t_,
              void const *block_offsets_)
      : BlockMatrix(rows_, cols_, block_size_, nonzeros_, data_, offsets_,
                    indices_) {
    offsets_t = const_cast<void *>(offsets_t_);
    indices_t = const_cast<void *>(indices_t_);
    block_offsets = const_cast<void *>(block_offsets_);
  }

  BlockMatrix(int rows_, int cols_, BlockSize block_size_, int nonzeros_,
              void const *data_, void const *offsets_, void const *indices_,
              void const *offsets_t_, void const *indices_t_,
              void const *block_offsets_, void const *bitmask_)
      : BlockMatrix(rows_, cols_, block_size_, nonzeros_, data_, offsets_,
                    indices_, offsets_t_, indices_t_, block_offsets_) {
    bitmask = const_cast<void *>(bitmask_);
  }
};

// Dense row-major matrix; the leading dimension follows from the transpose
// flag the operand is used with (see MatmulShape).
struct Matrix {
  int rows, cols;
  void *data;

  Matrix(int rows_, int cols_, void const *data_)
      : rows(rows_), cols(cols_), data(const_cast<void *>(data_)) {}
};

// Problem shape of op(A) * op(B) from the stored operand shapes.
struct MatmulShape {
  int m, n, k, lda, ldb, ldc;

  MatmulShape(int m_, int n_, int k_, bool transpose_a, bool transpose_b)
      : m(m_), n(n_), k(k_) {
    SetLeadingDims(transpose_a, transpose_b);
  }

  template <typename TypeA, typename TypeB>
  MatmulShape(const TypeA a, bool transpose_a, const TypeB b,
              bool transpose_b) {
    m = transpose_a ? a.cols : a.rows;
    k = transpose_a ? a.rows : a.cols;
    n = transpose_b ? b.rows : b.cols;
    SetLeadingDims(transpose_a, transpose_b);
  }

 private:
  void SetLeadingDims(bool transpose_a, bool transpose_b) {
    lda = transpose_a ? m : k;
    ldb = transpose_b ? k : n;
    ldc = n;
  }
};

template <typename TypeA, typename TypeB, typename TypeC>
inline bool ValidMatmul(const TypeA a, bool transpose_a, const TypeB b,
                        bool transpose_b, TypeC c) {
  MatmulShape shape(a, transpose_a, b, transpose_b);
  const int a_m = transpose_a ? a.cols : a.rows;
  const int a_k = transpose_a ? a.rows : a.cols;
  const int b_k = transpose_b ? b.cols : b.rows;
  const int b_n = transpose_b ? b.rows : b.cols;
  return a_m == shape.m && a_k == shape.k && b_k == shape.k &&
         b_n == shape.n && c.rows == shape.m && c.cols == shape.n;
}

#define SPUTNIK_HIP_CALL(expr)                                          \
  do {                                                                  \
    hipError_t sputnik_hip_status_ = (expr);                            \
    if (sputnik_hip_status_ != hipSuccess) {                            \
      std::fprintf(stderr, "HIP error %s at %s:%d\n",                   \
                   hipGetErrorString(sputnik_hip_status_), __FILE__,    \
                   __LINE__);                                           \
      std::abort();                                                     \
    }                                                                   \
  } while (0)

inline int NumBlocks(const BlockMatrix &a) {
  const int b = AsInt(a.block_size);
  return b == 0 ? 0 : a.nonzeros / (b * b);
}

// Caller-owned workspace for the transposed iteration order.
inline void AllocateTransposeBuffers(BlockMatrix &a) {
  const int block_cols = a.cols / AsInt(a.block_size);
  const size_t blocks = static_cast<size_t>(NumBlocks(a));
  SPUTNIK_HIP_CALL(hipMalloc(&a.offsets_t, (block_cols + 1) * sizeof(int)));
  SPUTNIK_HIP_CALL(hipMalloc(&a.indices_t, blocks * sizeof(short)));
  SPUTNIK_HIP_CALL(hipMalloc(&a.block_offsets, blocks * sizeof(int)));
}

inline void FreeTransposeBuffers(BlockMatrix &a) {
  for (void *p : {a.offsets_t, a.indices_t, a.block_offsets}) {
    if (p != nullptr) SPUTNIK_HIP_CALL(hipFree(p));
  }
}

// Caller-owned workspace for the per-block row index of a sparse output.
inline void AllocateRowIndicesBuffer(BlockMatrix &a) {
  const size_t blocks = static_cast<size_t>(NumBlocks(a));
  SPUTNIK_HIP_CALL(hipMalloc(&a.row_indices, blocks * sizeof(short)));
}

inline void FreeRowIndicesBuffer(BlockMatrix &a) {
  if (a.row_indices != nullptr) SPUTNIK_HIP_CALL(hipFree(a.row_indices));
}

}  // namespace block
}  // namespace sputnik

#endif  // SPUTNIK_BLOCK_ARGUMENTS_H_
