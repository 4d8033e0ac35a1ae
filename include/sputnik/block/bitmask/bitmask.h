// sputnik-amd: block bit matrix of a BCSR topology, built on the device and
// stream-ordered. Replaces reference sputnik/block/bitmask/bitmask.h:10-33
// and bitmask.cu:7-45 (a host build between blocking copies). Output is
// bit-identical: the BitMatrix layout of bit_matrix.h.
//
// Orientation follows the reference: when m.offsets_t is set, the bit matrix
// is over m's transposed iteration order (rows = m.cols / b, columns =
// m.rows / b, from offsets_t / indices_t), otherwise over m's rows. The
// library's DSS kernel does not need it (it intersects in LDS); it exists so
// that reference callers of AllocateBitmaskBuffers / Bitmask link and run.
#ifndef SPUTNIK_BLOCK_BITMASK_BITMASK_H_
#define SPUTNIK_BLOCK_BITMASK_BITMASK_H_

#include "sputnik/block/arguments.h"
#include "sputnik/block/bitmask/bit_matrix.h"

namespace sputnik {
namespace block {

// Writes m.bitmask (caller allocated, see AllocateBitmaskBuffers).
hipError_t Bitmask(BlockMatrix m, hipStream_t stream);

// Call after AllocateTransposeBuffers when the transposed orientation is
// wanted (the reference infers the orientation from offsets_t).
inline void AllocateBitmaskBuffers(BlockMatrix &m) {
  const bool trans = m.offsets_t != nullptr;
  const int b = AsInt(m.block_size);
  const int block_rows = (trans ? m.cols : m.rows) / b;
  const int block_cols = (trans ? m.rows : m.cols) / b;
  SPUTNIK_HIP_CALL(
      hipMalloc(&m.bitmask, BitMatrix::SizeInBytes(block_rows, block_cols)));
}

inline void FreeBitmaskBuffers(BlockMatrix &m) {
  if (m.bitmask != nullptr) SPUTNIK_HIP_CALL(hipFree(m.bitmask));
}

}  // namespace block
}  // namespace sputnik

#endif  // SPUTNIK_BLOCK_BITMASK_BITMASK_H_
