// sputnik-amd: transposed-iteration metadata of a BCSR matrix, built on the
// device and stream-ordered. Replaces the host proof of concept at reference
// sputnik/block/transpose/transpose.h:10 / transpose.cu:69-125; the output is
// bit-identical (stable order of blocks within a block-column).
#ifndef SPUTNIK_BLOCK_TRANSPOSE_TRANSPOSE_H_
#define SPUTNIK_BLOCK_TRANSPOSE_TRANSPOSE_H_

#include "sputnik/block/arguments.h"

namespace sputnik {
namespace block {

// Writes a.offsets_t, a.indices_t and a.block_offsets (caller allocated, see
// AllocateTransposeBuffers).
hipError_t Transpose(BlockMatrix a, hipStream_t stream);

}  // namespace block
}  // namespace sputnik

#endif  // SPUTNIK_BLOCK_TRANSPOSE_TRANSPOSE_H_
