// sputnik-amd: per-block row index of a BCSR matrix (device kernel).
// Replaces reference sputnik/block/row_indices/row_indices.h:10.
#ifndef SPUTNIK_BLOCK_ROW_INDICES_ROW_INDICES_H_
#define SPUTNIK_BLOCK_ROW_INDICES_ROW_INDICES_H_

#include "sputnik/block/arguments.h"

namespace sputnik {
namespace block {

// row_indices[k] = m for every stored block k of block-row m.
hipError_t RowIndices(BlockMatrix a, short *row_indices, hipStream_t stream);

}  // namespace block
}  // namespace sputnik

#endif  // SPUTNIK_BLOCK_ROW_INDICES_ROW_INDICES_H_
