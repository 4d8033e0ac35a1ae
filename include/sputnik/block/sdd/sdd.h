// sputnik-amd: SDD — C_bcsr = op(A_dense) * op(B_dense), computed only at the
// nonzero blocks of C. Replaces reference sputnik/block/sdd/sdd.h:10-15.
#ifndef SPUTNIK_BLOCK_SDD_SDD_H_
#define SPUTNIK_BLOCK_SDD_SDD_H_

#include "sputnik/block/arguments.h"
#include "sputnik/block/dtype.h"

namespace sputnik {
namespace block {

// Requires c.row_indices (see RowIndices / AllocateRowIndicesBuffer).
hipError_t Matmul(const Matrix a, bool transpose_a, const Matrix b,
                  bool transpose_b, BlockMatrix c, hipStream_t stream);

hipError_t Matmul(const Matrix a, bool transpose_a, const Matrix b,
                  bool transpose_b, BlockMatrix c, DataType dtype,
                  hipStream_t stream);

}  // namespace block
}  // namespace sputnik

#endif  // SPUTNIK_BLOCK_SDD_SDD_H_
