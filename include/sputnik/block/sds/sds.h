// sputnik-amd: SDS — C_bcsr = op(A_dense) * op(B_bcsr), computed only at the
// nonzero blocks of C. Replaces reference sputnik/block/sds/sds.h:10-22.
#ifndef SPUTNIK_BLOCK_SDS_SDS_H_
#define SPUTNIK_BLOCK_SDS_SDS_H_

#include "sputnik/block/arguments.h"
#include "sputnik/block/dtype.h"

namespace sputnik {
namespace block {

// Requires c.row_indices; a non-transposed B needs its transposed metadata
// (read in column order, as DDS NN/TN), built by Matmul or precomputed for
// MatmulEx.
hipError_t Matmul(const Matrix a, bool transpose_a, const BlockMatrix b,
                  bool transpose_b, BlockMatrix c, hipStream_t stream);

hipError_t MatmulEx(const Matrix a, bool transpose_a, const BlockMatrix b,
                    bool transpose_b, BlockMatrix c, hipStream_t stream);

hipError_t Matmul(const Matrix a, bool transpose_a, const BlockMatrix b,
                  bool transpose_b, BlockMatrix c, DataType dtype,
                  hipStream_t stream);

hipError_t MatmulEx(const Matrix a, bool transpose_a, const BlockMatrix b,
                    bool transpose_b, BlockMatrix c, DataType dtype,
                    hipStream_t stream);

}  // namespace block
}  // namespace sputnik

#endif  // SPUTNIK_BLOCK_SDS_SDS_H_
