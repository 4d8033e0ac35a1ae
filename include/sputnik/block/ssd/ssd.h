// sputnik-amd: SSD — C_bcsr = op(A_bcsr) * op(B_dense), computed only at the
// nonzero blocks of C. Replaces reference sputnik/block/ssd/ssd.h:10-22.
#ifndef SPUTNIK_BLOCK_SSD_SSD_H_
#define SPUTNIK_BLOCK_SSD_SSD_H_

#include "sputnik/block/arguments.h"
#include "sputnik/block/dtype.h"

namespace sputnik {
namespace block {

// Requires c.row_indices; a transposed A needs its transposed metadata
// workspaces (built by Matmul, precomputed for MatmulEx), as in the reference
// (ssd_*_tn_align8.cu:78-90).
hipError_t Matmul(const BlockMatrix a, bool transpose_a, const Matrix b,
                  bool transpose_b, BlockMatrix c, hipStream_t stream);

hipError_t MatmulEx(const BlockMatrix a, bool transpose_a, const Matrix b,
                    bool transpose_b, BlockMatrix c, hipStream_t stream);

hipError_t Matmul(const BlockMatrix a, bool transpose_a, const Matrix b,
                  bool transpose_b, BlockMatrix c, DataType dtype,
                  hipStream_t stream);

hipError_t MatmulEx(const BlockMatrix a, bool transpose_a, const Matrix b,
                    bool transpose_b, BlockMatrix c, DataType dtype,
                    hipStream_t stream);

}  // namespace block
}  // namespace sputnik

#endif  // SPUTNIK_BLOCK_SSD_SSD_H_
