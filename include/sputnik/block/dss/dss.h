// sputnik-amd: DSS — dense C = op(A_bcsr) * op(B_bcsr). Replaces reference
// sputnik/block/dss/dss.h:10-22.
#ifndef SPUTNIK_BLOCK_DSS_DSS_H_
#define SPUTNIK_BLOCK_DSS_DSS_H_

#include "sputnik/block/arguments.h"
#include "sputnik/block/dtype.h"

namespace sputnik {
namespace block {

// K <= 32768 (as the reference, dss_*_align8.cu). A transposed A and a
// non-transposed B need their transposed metadata (built by Matmul,
// precomputed for MatmulEx). The reference's bitmask workspaces are accepted
// but not needed (the intersection is built per output tile on the device).
hipError_t Matmul(const BlockMatrix a, bool transpose_a, const BlockMatrix b,
                  bool transpose_b, Matrix c, hipStream_t stream);

hipError_t MatmulEx(const BlockMatrix a, bool transpose_a, const BlockMatrix b,
                    bool transpose_b, Matrix c, hipStream_t stream);

hipError_t Matmul(const BlockMatrix a, bool transpose_a, const BlockMatrix b,
                  bool transpose_b, Matrix c, DataType dtype,
                  hipStream_t stream);

hipError_t MatmulEx(const BlockMatrix a, bool transpose_a, const BlockMatrix b,
                    bool transpose_b, Matrix c, DataType dtype,
                    hipStream_t stream);

}  // namespace block
}  // namespace sputnik

#endif  // SPUTNIK_BLOCK_DSS_DSS_H_
