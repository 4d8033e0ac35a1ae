// sputnik-amd: DDS — dense C = op(A_dense) * op(B_bcsr).
// Replaces reference sputnik/block/dds/dds.h:10-22.
#ifndef SPUTNIK_BLOCK_DDS_DDS_H_
#define SPUTNIK_BLOCK_DDS_DDS_H_

#include "sputnik/block/arguments.h"
#include "sputnik/block/dtype.h"

namespace sputnik {
namespace block {

// NN and TN read `b` in column order and therefore use (and, unless called
// through MatmulEx, build) b's transposed metadata.
hipError_t Matmul(const Matrix a, bool transpose_a, const BlockMatrix b,
                  bool transpose_b, Matrix c, hipStream_t stream);

hipError_t MatmulEx(const Matrix a, bool transpose_a, const BlockMatrix b,
                    bool transpose_b, Matrix c, hipStream_t stream);

hipError_t Matmul(const Matrix a, bool transpose_a, const BlockMatrix b,
                  bool transpose_b, Matrix c, DataType dtype,
                  hipStream_t stream);
hipError_t MatmulEx(const Matrix a, bool transpose_a, const BlockMatrix b,
                    bool transpose_b, Matrix c, DataType dtype,
                    hipStream_t stream);

}  // namespace block
}  // namespace sputnik

#endif  // SPUTNIK_BLOCK_DDS_DDS_H_
