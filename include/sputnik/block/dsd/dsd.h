// sputnik-amd: DSD — dense C = op(A_bcsr) * op(B_dense).
// Replaces reference sputnik/block/dsd/dsd.h:10-22 (cudaError_t/cudaStream_t ->
// hipError_t/hipStream_t; otherwise identical overloads).
#ifndef SPUTNIK_BLOCK_DSD_DSD_H_
#define SPUTNIK_BLOCK_DSD_DSD_H_

#include "sputnik/block/arguments.h"
#include "sputnik/block/dtype.h"

namespace sputnik {
namespace block {

// fp16 in, fp32 accumulate, fp16 out. Builds transposed metadata of `a` on
// the device when transpose_a (a.create_metadata == true).
hipError_t Matmul(const BlockMatrix a, bool transpose_a, const Matrix b,
                  bool transpose_b, Matrix c, hipStream_t stream);

// Same, but uses the transposed metadata already held in `a`.
hipError_t MatmulEx(const BlockMatrix a, bool transpose_a, const Matrix b,
                    bool transpose_b, Matrix c, hipStream_t stream);

// Element-type–explicit forms (bf16 is an extension over the reference).
hipError_t Matmul(const BlockMatrix a, bool transpose_a, const Matrix b,
                  bool transpose_b, Matrix c, DataType dtype,
                  hipStream_t stream);
hipError_t MatmulEx(const BlockMatrix a, bool transpose_a, const Matrix b,
                    bool transpose_b, Matrix c, DataType dtype,
                    hipStream_t stream);

}  // namespace block
}  // namespace sputnik

#endif  // SPUTNIK_BLOCK_DSD_DSD_H_
