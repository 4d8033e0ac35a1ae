// sputnik-amd: device metadata builders (see metadata.hip).
#ifndef SPUTNIK_AMD_METADATA_H_
#define SPUTNIK_AMD_METADATA_H_

#include <hip/hip_runtime_api.h>

namespace sputnik_amd {

hipError_t LaunchTransposeMetadata(int block_rows, int block_cols,
                                   const int *offsets, const short *indices,
                                   int *offsets_t, short *indices_t,
                                   int *block_offsets, hipStream_t stream);

hipError_t LaunchRowIndices(int block_rows, const int *offsets,
                            short *row_indices, hipStream_t stream);

}  // namespace sputnik_amd

#endif  // SPUTNIK_AMD_METADATA_H_
