// sputnik-amd: device metadata builders (see metadata.hip).
#ifndef SPUTNIK_AMD_METADATA_H_
#define SPUTNIK_AMD_METADATA_H_

#include <hip/hip_runtime_api.h>

namespace sputnik_amd {

// blocks: stored blocks (offsets[block_rows], from the matrix's nonzeros).
hipError_t LaunchTransposeMetadata(int block_rows, int block_cols, int blocks,
                                   const int *offsets, const short *indices,
                                   int *offsets_t, short *indices_t,
                                   int *block_offsets, hipStream_t stream);

// BitMatrix of a BCSR topology (reference bitmask.cu:7-45): block_rows x
// ceil(block_cols / 64) uint64 words, zeroed and then filled.
hipError_t LaunchBitmask(int block_rows, int block_cols, const int *offsets,
                         const short *indices, unsigned long long *bitmask,
                         hipStream_t stream);

hipError_t LaunchRowIndices(int block_rows, const int *offsets,
                            short *row_indices, hipStream_t stream);

// Block mask (uint8 [block_rows][block_cols], nonzero = present) -> BCSR
// offsets / ascending indices (reference matrix_utils.cu:254-289). `indices`
// must hold the mask's nonzero count (block_rows * block_cols bounds it).
hipError_t LaunchMaskToBcsr(int block_rows, int block_cols,
                            const unsigned char *mask, int *offsets,
                            short *indices, hipStream_t stream);

// MegaBlocks dMoE topology from cumulative padded expert bins.
hipError_t LaunchExpertTopology(const int *padded_bins, int num_experts,
                                int block_rows, int blocks_per_expert,
                                int *offsets, short *indices,
                                hipStream_t stream);

}  // namespace sputnik_amd

#endif  // SPUTNIK_AMD_METADATA_H_
