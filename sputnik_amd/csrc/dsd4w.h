// sputnik-amd: the 4-wave hand-scheduled DSD NN kernel (dsd4w.hip).
#ifndef SPUTNIK_AMD_DSD4W_H_
#define SPUTNIK_AMD_DSD4W_H_

#include <hip/hip_runtime.h>

#include "block_gemm.h"

namespace sputnik_amd {

// Whether the 4-wave kernel serves this prepared launch: DSD with S
// k-contiguous (A not transposed) and D n-contiguous (B not transposed) or
// k-contiguous (NT: B stored [n][k], N a multiple of 128), or A transposed
// through its column-order metadata (TN, TT),
// straight output, on the one-tile-per-CU 128 x 512 launch (plain or pair
// balanced; not split mode, not persistent, not the tall configuration).
// blocks: stored blocks of the sparse operand; below a mean of
// kDsd4wMinMean blocks per block-row (where pair balancing is off too) the
// 8-wave kernel keeps the launch (not measured against it there).
constexpr int kDsd4wMinMean = 2;
bool Dsd4wApplies(const GemmParams &p, long long blocks, bool s_kc, bool d_kc,
                  bool out_t, bool tall);

// Launches it; p as prepared for the 8-wave kernel (PrepareDsd +
// PreparePairs): the same grid, workspaces and epochs.
// epi: 0 one workgroup-wide staging image copied out after a barrier; 1
// every wave stages and stores its own 128 x 128 block (no barrier); 2 the
// same with the last block specialized (no dummy DMA / reads, conversion
// inside the final step's MFMAs); 3 the per-wave epilogue with the
// k-contiguous image in double slots of 128-B row pieces (gen_dsd4w.py); 4
// the same with one barrier every other step.
hipError_t LaunchDsd4w(int dtype, const GemmParams &p, int epi, bool nt,
                       hipStream_t stream, bool tn = false, bool tt = false);
// The per-wave epilogue: DSD 4096^3 same-process A/B (r04b, us) 8-wave /
// 4-wave workgroup epilogue / per-wave: 50% 63.5 / 61.2 / 60.6, 10% 27.4 /
// 28.4 / 27.1, 30% 43.7 / 45.2 / 43.7, 90% 97.7 / 93.9 / 93.0; the
// specialized last block (2) tied with it (60.8 / 27.2 / 43.7 / 93.1).
// Double slots (3, the default since r04m): 8-wave / per-wave / double-slot
// DSD 50% 63.3 / 59.2 / 58.2, 10% 27.4 / 25.5 / 24.9, 30% 43.3 / 40.7 /
// 40.8, 90% 98.7 / 92.3 / 91.3; DDS 20% 36.0 / 34.6 / 33.0, 50% 67.5 /
// 64.8 / 60.5, 10% 26.5 / 24.2 / 23.8, 90% 107.7 / 104.2 / 96.0.
constexpr int kDsd4wDefaultEpi = 3;

// DDS NN (op(B)^T rows = B's block-columns through its transposed metadata,
// A k-contiguous, transposed output) on the same kernel with the operand
// images swapped (dsd4w.hip kDds), per-wave epilogue; M a multiple of 128.
// DDS NT (op(B)^T rows = B's block-rows, k-contiguous): both images in
// double slots (kDds + kNt). DDS TN (A stored [k][m]): A's k-row slices per
// wave, read transposed (kDds + kTn). DDS TT: both (kDds + kTt).
bool Dds4wApplies(const GemmParams &p, long long blocks, bool s_kc, bool d_kc,
                  bool out_t, bool tall);
hipError_t LaunchDds4w(int dtype, const GemmParams &p, int epi, bool nt,
                       hipStream_t stream, bool tn = false, bool tt = false);

// Grouped SDD NN / NT / TT (dispatch.cpp UseGroupedSdd: up to 4 stored
// blocks of a block-row per workgroup, grid = the group count's upper
// bound), K a multiple of 128: dsd4w.hip kSdd / kNt / kTt.
bool Sdd4wApplies(const GemmParams &p, bool grouped, bool ta, bool tb, long long blocks = -1);
hipError_t LaunchSdd4w(int dtype, const GemmParams &p, bool ta, bool tb, int epi,
                       hipStream_t stream);

}  // namespace sputnik_amd

#endif  // SPUTNIK_AMD_DSD4W_H_
