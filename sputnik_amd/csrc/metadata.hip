// sputnik-amd: BCSR metadata builders on the device, stream-ordered.
//
// Transpose: replaces the host proof of concept of reference
// sputnik/block/transpose/transpose.cu:69-125 (two blocking D2H copies, a host
// std::stable_sort and three H2D copies per call). Output is bit-identical:
//   offsets_t     = [0] + cumsum(bincount(indices, cols/b))      (:103-104)
//   indices_t[j]  = block-row of the j-th block in stable column order (:93)
//   block_offsets = the stable argsort itself                      (:99-100)
// Stability: blocks of one column keep storage order. Storage order is
// block-row order, and a valid BCSR row holds each column at most once, so the
// rank of a block inside its column equals the number of earlier block-rows
// that hold that column. The kernel walks block-rows in order and hands out
// positions from per-column cursors in LDS, one block-row per step; within a
// step every block touches a different cursor, so no atomics are needed.
//
// RowIndices: replaces reference sputnik/block/row_indices/row_indices.cu:7-36
// (row_indices[k] = m for k in [offsets[m], offsets[m+1])).
//
// MaskToBcsr / ExpertTopology: device topology builders,
// so a training step builds its BCSR without host work.
#include <hip/hip_runtime.h>

#include "metadata.h"

namespace sputnik_amd {
namespace {

constexpr int kTransposeThreads = 1024;
constexpr int kMaxBlockCols = 32768;  // int16 block-column indices

__global__ void __launch_bounds__(kTransposeThreads)
    transpose_metadata_kernel(int block_rows, int block_cols,
                              const int *__restrict__ offsets,
                              const short *__restrict__ indices,
                              int *__restrict__ offsets_t,
                              short *__restrict__ indices_t,
                              int *__restrict__ block_offsets) {
  __shared__ int cursor[kMaxBlockCols];
  __shared__ int partial[kTransposeThreads];
  const int tid = threadIdx.x;
  const int blocks = offsets[block_rows];

  // 1. Histogram of block-columns.
  for (int c = tid; c < block_cols; c += kTransposeThreads) cursor[c] = 0;
  __syncthreads();
  for (int k = tid; k < blocks; k += kTransposeThreads)
    atomicAdd(&cursor[indices[k]], 1);
  __syncthreads();

  // 2. Exclusive scan -> offsets_t; cursor[c] = first slot of column c.
  const int per = (block_cols + kTransposeThreads - 1) / kTransposeThreads;
  const int c0 = min(tid * per, block_cols);
  const int c1 = min(c0 + per, block_cols);
  int sum = 0;
  for (int c = c0; c < c1; ++c) sum += cursor[c];
  partial[tid] = sum;
  __syncthreads();
  for (int stride = 1; stride < kTransposeThreads; stride <<= 1) {
    const int v = tid >= stride ? partial[tid - stride] : 0;
    __syncthreads();
    partial[tid] += v;
    __syncthreads();
  }
  int run = partial[tid] - sum;  // exclusive prefix of this thread's range
  for (int c = c0; c < c1; ++c) {
    const int n = cursor[c];
    cursor[c] = run;
    offsets_t[c] = run;
    run += n;
  }
  if (tid == 0) offsets_t[block_cols] = blocks;
  __syncthreads();

  // 3. Stable scatter, one block-row at a time.
  for (int r = 0; r < block_rows; ++r) {
    const int k0 = offsets[r];
    const int k1 = offsets[r + 1];
    for (int k = k0 + tid; k < k1; k += kTransposeThreads) {
      const int c = indices[k];
      const int pos = cursor[c];
      cursor[c] = pos + 1;
      indices_t[pos] = static_cast<short>(r);
      block_offsets[pos] = k;
    }
    __syncthreads();
  }
}

__global__ void __launch_bounds__(64)
    row_indices_kernel(int block_rows, const int *__restrict__ offsets,
                       short *__restrict__ row_indices) {
  const int r = blockIdx.x;
  if (r >= block_rows) return;
  const int k0 = offsets[r];
  const int k1 = offsets[r + 1];
  for (int k = k0 + threadIdx.x; k < k1; k += 64)
    row_indices[k] = static_cast<short>(r);
}

// ---- block mask -> BCSR (reference matrix_utils.cu:254-289: a row-major
// scan of the block mask emits each row's present columns in ascending
// order; with pad_rows_to = 1 there is no padding). Three stream-ordered
// launches: per-row counts, one exclusive scan, per-row compaction.
constexpr int kScanThreads = 1024;

__global__ void __launch_bounds__(64)
    mask_row_count_kernel(int block_rows, int block_cols,
                          const unsigned char *__restrict__ mask,
                          int *__restrict__ offsets) {
  const int r = blockIdx.x;
  if (r >= block_rows) return;
  const unsigned char *row = mask + (long long)r * block_cols;
  int n = 0;
  for (int c = threadIdx.x; c < block_cols; c += 64) n += row[c] != 0;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) n += __shfl_xor(n, d, 64);
  if (threadIdx.x == 0) offsets[r + 1] = n;
}

// offsets[1..R] hold the row counts on entry; exclusive prefix sums on exit
// (offsets[0] = 0), one workgroup, each thread a contiguous run of rows.
__global__ void __launch_bounds__(kScanThreads)
    offsets_scan_kernel(int block_rows, int *__restrict__ offsets) {
  __shared__ int partial[kScanThreads];
  const int tid = threadIdx.x;
  const int per = (block_rows + kScanThreads - 1) / kScanThreads;
  const int r0 = min(tid * per, block_rows);
  const int r1 = min(r0 + per, block_rows);
  int sum = 0;
  for (int r = r0; r < r1; ++r) sum += offsets[r + 1];
  partial[tid] = sum;
  __syncthreads();
  for (int stride = 1; stride < kScanThreads; stride <<= 1) {
    const int v = tid >= stride ? partial[tid - stride] : 0;
    __syncthreads();
    partial[tid] += v;
    __syncthreads();
  }
  int run = partial[tid] - sum;
  for (int r = r0; r < r1; ++r) {
    const int n = offsets[r + 1];
    offsets[r + 1] = run + n;
    run += n;
  }
  if (tid == 0) offsets[0] = 0;
}

__global__ void __launch_bounds__(64)
    mask_row_emit_kernel(int block_rows, int block_cols,
                         const unsigned char *__restrict__ mask,
                         const int *__restrict__ offsets,
                         short *__restrict__ indices) {
  const int r = blockIdx.x;
  if (r >= block_rows) return;
  const unsigned char *row = mask + (long long)r * block_cols;
  const int lane = threadIdx.x;
  int pos = offsets[r];
  for (int c0 = 0; c0 < block_cols; c0 += 64) {
    const int c = c0 + lane;
    const bool present = c < block_cols && row[c] != 0;
    const unsigned long long bal = __ballot(present);
    if (present)
      indices[pos + __popcll(bal & ((1ull << lane) - 1))] =
          static_cast<short>(c);
    pos += __popcll(bal);
  }
}

// ---- MoE expert topology (the MegaBlocks dMoE layout, BASELINE config 4):
// block-row r holds tokens of expert e(r) = #{e : padded_bins[e] <= 128 r}
// (padded_bins = cumulative token counts, each padded to a multiple of 128)
// and owns that expert's blocks_per_expert block-columns.
__global__ void __launch_bounds__(256)
    expert_topology_kernel(const int *__restrict__ padded_bins,
                           int num_experts, int block_rows,
                           int blocks_per_expert, int *__restrict__ offsets,
                           short *__restrict__ indices) {
  const int r = blockIdx.x * blockDim.x + threadIdx.x;
  if (r > block_rows) return;
  offsets[r] = r * blocks_per_expert;
  if (r == block_rows) return;
  const int token = r * 128;
  int lo = 0, hi = num_experts;  // upper bound of token in padded_bins
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (padded_bins[mid] <= token) lo = mid + 1; else hi = mid;
  }
  const int e = min(lo, num_experts - 1);
  short *out = indices + (long long)r * blocks_per_expert;
  for (int j = 0; j < blocks_per_expert; ++j)
    out[j] = static_cast<short>(e * blocks_per_expert + j);
}

}  // namespace

hipError_t LaunchMaskToBcsr(int block_rows, int block_cols,
                            const unsigned char *mask, int *offsets,
                            short *indices, hipStream_t stream) {
  if (block_rows < 0 || block_cols < 0 || block_cols > kMaxBlockCols)
    return hipErrorInvalidValue;
  if (block_rows == 0) {
    return hipMemsetAsync(offsets, 0, sizeof(int), stream);
  }
  hipLaunchKernelGGL(mask_row_count_kernel, dim3(block_rows), dim3(64), 0,
                     stream, block_rows, block_cols, mask, offsets);
  hipLaunchKernelGGL(offsets_scan_kernel, dim3(1), dim3(kScanThreads), 0,
                     stream, block_rows, offsets);
  hipLaunchKernelGGL(mask_row_emit_kernel, dim3(block_rows), dim3(64), 0,
                     stream, block_rows, block_cols, mask, offsets, indices);
  return hipGetLastError();
}

hipError_t LaunchExpertTopology(const int *padded_bins, int num_experts,
                                int block_rows, int blocks_per_expert,
                                int *offsets, short *indices,
                                hipStream_t stream) {
  if (num_experts <= 0 || block_rows < 0 || blocks_per_expert <= 0 ||
      (long long)num_experts * blocks_per_expert > kMaxBlockCols)
    return hipErrorInvalidValue;
  const int n = block_rows + 1;
  hipLaunchKernelGGL(expert_topology_kernel, dim3((n + 255) / 256), dim3(256),
                     0, stream, padded_bins, num_experts, block_rows,
                     blocks_per_expert, offsets, indices);
  return hipGetLastError();
}

hipError_t LaunchTransposeMetadata(int block_rows, int block_cols,
                                   const int *offsets, const short *indices,
                                   int *offsets_t, short *indices_t,
                                   int *block_offsets, hipStream_t stream) {
  if (block_cols > kMaxBlockCols || block_rows < 0 || block_cols < 0)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(transpose_metadata_kernel, dim3(1),
                     dim3(kTransposeThreads), 0, stream, block_rows,
                     block_cols, offsets, indices, offsets_t, indices_t,
                     block_offsets);
  return hipGetLastError();
}

hipError_t LaunchRowIndices(int block_rows, const int *offsets,
                            short *row_indices, hipStream_t stream) {
  if (block_rows <= 0) return hipSuccess;
  hipLaunchKernelGGL(row_indices_kernel, dim3(block_rows), dim3(64), 0, stream,
                     block_rows, offsets, row_indices);
  return hipGetLastError();
}

}  // namespace sputnik_amd
