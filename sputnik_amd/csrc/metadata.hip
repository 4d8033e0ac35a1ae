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
// that hold that column. Each workgroup owns a slice of block-columns and
// builds, in LDS, the slice's column-major bit matrix (bit r of column c set
// when block-row r holds c) plus a per-word prefix count; a block's rank is
// then one prefix lookup plus one popcount, with no ordering between threads
// and no communication between workgroups (each counts the blocks left of
// its slice itself).
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
constexpr int kTransposeWaves = kTransposeThreads / 64;
constexpr int kMaxBlockCols = 32768;  // int16 block-column indices
// LDS words (32 rows each) of one slice: bit words + their prefix counts.
constexpr int kTransposeWords = 16384;
// Blocks per thread kept in registers by the one-slice path.
constexpr int kTransposeCache = 4;

// Calls f(row, entry, column) for every stored block of `slice` columns
// [c0, c1), one wave per block-row.
template <typename F>
__device__ __forceinline__ void for_slice_blocks(int block_rows,
                                                 const int *offsets,
                                                 const short *indices, int c0,
                                                 int c1, F f) {
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  for (int r = wave; r < block_rows; r += kTransposeWaves) {
    const int k1 = offsets[r + 1];
    for (int k = offsets[r] + lane; k < k1; k += 64) {
      const int c = indices[k];
      if (c >= c0 && c < c1) f(r, k, c);
    }
  }
}

// Exclusive prefix of v over the workgroup's threads (thread order) and the
// total: wave scans by shuffles, then the wave totals; two barriers.
__device__ __forceinline__ int block_exclusive_scan(int v, int *wsum,
                                                    int *total) {
  const int lane = threadIdx.x & 63;
  const int wave = threadIdx.x >> 6;
  int incl = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const int t = __shfl_up(incl, d, 64);
    if (lane >= d) incl += t;
  }
  if (lane == 63) wsum[wave] = incl;
  __syncthreads();
  int below = 0, all = 0;
#pragma unroll
  for (int i = 0; i < kTransposeWaves; ++i) {
    const int t = wsum[i];
    below += i < wave ? t : 0;
    all += t;
  }
  __syncthreads();  // wsum may be reused
  *total = all;
  return below + incl - v;
}

__global__ void __launch_bounds__(kTransposeThreads)
    transpose_metadata_kernel(int block_rows, int block_cols, int slice,
                              int blocks, const int *__restrict__ offsets,
                              const short *__restrict__ indices,
                              int *__restrict__ offsets_t,
                              short *__restrict__ indices_t,
                              int *__restrict__ block_offsets) {
  __shared__ unsigned bits[kTransposeWords];
  __shared__ int prefix[kTransposeWords];
  __shared__ int partial[kTransposeThreads];
  __shared__ int wsum[kTransposeWaves];
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int words = (block_rows + 31) >> 5;  // per column
  const int c0 = blockIdx.x * slice;
  const int c1 = min(c0 + slice, block_cols);
  const int ncols = c1 - c0;

  // 1. Bit matrix of the slice; blocks left of the slice (the slice's base).
  // Small matrices (one slice, a few blocks per thread) keep each block's
  // (row, column) in registers: one round trip to memory for the offsets
  // (staged in `prefix`, free until step 2) and the indices, issued together;
  // a block's row is a binary search of the staged offsets.
  const bool cached = gridDim.x == 1 &&
                      blocks <= kTransposeCache * kTransposeThreads &&
                      block_rows < kTransposeWords;
  int crow[kTransposeCache], ccol[kTransposeCache];
  if (cached) {
    int *offs = prefix;
    for (int i = tid; i <= block_rows; i += kTransposeThreads)
      offs[i] = offsets[i];
#pragma unroll
    for (int q = 0; q < kTransposeCache; ++q) {
      const int k = tid + q * kTransposeThreads;
      ccol[q] = k < blocks ? indices[k] : -1;
    }
    for (int w = tid; w < ncols * words; w += kTransposeThreads) bits[w] = 0;
    __syncthreads();
#pragma unroll
    for (int q = 0; q < kTransposeCache; ++q) {
      const int k = tid + q * kTransposeThreads;
      if (ccol[q] < 0) continue;
      int lo = 0, hi = block_rows;  // offs[lo] <= k < offs[hi]
      while (hi - lo > 1) {
        const int mid = (lo + hi) >> 1;
        if (offs[mid] <= k) lo = mid; else hi = mid;
      }
      crow[q] = lo;
      atomicOr(&bits[ccol[q] * words + (lo >> 5)], 1u << (lo & 31));
    }
  } else {
    for (int w = tid; w < ncols * words; w += kTransposeThreads) bits[w] = 0;
    __syncthreads();
    for_slice_blocks(block_rows, offsets, indices, c0, c1,
                     [&](int r, int, int c) {
                       atomicOr(&bits[(c - c0) * words + (r >> 5)],
                                1u << (r & 31));
                     });
  }
  // Blocks left of the slice (none for the first slice).
  int base = 0;
  if (c0 > 0) {
    int left = 0;
    for (int k = tid; k < blocks; k += kTransposeThreads)
      left += indices[k] < c0 ? 1 : 0;
    block_exclusive_scan(left, wsum, &base);
  } else {
    __syncthreads();
  }

  // 2. Per-column word prefix counts (one wave per column, 64 words a pass)
  //    and column totals.
  const int wave = tid >> 6;
  if (words == 1) {  // <= 32 block-rows: one word per column, no scan
    for (int cl = tid; cl < ncols; cl += kTransposeThreads) {
      prefix[cl] = 0;
      partial[cl] = __popc(bits[cl]);
    }
  } else
  for (int cl = wave; cl < ncols; cl += kTransposeWaves) {
    int run = 0;
    for (int w0 = 0; w0 < words; w0 += 64) {
      const int w = w0 + lane;
      const int n = w < words ? __popc(bits[cl * words + w]) : 0;
      int incl = n;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int v = __shfl_up(incl, d, 64);
        if (lane >= d) incl += v;
      }
      if (w < words) prefix[cl * words + w] = run + incl - n;
      run += __shfl(incl, 63, 64);
    }
    if (lane == 0) partial[cl] = run;  // ncols <= kTransposeThreads
  }
  __syncthreads();

  // 3. Exclusive scan of the column totals -> offsets_t (slice <= threads:
  //    thread t owns column c0 + t).
  if (ncols <= 64) {  // one wave scans (no workgroup scan barriers)
    if (wave == 0) {
      const int v = lane < ncols ? partial[lane] : 0;
      int incl = v;
#pragma unroll
      for (int d = 1; d < 64; d <<= 1) {
        const int t = __shfl_up(incl, d, 64);
        if (lane >= d) incl += t;
      }
      const int first = base + incl - v;
      if (lane < ncols) {
        partial[lane] = first;  // first slot of column c0 + lane
        offsets_t[c0 + lane] = first;
      }
      if (c1 == block_cols && lane == 0) offsets_t[block_cols] = blocks;
    }
  } else {
    const int mine = tid < ncols ? partial[tid] : 0;
    int unused;
    const int first = base + block_exclusive_scan(mine, wsum, &unused);
    if (tid < ncols) {
      partial[tid] = first;  // first slot of column c0 + tid
      offsets_t[c0 + tid] = first;
    }
    if (c1 == block_cols && tid == 0) offsets_t[block_cols] = blocks;
  }
  __syncthreads();

  // 4. Scatter: slot = column start + rank of the block-row in its column.
  auto scatter = [&](int r, int k, int c) {
    const int cl = c - c0;
    const int w = cl * words + (r >> 5);
    const int rank = prefix[w] + __popc(bits[w] & ((1u << (r & 31)) - 1u));
    const int pos = partial[cl] + rank;
    indices_t[pos] = static_cast<short>(r);
    block_offsets[pos] = k;
  };
  if (cached) {
#pragma unroll
    for (int q = 0; q < kTransposeCache; ++q)
      if (ccol[q] >= 0) scatter(crow[q], tid + q * kTransposeThreads, ccol[q]);
  } else {
    for_slice_blocks(block_rows, offsets, indices, c0, c1, scatter);
  }
}

// ---- Bitmask (reference sputnik/block/bitmask/bitmask.cu:7-45 with the
// BitMatrix layout of bit_matrix.h:14-40): a row-major bit matrix of
// ceil(cols/64) uint64 words per block-row, bit j % 64 of word j / 64 set
// when the row holds block-column j. The words are zeroed by the launcher;
// one wave per block-row ORs its blocks in.
__global__ void __launch_bounds__(256)
    bitmask_kernel(int block_rows, int words_per_row,
                   const int *__restrict__ offsets,
                   const short *__restrict__ indices,
                   unsigned long long *__restrict__ bitmask) {
  const int r = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (r >= block_rows) return;
  const int lane = threadIdx.x & 63;
  const int k1 = offsets[r + 1];
  for (int k = offsets[r] + lane; k < k1; k += 64) {
    const int j = indices[k];
    atomicOr(bitmask + (long long)r * words_per_row + (j >> 6),
             1ull << (j & 63));
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

hipError_t LaunchTransposeMetadata(int block_rows, int block_cols, int blocks,
                                   const int *offsets, const short *indices,
                                   int *offsets_t, short *indices_t,
                                   int *block_offsets, hipStream_t stream) {
  if (block_cols > kMaxBlockCols || block_rows < 0 || block_cols < 0)
    return hipErrorInvalidValue;
  if (block_cols == 0)
    return hipMemsetAsync(offsets_t, 0, sizeof(int), stream);
  const int words = (block_rows + 31) / 32;
  // Columns per workgroup: the slice's bit words and prefixes fit in LDS,
  // and its column totals fit one per thread.
  int slice = words == 0 ? block_cols : kTransposeWords / words;
  slice = slice < 1 ? 1 : slice;
  slice = slice > kTransposeThreads ? kTransposeThreads : slice;
  slice = slice > block_cols ? block_cols : slice;
  const int grid = (block_cols + slice - 1) / slice;
  hipLaunchKernelGGL(transpose_metadata_kernel, dim3(grid),
                     dim3(kTransposeThreads), 0, stream, block_rows,
                     block_cols, slice, blocks, offsets, indices, offsets_t,
                     indices_t, block_offsets);
  return hipGetLastError();
}

hipError_t LaunchBitmask(int block_rows, int block_cols, const int *offsets,
                         const short *indices, unsigned long long *bitmask,
                         hipStream_t stream) {
  if (block_rows < 0 || block_cols < 0 || block_cols > kMaxBlockCols)
    return hipErrorInvalidValue;
  const int words = (block_cols + 63) / 64;
  const size_t bytes = (size_t)words * block_rows * sizeof(unsigned long long);
  if (bytes == 0) return hipSuccess;
  const hipError_t e = hipMemsetAsync(bitmask, 0, bytes, stream);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(bitmask_kernel, dim3((block_rows + 3) / 4), dim3(256), 0,
                     stream, block_rows, words, offsets, indices, bitmask);
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
