// Dense layout helper for the SDD dispatcher (dispatch.cpp UseBtTranspose):
// out = in^T for a row-major [rows][cols] matrix of 2-byte elements (fp16 /
// bf16 bit patterns), rows and cols multiples of 64. Used to turn an SDD NT
// / TT operand B^T ([N][K], k-contiguous rows) into B ([K][N]) once per call
// when B is too large for the MALL and the product is dense enough that the
// N-major kernel's saving outweighs the copy.
//
// One workgroup per 64 x 64 tile: 256 threads, each loads 16 consecutive
// elements of one input row (2 x 16 B, so a row's 128 B come from 4
// neighbouring lanes), stages them in LDS, and writes 16 consecutive
// elements of one output row gathered down a tile column. The LDS pitch is
// 66 elements (33 dwords, odd), so the column gathers of neighbouring rows
// fall in different banks. HBM-bound: 2 x rows x cols x 2 bytes per call.

#include <hip/hip_runtime.h>

#include <cstdint>

#include "layout.h"

namespace sputnik_amd {
namespace {

constexpr int kTile = 64;
constexpr int kPitch = 66;
typedef unsigned v4u __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256)
    transpose16_kernel(const uint16_t *__restrict__ in, long long ld_in,
                       uint16_t *__restrict__ out, long long ld_out) {
  __shared__ uint16_t tile[kTile * kPitch];
  const int t = threadIdx.x;
  const long long r0 = (long long)blockIdx.y * kTile;  // input rows
  const long long c0 = (long long)blockIdx.x * kTile;  // input cols
  {
    const int r = t >> 2, c = (t & 3) * 16;
    const v4u *src = reinterpret_cast<const v4u *>(in + (r0 + r) * ld_in + c0 + c);
    const v4u v0 = __builtin_nontemporal_load(src);
    const v4u v1 = __builtin_nontemporal_load(src + 1);
    const uint32_t w[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    uint16_t *dst = tile + r * kPitch + c;
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      dst[2 * i] = (uint16_t)(w[i] & 0xffffu);
      dst[2 * i + 1] = (uint16_t)(w[i] >> 16);
    }
  }
  __syncthreads();
  {
    const int oc = t >> 2, rr = (t & 3) * 16;  // output row oc = input col
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i)
      w[i] = (uint32_t)tile[(rr + 2 * i) * kPitch + oc] |
             ((uint32_t)tile[(rr + 2 * i + 1) * kPitch + oc] << 16);
    v4u *dst = reinterpret_cast<v4u *>(out + (c0 + oc) * ld_out + r0 + rr);
    dst[0] = v4u{w[0], w[1], w[2], w[3]};
    dst[1] = v4u{w[4], w[5], w[6], w[7]};
  }
}

}  // namespace

hipError_t LaunchTranspose16(const void *in, int rows, int cols, void *out,
                             hipStream_t stream) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  if (rows % kTile != 0 || cols % kTile != 0) return hipErrorInvalidValue;
  const dim3 grid(cols / kTile, rows / kTile), block(256);
  hipLaunchKernelGGL(transpose16_kernel, grid, block, 0, stream,
                     static_cast<const uint16_t *>(in), (long long)cols,
                     static_cast<uint16_t *>(out), (long long)rows);
  return hipGetLastError();
}

}  // namespace sputnik_amd
