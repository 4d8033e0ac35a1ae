// Per-CU L2 -> CU read throughput on gfx950 by load form (experiment, not
// part of the library): one 512-thread workgroup per CU, every wave streams
// 1 KiB wave-instructions from an L2-resident buffer with ~3 steps in flight.
//   mode 0: buffer_load_dwordx4 ... lds (LDS-DMA) into a per-wave LDS ring
//   mode 1: buffer_load_dwordx4 to VGPRs (xor-folded, nothing stored)
//   mode 2: buffer_load_dwordx4 to VGPRs + ds_write_b128 into the ring
//   mode 3: LDS-DMA in the S-operand shape: 16 rows x 64 B per instruction,
//           rows 256 B apart (a 128x128 fp16 block read 32 k at a time)
// Build: hipcc -O3 --offload-arch=gfx950 l2_to_cu.hip -o l2_to_cu
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
#define LDS(p) ((__attribute__((address_space(3))) void *)(p))

template <int kMode, int kPer>
__global__ void __launch_bounds__(512, 1)
    stream(const char *src, unsigned span, int iters, unsigned *sink) {
  __shared__ __attribute__((aligned(1024))) char lds[8 * 16384];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<char *>(src), 0, 0x7fffffff, 0x00020000);
  char *ring = lds + wave * 16384;
  unsigned base = ((blockIdx.x * 8 + wave) * 4096u) % span;
  v4u acc = {0, 0, 0, 0};
#pragma unroll 4
  for (int it = 0; it < iters; ++it) {
    char *slot = ring + (it & 3) * 4096;
#pragma unroll
    for (int q = 0; q < kPer; ++q) {
      unsigned off = (base + q * 1024 + lane * 16) % span;
      if constexpr (kMode == 3)
        off = (base + q * 4096 + (lane >> 2) * 256 + (lane & 3) * 16 +
               (it & 3) * 64) % span;
      if constexpr (kMode == 0 || kMode == 3) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(r, LDS(slot + q * 1024), 16,
                                                 off, 0, 0, 0);
      } else {
        v4u v = __builtin_amdgcn_raw_buffer_load_b128(r, off, 0, 0);
        if constexpr (kMode == 1) {
          acc ^= v;
        } else {
          *reinterpret_cast<v4u *>(slot + q * 1024 + lane * 16) = v;
        }
      }
    }
    if constexpr (kMode == 0 || kMode == 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * kPer) : "memory");
    base = (base + kPer * 1024 * 256 * 8) % span;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned x = acc.x ^ acc.y ^ acc.z ^ acc.w ^
               *reinterpret_cast<unsigned *>(lds + (threadIdx.x * 64) % sizeof(lds));
  if (x == 0x12345678u) sink[0] = x;
}

template <int kMode>
float run(const char *src, unsigned span, int iters, unsigned *sink, int grid) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w)
    hipLaunchKernelGGL((stream<kMode, 4>), dim3(grid), dim3(512), 0, 0, src, span, iters, sink);
  hipEventRecord(a);
  const int reps = 10;
  for (int w = 0; w < reps; ++w)
    hipLaunchKernelGGL((stream<kMode, 4>), dim3(grid), dim3(512), 0, 0, src, span, iters, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main(int argc, char **argv) {
  const unsigned span = argc > 1 ? atoi(argv[1]) << 20 : 2u << 20;  // MiB
  const int iters = 2000, grid = 256;
  char *src;
  unsigned *sink;
  hipMalloc(&src, span);
  hipMemset(src, 1, span);
  hipMalloc(&sink, 64);
  const double bytes = (double)grid * 8 * 4 * 1024 * iters;
  const char *names[4] = {"lds_dma", "vgpr", "vgpr+ds_write", "lds_dma_64B_rows"};
  float t[4];
  t[0] = run<0>(src, span, iters, sink, grid);
  t[1] = run<1>(src, span, iters, sink, grid);
  t[2] = run<2>(src, span, iters, sink, grid);
  t[3] = run<3>(src, span, iters, sink, grid);
  for (int m = 0; m < 4; ++m)
    printf("{\"mode\": \"%s\", \"span_MiB\": %u, \"ms\": %.3f, \"TBps\": %.2f, \"GBps_per_CU\": %.1f}\n",
           names[m], span >> 20, t[m], bytes / t[m] / 1e9, bytes / t[m] / 1e6 / grid);
  return 0;
}
