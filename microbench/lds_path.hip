// Does LDS-DMA landing compete with fragment reads for the LDS on gfx950?
// (experiment, not part of the library; DESIGN.md §3.1 "What bounds the
// k-loop"). One 512-thread workgroup per CU, the headline kernel's wave
// count. Per "step" a DMA wave issues 5 buffer_load_dwordx4 ... lds (5 KiB,
// L2-resident source, two steps in flight) and a read wave issues 12
// ds_read_b128 (12 KiB) and waits for them, as the k-loop's two halves do.
//   mode 0: waves 0-3 stream DMA, waves 4-7 idle
//   mode 1: waves 4-7 read, waves 0-3 idle
//   mode 2: both at once (waves 0-3 DMA, 4-7 read)
//   mode 3: all 8 waves DMA          mode 4: all 8 waves read
// If mode 2 takes about the longer of modes 0 and 1, the two paths are
// independent; about their sum, they share the LDS.
// Build: hipcc -O3 --offload-arch=gfx950 lds_path.hip -o lds_path
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef unsigned v4u __attribute__((ext_vector_type(4)));
#define LDS(p) ((__attribute__((address_space(3))) void *)(p))

template <int kMode>
__global__ void __launch_bounds__(512, 1)
    lds_path(const char *src, unsigned span, int iters, unsigned *sink) {
  __shared__ __attribute__((aligned(1024))) char lds[8 * 20480];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const bool dma = kMode == 3 || (kMode != 4 && wave < 4);
  const bool rd = kMode == 4 || (kMode != 3 && wave >= 4);
  const bool on = (kMode == 0 && wave < 4) || (kMode == 1 && wave >= 4) ||
                  kMode >= 2;
  v4u acc = {0, 0, 0, 0};
  if (on && dma) {
    const __amdgpu_buffer_rsrc_t r = __builtin_amdgcn_make_buffer_rsrc(
        const_cast<char *>(src), 0, 0x7fffffff, 0x00020000);
    char *ring = lds + wave * 20480;
    unsigned base = ((blockIdx.x * 8 + wave) * 8192u) % span;
#pragma unroll 4
    for (int it = 0; it < iters; ++it) {
      char *slot = ring + (it & 3) * 5120;
#pragma unroll
      for (int q = 0; q < 5; ++q)
        __builtin_amdgcn_raw_ptr_buffer_load_lds(
            r, LDS(slot + q * 1024), 16, (base + q * 1024 + lane * 16) % span,
            0, 0, 0);
      asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
      base = (base + 5 * 1024 * 2048) % span;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (on && rd) {
    const char *img = lds + (wave & 3) * 20480;
#pragma unroll 2
    for (int it = 0; it < iters; ++it) {
      const char *s = img + (it & 3) * 5120 + lane * 16;
      v4u v[12];
#pragma unroll
      for (int q = 0; q < 12; ++q)
        v[q] = *reinterpret_cast<const v4u *>(s + (q % 5) * 1024);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int q = 0; q < 12; ++q) acc ^= v[q];
    }
  }
  __syncthreads();
  const unsigned x = acc.x ^ acc.y ^ acc.z ^ acc.w;
  if (x == 0x12345678u) sink[0] = x;
}

template <int kMode>
float run(const char *src, unsigned span, int iters, unsigned *sink, int grid) {
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  for (int w = 0; w < 3; ++w)
    hipLaunchKernelGGL(lds_path<kMode>, dim3(grid), dim3(512), 0, 0, src, span,
                       iters, sink);
  hipEventRecord(a);
  const int reps = 10;
  for (int w = 0; w < reps; ++w)
    hipLaunchKernelGGL(lds_path<kMode>, dim3(grid), dim3(512), 0, 0, src, span,
                       iters, sink);
  hipEventRecord(b);
  hipEventSynchronize(b);
  float ms = 0;
  hipEventElapsedTime(&ms, a, b);
  return ms / reps;
}

int main(int argc, char **argv) {
  const unsigned span = (argc > 1 ? atoi(argv[1]) : 2) << 20;  // MiB (L2-resident)
  const int iters = 4000, grid = 256;
  char *src;
  unsigned *sink;
  if (hipMalloc(&src, span) != hipSuccess || hipMalloc(&sink, 64) != hipSuccess)
    return 1;
  hipMemset(src, 1, span);
  const char *names[5] = {"dma_4w", "read_4w", "dma_4w+read_4w", "dma_8w",
                          "read_8w"};
  float t[5];
  t[0] = run<0>(src, span, iters, sink, grid);
  t[1] = run<1>(src, span, iters, sink, grid);
  t[2] = run<2>(src, span, iters, sink, grid);
  t[3] = run<3>(src, span, iters, sink, grid);
  t[4] = run<4>(src, span, iters, sink, grid);
  for (int m = 0; m < 5; ++m)
    printf("{\"mode\": \"%s\", \"span_MiB\": %u, \"ms\": %.3f, "
           "\"us_per_step\": %.4f}\n",
           names[m], span >> 20, t[m], t[m] * 1e3 / iters);
  return hipDeviceSynchronize() == hipSuccess ? 0 : 1;
}
