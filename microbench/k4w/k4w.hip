// Experiment: 4-wave DSD NN kernel with a hand-scheduled k-loop
// (gen_k4w.py). One workgroup = 4 waves, one per SIMD, 128 x 512 output tile,
// no pair balancing. Build: see run_k4w.py.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "k4w_loop.inc"

namespace {

struct K4wParams {
  const char *s_data;
  const int *s_offsets;
  const short *s_indices;
  const char *d_data;
  char *c_data;
  long long d_ld;  // bytes
  long long c_ld;  // bytes
  int num_rows;
  int num_jtiles;
  int j_limit;
  unsigned long long *debug;
};

__device__ __forceinline__ int tr_key(int k) {
  return (k & 3) | (((k >> 3) & 1) << 2);
}

__device__ __forceinline__ int xcd_tile(int bid, int nwg) {
  const int xcd = bid & 7;
  const int q = nwg >> 3;
  const int r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

__device__ __forceinline__ int sload_short(const short *base, int e) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(base + e);
  const int v = *reinterpret_cast<const __attribute__((address_space(4))) int *>(
      a & ~uintptr_t(3));
  return ((a & 2) ? (v >> 16) : v) & 0xffff;
}

template <bool kBf16, int kVar>
__global__ void __launch_bounds__(256, 1) k4w_dsd_nn(const K4wParams p) {
  __shared__ __attribute__((aligned(1024))) char lds[163840];
  const unsigned long long r_entry = __builtin_amdgcn_s_memrealtime();
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint32_t lbase =
      (uint32_t)(uintptr_t)((__attribute__((address_space(3))) char *)lds);

  // dense-panel-major tile order: an XCD walks the rows of one panel
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int jt = tile / p.num_rows;
  const int row = tile % p.num_rows;
  const int j0 = jt * 512;
  const int e0 = __builtin_amdgcn_readfirstlane(p.s_offsets[row]);
  const int e1 = __builtin_amdgcn_readfirstlane(p.s_offsets[row + 1]);
  const int nblk = e1 - e0;
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  if (nblk == 0) {
    const v4u z = {0u, 0u, 0u, 0u};
    for (int id = tid; id < 128 * 64; id += 256) {
      const int r = id >> 6, cc = id & 63;
      const int jc = j0 + cc * 8;
      if (jc >= p.j_limit) continue;
      __builtin_nontemporal_store(
          z, reinterpret_cast<v4u *>(p.c_data + ((long long)row * 128 + r) * p.c_ld +
                                     (long long)jc * 2));
    }
    return;
  }
  const int elast = e1 - 1;
  const int kb0 = sload_short(p.s_indices, e0);
  const int kb1 = sload_short(p.s_indices, e0 + 1 <= elast ? e0 + 1 : elast);

  const uint32_t vsl = (uint32_t)(lane * 16 + wave * 2048);
  // S DMA: rows 32 w + l/4 (+16 for q = 1), chunk (l%4) ^ key(row)
  const int srow = 32 * wave + (lane >> 2);
  const uint32_t vs = (uint32_t)(srow * 256 + (((lane & 3) ^ ((srow >> 1) & 3)) << 4));
  // D DMA: k = 4 q + l/16, chunk pc = l%16 -> source chunk c(x), x = (q>>1)&1
  uint32_t vd[2];
  for (int x = 0; x < 2; ++x) {
    const int k = (lane >> 4) + 8 * x;  // representative k with bit 3 = x
    const int pc = lane & 15;
    const int c = (((pc >> 1) ^ tr_key(k)) << 1) | (pc & 1);
    const int col = j0 + 128 * wave + c * 8;
    vd[x] = col < p.j_limit ? (uint32_t)((lane >> 4) * p.d_ld + c * 16) : 0x80000000u;
  }
  // S fragment reads
  const int r16 = lane & 15, g = lane >> 4;
  const uint32_t vrs = lbase + (uint32_t)(r16 * 64 + ((g ^ ((r16 >> 1) & 3)) << 4));
  // D fragment reads (wave image at 32K + 32K w)
  const int q = (lane >> 2) & 3, pp = lane & 3;
  const int kr = 8 * g + q;
  uint32_t vrd[8];
  for (int n = 0; n < 8; ++n)
    vrd[n] = lbase + 32768u + 32768u * wave +
             (uint32_t)(kr * 256 + pp * 8 + ((n ^ tr_key(kr)) << 5));
  const uint32_t vw0 = lbase + (uint32_t)(r16 * 1040 + (128 * wave + 4 * g) * 2);
  const uint32_t vw1 = vw0 + 64 * 1040;

  const uint64_t sd = (uint64_t)p.s_data;
  const uint64_t dt = (uint64_t)(p.d_data + (long long)(j0 + 128 * wave) * 2);
  const uint64_t ix = (uint64_t)p.s_indices;
  const uint32_t k128 = (uint32_t)(128 * p.d_ld);
  const uint32_t k32 = (uint32_t)(32 * p.d_ld);
  const uint32_t k4 = (uint32_t)(4 * p.d_ld);
  const uint32_t ms = lbase + 2048u * wave;
  const uint32_t md = lbase + 32768u + 32768u * wave;

  unsigned long long t0 = 0, t1 = 0, r0 = 0, r1 = 0;
#define K4W_OPERANDS                                                         \
  [t0] "=&s"(t0), [t1] "=&s"(t1), [r0] "=&s"(r0), [r1] "=&s"(r1)              \
  : [sdlo] "s"((uint32_t)sd), [sdhi] "s"((uint32_t)(sd >> 32)),             \
    [dtlo] "s"((uint32_t)dt), [dthi] "s"((uint32_t)(dt >> 32)),             \
    [k128] "s"(k128), [k32] "s"(k32), [k4] "s"(k4),                          \
    [ixlo] "s"((uint32_t)ix), [ixhi] "s"((uint32_t)(ix >> 32)),             \
    [e0] "s"(e0), [elast] "s"(elast), [kb0] "s"(kb0), [kb1] "s"(kb1),        \
    [nblk] "s"(nblk), [ms] "s"(ms), [md] "s"(md), [vs] "v"(vs),              \
    [vd0] "v"(vd[0]), [vd1] "v"(vd[1]), [vrs] "v"(vrs), [vrd0] "v"(vrd[0]), \
    [vrd1] "v"(vrd[1]), [vrd2] "v"(vrd[2]), [vrd3] "v"(vrd[3]),             \
    [vrd4] "v"(vrd[4]), [vrd5] "v"(vrd[5]), [vrd6] "v"(vrd[6]),             \
    [vrd7] "v"(vrd[7]), [vw0] "v"(vw0), [vw1] "v"(vw1), [vsl] "v"(vsl)
  if constexpr (kBf16)
    asm volatile(K4W_ASM_BF16_V0 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 0)
    asm volatile(K4W_ASM_F16_V0 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 1)
    asm volatile(K4W_ASM_F16_V1 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 2)
    asm volatile(K4W_ASM_F16_V2 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 3)
    asm volatile(K4W_ASM_F16_V3 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 4)
    asm volatile(K4W_ASM_F16_V4 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 5)
    asm volatile(K4W_ASM_F16_V5 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 6)
    asm volatile(K4W_ASM_F16_V6 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 7)
    asm volatile(K4W_ASM_F16_V7 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 8)
    asm volatile(K4W_ASM_F16_V8 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 9)
    asm volatile(K4W_ASM_F16_V9 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 10)
    asm volatile(K4W_ASM_F16_V10 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 11)
    asm volatile(K4W_ASM_F16_V11 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 12)
    asm volatile(K4W_ASM_F16_V12 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 13)
    asm volatile(K4W_ASM_F16_V13 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 14)
    asm volatile(K4W_ASM_F16_V14 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 15)
    asm volatile(K4W_ASM_F16_V15 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 16)
    asm volatile(K4W_ASM_F16_V16 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 17)
    asm volatile(K4W_ASM_F16_V17 : K4W_OPERANDS : K4W_CLOBBERS);
  else if constexpr (kVar == 18)
    asm volatile(K4W_ASM_F16_V18 : K4W_OPERANDS : K4W_CLOBBERS);
  else
    asm volatile(K4W_ASM_F16_V19 : K4W_OPERANDS : K4W_CLOBBERS);
  const unsigned long long r_asm = __builtin_amdgcn_s_memrealtime();
  __syncthreads();
  // staging [128][1040 B] -> C, 16-byte nontemporal stores
  for (int id = tid; id < 128 * 64; id += 256) {
    const int r = id >> 6, cc = id & 63;
    const int jc = j0 + cc * 8;
    if (jc >= p.j_limit) continue;
    const v4u v = *reinterpret_cast<const v4u *>(lds + r * 1040 + cc * 16);
    __builtin_nontemporal_store(
        v, reinterpret_cast<v4u *>(p.c_data + ((long long)row * 128 + r) * p.c_ld +
                                   (long long)jc * 2));
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const unsigned long long r_end = __builtin_amdgcn_s_memrealtime();
  if (p.debug != nullptr && tid == 0) {
    unsigned long long *d = p.debug + blockIdx.x * 8;
    d[0] = t0; d[1] = t1; d[2] = r0; d[3] = r1;
    d[4] = r_entry; d[5] = r_asm; d[6] = r_end; d[7] = 0;
  }
}

}  // namespace

extern "C" int k4w_dsd(const void *s_data, const int *offsets, const short *indices,
                       const void *d, void *c, int m, int k, int n, int bf16,
                       int variant, hipStream_t stream, void *debug) {
  K4wParams p;
  p.s_data = (const char *)s_data;
  p.s_offsets = offsets;
  p.s_indices = indices;
  p.d_data = (const char *)d;
  p.c_data = (char *)c;
  p.d_ld = (long long)n * 2;
  p.c_ld = (long long)n * 2;
  p.num_rows = m / 128;
  p.num_jtiles = (n + 511) / 512;
  p.j_limit = n;
  p.debug = (unsigned long long *)debug;
  const int grid = p.num_rows * p.num_jtiles;
  (void)k;
#define K4W_LAUNCH(B, V) \
  hipLaunchKernelGGL((k4w_dsd_nn<B, V>), dim3(grid), dim3(256), 0, stream, p)
  if (bf16) K4W_LAUNCH(true, 0);
  else if (variant == 1) K4W_LAUNCH(false, 1);
  else if (variant == 2) K4W_LAUNCH(false, 2);
  else if (variant == 3) K4W_LAUNCH(false, 3);
  else if (variant == 4) K4W_LAUNCH(false, 4);
  else if (variant == 5) K4W_LAUNCH(false, 5);
  else if (variant == 6) K4W_LAUNCH(false, 6);
  else if (variant == 7) K4W_LAUNCH(false, 7);
  else if (variant == 8) K4W_LAUNCH(false, 8);
  else if (variant == 9) K4W_LAUNCH(false, 9);
  else if (variant == 10) K4W_LAUNCH(false, 10);
  else if (variant == 11) K4W_LAUNCH(false, 11);
  else if (variant == 12) K4W_LAUNCH(false, 12);
  else if (variant == 13) K4W_LAUNCH(false, 13);
  else if (variant == 14) K4W_LAUNCH(false, 14);
  else if (variant == 15) K4W_LAUNCH(false, 15);
  else if (variant == 16) K4W_LAUNCH(false, 16);
  else if (variant == 17) K4W_LAUNCH(false, 17);
  else if (variant == 18) K4W_LAUNCH(false, 18);
  else if (variant == 19) K4W_LAUNCH(false, 19);
  else K4W_LAUNCH(false, 0);
  return (int)hipGetLastError();
}
