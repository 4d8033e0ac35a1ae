// Which XCD (XCC_ID hardware register) each workgroup of a launch lands on:
// out[b] = XCC id of workgroup b. Diagnoses whether blockIdx % 8 maps to a
// fixed physical XCD or to a rotation that depends on the process's
// dispatch history (DESIGN.md section 0e, config 5 / pair placement).
// Build: hipcc -O2 --offload-arch=gfx950 -shared -fPIC xcc_map.hip -o libxcc_map.so
#include <hip/hip_runtime.h>

__global__ void xcc_map_kernel(int *out) {
  if (threadIdx.x == 0) {
    unsigned v;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
    out[blockIdx.x] = (int)(v & 0xf);
  }
}

extern "C" int xcc_map(int *out, int grid, hipStream_t stream) {
  hipLaunchKernelGGL(xcc_map_kernel, dim3(grid), dim3(64), 0, stream, out);
  return (int)hipGetLastError();
}
