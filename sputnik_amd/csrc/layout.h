// Dense layout helpers (layout.hip).
#ifndef SPUTNIK_AMD_LAYOUT_H_
#define SPUTNIK_AMD_LAYOUT_H_

#include <hip/hip_runtime.h>

namespace sputnik_amd {

// out ([cols][rows], row-major) = in^T for in [rows][cols] row-major, 2-byte
// elements; rows and cols multiples of 64 (else hipErrorInvalidValue).
hipError_t LaunchTranspose16(const void *in, int rows, int cols, void *out,
                             hipStream_t stream);

}  // namespace sputnik_amd

#endif  // SPUTNIK_AMD_LAYOUT_H_
