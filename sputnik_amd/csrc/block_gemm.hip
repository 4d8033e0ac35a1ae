// sputnik-amd: instantiations of the block-sparse GEMM kernel and the
// variant dispatch. Replaces the reference's per-variant CUTLASS files
// (sputnik/block/{dsd,dds,sdd}/cutlass/*_align8.cu) and the first-fit
// registries (dsd/cutlass/dsd.cu:30-66 and siblings): the variant is a pure
// function of (product, transposes, dtype), so no registry is needed.
#include <type_traits>

#include "block_gemm.h"

namespace sputnik_amd {
namespace {

template <typename T, bool kSparseOut, bool kSKC, bool kDKC, bool kOutT,
          class Cfg>
hipError_t LaunchCfg(const GemmParams &p, hipStream_t stream) {
  hipLaunchKernelGGL((block_gemm_kernel<T, kSparseOut, kSKC, kDKC, kOutT, Cfg>),
                     dim3(p.grid > 0 ? p.grid : p.num_tiles),
                     dim3(64 * Cfg::kWaves), 0,
                     stream, p);
  return hipGetLastError();
}

template <typename T, bool kSparseOut, bool kSKC, bool kDKC, bool kOutT>
hipError_t Launch(const GemmParams &p, bool grouped, hipStream_t stream) {
  if (p.num_tiles <= 0) return hipSuccess;
  if constexpr (kSparseOut) {
    if (grouped)
      return LaunchCfg<T, true, kSKC, kDKC, false, CfgSddGrouped>(p, stream);
    return LaunchCfg<T, true, kSKC, kDKC, false, CfgSdd>(p, stream);
  } else {
    // Tall sparse operands (many more tiles than CUs, no pair balancing):
    // two 128x256 workgroups per CU, so one tile's prologue and epilogue
    // overlap the other's pipeline.
    if (grouped)
      return LaunchCfg<T, false, kSKC, kDKC, kOutT, CfgTall>(p, stream);
    // Split mode (few tiles): two workgroups per tile, its own kernel.
    if (p.pair != 0 && p.pair_split > 1) {
      if (p.split_bn == 128)
        return LaunchCfg<T, false, kSKC, kDKC, kOutT, CfgSplit128>(p, stream);
      if (p.split_bn == 256)
        return LaunchCfg<T, false, kSKC, kDKC, kOutT, CfgSplit256>(p, stream);
      return LaunchCfg<T, false, kSKC, kDKC, kOutT, CfgSplit>(p, stream);
    }
    return LaunchCfg<T, false, kSKC, kDKC, kOutT, CfgSparse>(p, stream);
  }
}

template <typename T>
hipError_t LaunchTyped(bool sparse_out, bool s_kc, bool d_kc, bool out_t,
                       bool g, const GemmParams &p, hipStream_t stream) {
  const int code = (s_kc ? 4 : 0) | (d_kc ? 2 : 0) | (out_t ? 1 : 0);
  if (sparse_out) {
    switch (code & 6) {
      case 6: return Launch<T, true, true, true, false>(p, g, stream);   // SDD NT
      case 4: return Launch<T, true, true, false, false>(p, g, stream);  // SDD NN
      case 2: return Launch<T, true, false, true, false>(p, g, stream);  // SDD TT
      default: return Launch<T, true, false, false, false>(p, g, stream);  // TN
    }
  }
  switch (code) {
    case 4: return Launch<T, false, true, false, false>(p, g, stream);  // DSD NN
    case 6: return Launch<T, false, true, true, false>(p, g, stream);   // DSD NT
    case 0: return Launch<T, false, false, false, false>(p, g, stream); // DSD TN
    case 2: return Launch<T, false, false, true, false>(p, g, stream);  // DSD TT
    case 3: return Launch<T, false, false, true, true>(p, g, stream);   // DDS NN
    case 7: return Launch<T, false, true, true, true>(p, g, stream);    // DDS NT
    case 1: return Launch<T, false, false, false, true>(p, g, stream);  // DDS TN
    default: return Launch<T, false, true, false, true>(p, g, stream);  // DDS TT
  }
}

template <typename T>
hipError_t LaunchSparseIn(bool s_kc, bool d_kc, bool out_t,
                          const GemmParams &p, hipStream_t stream) {
  if (p.num_tiles <= 0) return hipSuccess;
  const int code = (s_kc ? 4 : 0) | (d_kc ? 2 : 0) | (out_t ? 1 : 0);
#define SPUTNIK_SS(SKC, DKC, OUTT)                                         \
  hipLaunchKernelGGL(                                                      \
      (block_gemm_kernel<T, true, SKC, DKC, OUTT, CfgSs, true>),       \
      dim3(p.num_tiles), dim3(64 * CfgSs::kWaves), 0,          \
      stream, p);                                                          \
  return hipGetLastError()
  switch (code) {
    case 4: SPUTNIK_SS(true, false, false);   // SSD NN
    case 6: SPUTNIK_SS(true, true, false);    // SSD NT
    case 0: SPUTNIK_SS(false, false, false);  // SSD TN
    case 2: SPUTNIK_SS(false, true, false);   // SSD TT
    case 3: SPUTNIK_SS(false, true, true);    // SDS NN
    case 7: SPUTNIK_SS(true, true, true);     // SDS NT
    case 1: SPUTNIK_SS(false, false, true);   // SDS TN
    default: SPUTNIK_SS(true, false, true);   // SDS TT
  }
#undef SPUTNIK_SS
}

template <typename T>
hipError_t LaunchDss(bool s_kc, bool d_kc, const GemmParams &p,
                     hipStream_t stream) {
  if (p.num_tiles <= 0) return hipSuccess;
#define SPUTNIK_DSS(SKC, DKC)                                              \
  hipLaunchKernelGGL(                                                      \
      (block_gemm_kernel<T, false, SKC, DKC, false, CfgDss, false,      \
                         true>),                                           \
      dim3(p.num_tiles), dim3(64 * CfgDss::kWaves), 0,     \
      stream, p);                                                          \
  return hipGetLastError()
  if (s_kc && !d_kc) { SPUTNIK_DSS(true, false); }    // DSS NN
  if (s_kc && d_kc) { SPUTNIK_DSS(true, true); }      // DSS NT
  if (!s_kc && !d_kc) { SPUTNIK_DSS(false, false); }  // DSS TN
  SPUTNIK_DSS(false, true);                           // DSS TT
#undef SPUTNIK_DSS
}

}  // namespace

hipError_t LaunchBlockGemmDss(int dtype, bool s_kc, bool d_kc,
                              const GemmParams &params, hipStream_t stream) {
  if (dtype == 1) return LaunchDss<__bf16>(s_kc, d_kc, params, stream);
  return LaunchDss<_Float16>(s_kc, d_kc, params, stream);
}

hipError_t LaunchBlockGemmSparseIn(int dtype, bool s_kc, bool d_kc, bool out_t,
                                   const GemmParams &params,
                                   hipStream_t stream) {
  if (dtype == 1)
    return LaunchSparseIn<__bf16>(s_kc, d_kc, out_t, params, stream);
  return LaunchSparseIn<_Float16>(s_kc, d_kc, out_t, params, stream);
}

hipError_t LaunchBlockGemm(int dtype, bool sparse_out, bool s_kc, bool d_kc,
                           bool out_t, bool grouped, const GemmParams &params,
                           hipStream_t stream) {
  if (dtype == 1)
    return LaunchTyped<__bf16>(sparse_out, s_kc, d_kc, out_t, grouped, params,
                               stream);
  return LaunchTyped<_Float16>(sparse_out, s_kc, d_kc, out_t, grouped, params,
                               stream);
}

}  // namespace sputnik_amd
