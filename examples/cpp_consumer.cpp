// A C++ caller written against the reference's public API, the way
// MegaBlocks' extension or the reference's own tests drive it
// (sputnik/block/dsd/dsd_test.cu, sdd_test.cu): only `#include
// "sputnik/sputnik.h"`, `sputnik::block` descriptors and overloads, caller-
// owned device buffers, hipError_t return codes. Built against
// libsputnik.so by sputnik_amd/Makefile; tests/test_cpp_consumer.py runs it
// on the GPU. It checks DSD NN, DSD TN through MatmulEx + Transpose, and SDD
// with RowIndices against a host loop (double accumulation of fp16 inputs)
// and prints one line per check; exit status 0 = all passed.
#include <hip/hip_fp16.h>
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <random>
#include <vector>

#include "sputnik/sputnik.h"

namespace sb = sputnik::block;

#define CHECK_HIP(x)                                                   \
  do {                                                                 \
    hipError_t e_ = (x);                                               \
    if (e_ != hipSuccess) {                                            \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__,           \
                   hipGetErrorString(e_));                             \
      std::exit(2);                                                    \
    }                                                                  \
  } while (0)

namespace {

constexpr int kB = 128;

struct Bcsr {
  int rows, cols;
  std::vector<int> offsets;
  std::vector<short> indices;
  std::vector<float> values;  // fp16-representable, block-major
};

float RoundF16(float x) { return __half2float(__float2half(x)); }

Bcsr RandomBcsr(int rows, int cols, double density, std::mt19937 &gen) {
  Bcsr m{rows, cols, {0}, {}, {}};
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  std::bernoulli_distribution keep(density);
  for (int r = 0; r < rows / kB; ++r) {
    for (int c = 0; c < cols / kB; ++c)
      if (keep(gen)) m.indices.push_back(static_cast<short>(c));
    m.offsets.push_back(static_cast<int>(m.indices.size()));
  }
  m.values.resize(m.indices.size() * kB * kB);
  for (auto &v : m.values) v = RoundF16(u(gen));
  return m;
}

std::vector<float> Dense(const Bcsr &m) {
  std::vector<float> d(static_cast<size_t>(m.rows) * m.cols, 0.f);
  for (int r = 0; r < m.rows / kB; ++r)
    for (int e = m.offsets[r]; e < m.offsets[r + 1]; ++e)
      for (int i = 0; i < kB; ++i)
        for (int j = 0; j < kB; ++j)
          d[(size_t)(r * kB + i) * m.cols + m.indices[e] * kB + j] =
              m.values[(size_t)e * kB * kB + i * kB + j];
  return d;
}

template <typename T>
T *ToDevice(const std::vector<T> &h) {
  T *d = nullptr;
  CHECK_HIP(hipMalloc(&d, std::max<size_t>(h.size(), 1) * sizeof(T)));
  if (!h.empty())
    CHECK_HIP(hipMemcpy(d, h.data(), h.size() * sizeof(T),
                        hipMemcpyHostToDevice));
  return d;
}

__half *HalfToDevice(const std::vector<float> &h) {
  std::vector<__half> t(h.size());
  for (size_t i = 0; i < h.size(); ++i) t[i] = __float2half(h[i]);
  return ToDevice(t);
}

std::vector<float> HalfFromDevice(const __half *d, size_t n) {
  std::vector<__half> t(n);
  CHECK_HIP(hipMemcpy(t.data(), d, n * sizeof(__half), hipMemcpyDeviceToHost));
  std::vector<float> h(n);
  for (size_t i = 0; i < n; ++i) h[i] = __half2float(t[i]);
  return h;
}

// C[m x n] = op(A)[m x k] * B[k x n], A given densely as stored (ta: k x m).
std::vector<double> HostGemm(const std::vector<float> &a, bool ta, int m,
                             int k, const std::vector<float> &b, int n) {
  std::vector<double> c((size_t)m * n, 0.0);
  for (int i = 0; i < m; ++i)
    for (int l = 0; l < k; ++l) {
      const double av = ta ? a[(size_t)l * m + i] : a[(size_t)i * k + l];
      if (av == 0.0) continue;
      for (int j = 0; j < n; ++j) c[(size_t)i * n + j] += av * b[(size_t)l * n + j];
    }
  return c;
}

// |gpu - ref| <= 1e-2 (|ref| + rms(ref)), the north-star fp16 tolerance.
bool Close(const std::vector<float> &gpu, const std::vector<double> &ref,
           const char *what) {
  double ss = 0;
  for (double r : ref) ss += r * r;
  const double rms = std::sqrt(ss / std::max<size_t>(ref.size(), 1));
  size_t bad = 0;
  for (size_t i = 0; i < ref.size(); ++i)
    if (!(std::fabs(gpu[i] - ref[i]) <= 1e-2 * (std::fabs(ref[i]) + rms))) ++bad;
  std::printf("%s: %s (%zu of %zu out of tolerance)\n", what,
              bad ? "FAIL" : "ok", bad, ref.size());
  return bad == 0;
}

}  // namespace

int main() {
  std::mt19937 gen(7);
  std::uniform_real_distribution<float> u(-1.f, 1.f);
  hipStream_t stream;
  CHECK_HIP(hipStreamCreate(&stream));
  bool ok = true;
  const int m = 512, k = 768, n = 264;

  // ---- DSD NN: C = A B ------------------------------------------------
  Bcsr a = RandomBcsr(m, k, 0.4, gen);
  std::vector<float> b((size_t)k * n);
  for (auto &v : b) v = RoundF16(u(gen));
  __half *d_a = HalfToDevice(a.values), *d_b = HalfToDevice(b);
  int *d_off = ToDevice(a.offsets);
  short *d_idx = ToDevice(a.indices);
  __half *d_c = nullptr;
  CHECK_HIP(hipMalloc(&d_c, (size_t)m * n * sizeof(__half)));
  sb::BlockMatrix sa(m, k, sb::AsBlockSize(kB),
                     static_cast<int>(a.indices.size()) * kB * kB, d_a, d_off,
                     d_idx);
  sb::Matrix mb(k, n, d_b), mc(m, n, d_c);
  CHECK_HIP(sb::Matmul(sa, false, mb, false, mc, stream));
  CHECK_HIP(hipStreamSynchronize(stream));
  ok &= Close(HalfFromDevice(d_c, (size_t)m * n),
              HostGemm(Dense(a), false, m, k, b, n), "dsd nn");

  // ---- DSD TN through MatmulEx: C' = A^T B', transposed metadata built
  // once with Transpose (the MegaBlocks backward pattern) -----------------
  std::vector<float> b2((size_t)m * n);
  for (auto &v : b2) v = RoundF16(u(gen));
  __half *d_b2 = HalfToDevice(b2), *d_c2 = nullptr;
  CHECK_HIP(hipMalloc(&d_c2, (size_t)k * n * sizeof(__half)));
  sb::AllocateTransposeBuffers(sa);
  CHECK_HIP(sb::Transpose(sa, stream));
  sb::Matrix mb2(m, n, d_b2), mc2(k, n, d_c2);
  CHECK_HIP(sb::MatmulEx(sa, true, mb2, false, mc2, stream));
  CHECK_HIP(hipStreamSynchronize(stream));
  ok &= Close(HalfFromDevice(d_c2, (size_t)k * n),
              HostGemm(Dense(a), true, k, m, b2, n), "dsd tn (MatmulEx)");

  // ---- SDD: C_bcsr = X W at C's blocks, RowIndices first -----------------
  Bcsr topo = RandomBcsr(m, 384, 0.5, gen);
  std::vector<float> x((size_t)m * k), w((size_t)k * 384);
  for (auto &v : x) v = RoundF16(u(gen));
  for (auto &v : w) v = RoundF16(u(gen));
  __half *d_x = HalfToDevice(x), *d_w = HalfToDevice(w);
  const int nb = static_cast<int>(topo.indices.size());
  __half *d_s = nullptr;
  CHECK_HIP(hipMalloc(&d_s, std::max(nb, 1) * kB * kB * sizeof(__half)));
  int *d_toff = ToDevice(topo.offsets);
  short *d_tidx = ToDevice(topo.indices);
  sb::BlockMatrix sc(m, 384, sb::AsBlockSize(kB), nb * kB * kB, d_s, d_toff,
                     d_tidx);
  sb::AllocateRowIndicesBuffer(sc);
  CHECK_HIP(sb::RowIndices(sc, static_cast<short *>(sc.row_indices), stream));
  sb::Matrix mx(m, k, d_x), mw(k, 384, d_w);
  CHECK_HIP(sb::Matmul(mx, false, mw, false, sc, stream));
  CHECK_HIP(hipStreamSynchronize(stream));
  const std::vector<double> full = HostGemm(x, false, m, k, w, 384);
  std::vector<double> ref_blocks;
  for (int r = 0; r < m / kB; ++r)
    for (int e = topo.offsets[r]; e < topo.offsets[r + 1]; ++e)
      for (int i = 0; i < kB; ++i)
        for (int j = 0; j < kB; ++j)
          ref_blocks.push_back(
              full[(size_t)(r * kB + i) * 384 + topo.indices[e] * kB + j]);
  ok &= Close(HalfFromDevice(d_s, (size_t)nb * kB * kB), ref_blocks, "sdd");

  // ---- error convention: block size 64 is not supported (dsd.cu:16) -----
  sb::BlockMatrix s64 = sa;
  s64.block_size = sb::AsBlockSize(64);
  const bool rc_ok = sb::Matmul(s64, false, mb, false, mc, stream) ==
                     hipErrorNotSupported;
  std::printf("block 64 -> hipErrorNotSupported: %s\n", rc_ok ? "ok" : "FAIL");
  ok &= rc_ok;

  sb::FreeTransposeBuffers(sa);
  sb::FreeRowIndicesBuffer(sc);
  for (void *p : {(void *)d_a, (void *)d_b, (void *)d_off, (void *)d_idx,
                  (void *)d_c, (void *)d_b2, (void *)d_c2, (void *)d_x,
                  (void *)d_w, (void *)d_s, (void *)d_toff, (void *)d_tidx})
    CHECK_HIP(hipFree(p));
  CHECK_HIP(hipStreamDestroy(stream));
  std::printf("%s\n", ok ? "ALL OK" : "FAILED");
  return ok ? 0 : 1;
}
