// Host-side optimizers for ZeRO-Offload: Adam/AdamW, Lion, Adagrad over fp32 master partitions.
//
// Capability parity: reference csrc/adam/cpu_adam_impl.cpp + csrc/includes/cpu_adam.h (AVX-512/AVX2 +
// OpenMP, TILE 128M), csrc/lion/cpu_lion*.cpp and csrc/adagrad/cpu_adagrad.cpp (N5).
//
// Design: straight-line loops the compiler vectorises for each `target_clones` ISA (AVX-512 on EPYC
// Zen4/5 hosts of MI355X nodes, AVX2 fallback), OpenMP static schedule over cache-sized tiles.
// Gradients may be fp32 or bf16 (the dtype RCCL reduced them in); the updated parameter can be written
// back as bf16 straight into a pinned staging buffer that feeds the H2D copy -- no extra cast pass.
#include <omp.h>

#include <cmath>
#include <cstdint>
#include <cstring>

#define HDS_EXPORT extern "C" __attribute__((visibility("default")))
#define HDS_CLONES __attribute__((target_clones("avx512f", "avx2", "default")))

namespace {

inline float bf16_to_f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  std::memcpy(&f, &u, 4);
  return f;
}

inline uint16_t f_to_bf16(float f) {
  uint32_t u;
  std::memcpy(&u, &f, 4);
  if ((u & 0x7f800000u) == 0x7f800000u && (u & 0x7fffffu)) return (uint16_t)((u >> 16) | 0x40);  // NaN
  u += 0x7fffu + ((u >> 16) & 1u);  // round to nearest even
  return (uint16_t)(u >> 16);
}

constexpr int64_t kTile = 1 << 20;

// Process-wide thread count of the host kernels (0: OpenMP's default). omp_set_num_threads() only sets the CALLING
// thread's ICV, and the kernels are called from the training thread and from copy-pipeline worker threads alike, so
// every parallel region names its count explicitly.
int g_threads = 0;
inline int nthreads() { return g_threads > 0 ? g_threads : omp_get_max_threads(); }

}  // namespace

// gdtype: 0 fp32, 1 bf16. out_bf16 may be null.
HDS_CLONES HDS_EXPORT int hds_cpu_adam(float* p, const void* g, int gdtype, float* m, float* v, uint16_t* out_bf16,
                                       int64_t n, float lr, float b1, float b2, float eps, float wd, float bc1,
                                       float bc2, int adamw, float gscale) {
  const float step_size = lr / bc1;
  const float inv_sqrt_bc2 = 1.0f / std::sqrt(bc2);
#pragma omp parallel for schedule(static) num_threads(nthreads())
  for (int64_t t0 = 0; t0 < n; t0 += kTile) {
    const int64_t t1 = t0 + kTile < n ? t0 + kTile : n;
    if (gdtype == 0) {
      const float* gf = (const float*)g;
#pragma omp simd
      for (int64_t i = t0; i < t1; ++i) {
        float gi = gf[i] * gscale;
        float pi = p[i];
        if (!adamw && wd != 0.f) gi += wd * pi;
        const float mi = b1 * m[i] + (1.f - b1) * gi;
        const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
        m[i] = mi;
        v[i] = vi;
        float upd = mi / (std::sqrt(vi) * inv_sqrt_bc2 + eps);
        if (adamw && wd != 0.f) pi -= lr * wd * pi;
        pi -= step_size * upd;
        p[i] = pi;
      }
    } else {
      const uint16_t* gh = (const uint16_t*)g;
#pragma omp simd
      for (int64_t i = t0; i < t1; ++i) {
        float gi = bf16_to_f(gh[i]) * gscale;
        float pi = p[i];
        if (!adamw && wd != 0.f) gi += wd * pi;
        const float mi = b1 * m[i] + (1.f - b1) * gi;
        const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
        m[i] = mi;
        v[i] = vi;
        float upd = mi / (std::sqrt(vi) * inv_sqrt_bc2 + eps);
        if (adamw && wd != 0.f) pi -= lr * wd * pi;
        pi -= step_size * upd;
        p[i] = pi;
      }
    }
    if (out_bf16) {
      for (int64_t i = t0; i < t1; ++i) out_bf16[i] = f_to_bf16(p[i]);
    }
  }
  return 0;
}

HDS_CLONES HDS_EXPORT int hds_cpu_lion(float* p, const void* g, int gdtype, float* m, uint16_t* out_bf16, int64_t n,
                                       float lr, float b1, float b2, float wd, float gscale) {
#pragma omp parallel for schedule(static) num_threads(nthreads())
  for (int64_t t0 = 0; t0 < n; t0 += kTile) {
    const int64_t t1 = t0 + kTile < n ? t0 + kTile : n;
    for (int64_t i = t0; i < t1; ++i) {
      const float gi = (gdtype == 0 ? ((const float*)g)[i] : bf16_to_f(((const uint16_t*)g)[i])) * gscale;
      const float c = b1 * m[i] + (1.f - b1) * gi;
      const float s = c > 0.f ? 1.f : (c < 0.f ? -1.f : 0.f);
      float pi = p[i] * (1.f - lr * wd) - lr * s;
      m[i] = b2 * m[i] + (1.f - b2) * gi;
      p[i] = pi;
      if (out_bf16) out_bf16[i] = f_to_bf16(pi);
    }
  }
  return 0;
}

HDS_CLONES HDS_EXPORT int hds_cpu_adagrad(float* p, const void* g, int gdtype, float* s, uint16_t* out_bf16,
                                          int64_t n, float lr, float eps, float wd, float gscale) {
#pragma omp parallel for schedule(static) num_threads(nthreads())
  for (int64_t t0 = 0; t0 < n; t0 += kTile) {
    const int64_t t1 = t0 + kTile < n ? t0 + kTile : n;
    for (int64_t i = t0; i < t1; ++i) {
      float gi = (gdtype == 0 ? ((const float*)g)[i] : bf16_to_f(((const uint16_t*)g)[i])) * gscale;
      gi += wd * p[i];
      s[i] += gi * gi;
      const float pi = p[i] - lr * gi / (std::sqrt(s[i]) + eps);
      p[i] = pi;
      if (out_bf16) out_bf16[i] = f_to_bf16(pi);
    }
  }
  return 0;
}

// sum of squares + non-finite flag over a host gradient partition (for clipping under offload)
HDS_CLONES HDS_EXPORT double hds_cpu_sumsq(const void* g, int gdtype, int64_t n, int* found_inf) {
  double acc = 0.0;
  int bad = 0;
#pragma omp parallel for reduction(+ : acc) reduction(| : bad) schedule(static) num_threads(nthreads())
  for (int64_t i = 0; i < n; ++i) {
    const float x = gdtype == 0 ? ((const float*)g)[i] : bf16_to_f(((const uint16_t*)g)[i]);
    acc += (double)x * x;
    bad |= !std::isfinite(x);
  }
  if (found_inf) *found_inf |= bad;
  return acc;
}

HDS_EXPORT int hds_cpu_num_threads() { return nthreads(); }

HDS_EXPORT int hds_cpu_set_num_threads(int n) {
  g_threads = n > 0 ? n : 0;
  if (n > 0) omp_set_num_threads(n);
  return 0;
}
