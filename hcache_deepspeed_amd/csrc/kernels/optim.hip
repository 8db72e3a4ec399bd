// Fused optimizers for gfx950: Adam/AdamW, Lion, LAMB, Adagrad; flat-shard and multi-tensor forms,
// plus the grad-norm / overflow reduction the ZeRO step needs.
//
// Capability parity: reference csrc/adam/multi_tensor_adam.cu (K1), csrc/lion/multi_tensor_lion.cu
// (K2), csrc/lamb/fused_lamb_cuda_kernel.cu (K3).
//
// MI355X-first design:
//   * ZeRO keeps every optimizer partition as ONE flat fp32 buffer, so the hot path is the flat
//     kernel: a grid-stride stream over [p32, m, v] (fp32) + g (bf16 or fp32), 16-byte accesses,
//     that also writes the bf16 working copy of the parameter in the same pass (no separate
//     fp32->bf16 cast kernel, no separate unscale/clip kernel: `gscale` and the optional
//     device-side `dev_scale` are folded into the gradient read).
//   * `found_inf` (device int, optional) turns the whole update into a no-op without a host sync
//     -- dynamic loss scaling never round-trips to the CPU on the fast path.
//   * the multi-tensor form (FusedAdam over arbitrary parameter lists) walks a device-resident
//     chunk table instead of the reference's fixed-depth kernel-argument struct, so one launch
//     covers any number of tensors.
#include <cstdlib>

#include "hds_common.h"

using namespace hds;

namespace {

struct AdamHP {
  float lr, b1, b2, eps, wd, bc1, bc2;  // bc = 1 - beta^t (bias corrections, 1 when disabled)
  int adamw;                            // 1: decoupled weight decay; 0: L2 added to the gradient
};

__device__ __forceinline__ float load_scale(float gscale, const float* dev_scale) {
  return dev_scale ? gscale * dev_scale[0] : gscale;
}

template <typename PT, typename GT>
__device__ __forceinline__ void adam_elem(float& p, float g, float& m, float& v, const AdamHP& h) {
  if (!h.adamw && h.wd != 0.f) g += h.wd * p;
  m = h.b1 * m + (1.f - h.b1) * g;
  v = h.b2 * v + (1.f - h.b2) * g * g;
  const float mh = m / h.bc1;
  const float denom = sqrtf(v / h.bc2) + h.eps;
  float upd = mh / denom;
  if (h.adamw && h.wd != 0.f) upd += h.wd * p;
  p -= h.lr * upd;
}

// NT (variant 1): the fp32 state and the bf16 copy are written with non-temporal (streaming) stores -- every byte the
// step writes is read again only in the next step, so allocating it in L2 only evicts the stream's read lines
__device__ __forceinline__ void st8_nt(float* p, const float (&v)[8]) {
  __builtin_nontemporal_store(f32x4{v[0], v[1], v[2], v[3]}, reinterpret_cast<f32x4*>(p));
  __builtin_nontemporal_store(f32x4{v[4], v[5], v[6], v[7]}, reinterpret_cast<f32x4*>(p + 4));
}
__device__ __forceinline__ void st8_nt(bf16* p, const float (&v)[8]) {
  bf16x8 r;
#pragma unroll
  for (int i = 0; i < 8; ++i) r[i] = (bf16)v[i];
  __builtin_nontemporal_store(*reinterpret_cast<u32x4*>(&r), reinterpret_cast<u32x4*>(p));
}

// p: master (PT = float or bf16), g: grad, m/v: fp32 state, lp: optional low-precision copy of p
template <typename PT, typename GT, bool NT = false>
__global__ __launch_bounds__(256) void adam_flat(PT* __restrict__ p, const GT* __restrict__ g, float* __restrict__ m,
                                                 float* __restrict__ v, bf16* __restrict__ lp, int64_t n, AdamHP h,
                                                 float gscale, const float* __restrict__ dev_scale,
                                                 const int* __restrict__ found_inf) {
  if (found_inf && *found_inf) return;
  const float sc = load_scale(gscale, dev_scale);
  const int64_t nvec = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    float pv[8], gv[8], mv[8], vv[8];
    Vec8<PT>::load(p + i * 8, pv);
    Vec8<GT>::load(g + i * 8, gv);
    Vec8<float>::load(m + i * 8, mv);
    Vec8<float>::load(v + i * 8, vv);
#pragma unroll
    for (int j = 0; j < 8; ++j) adam_elem<PT, GT>(pv[j], gv[j] * sc, mv[j], vv[j], h);
    if constexpr (NT) {
      st8_nt(p + i * 8, pv);
      st8_nt(m + i * 8, mv);
      st8_nt(v + i * 8, vv);
      if (lp) st8_nt(lp + i * 8, pv);
    } else {
      Vec8<PT>::store(p + i * 8, pv);
      Vec8<float>::store(m + i * 8, mv);
      Vec8<float>::store(v + i * 8, vv);
      if (lp) Vec8<bf16>::store(lp + i * 8, pv);
    }
  }
  // tail
  for (int64_t i = nvec * 8 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float pv = to_f(p[i]), mv = m[i], vv = v[i];
    adam_elem<PT, GT>(pv, to_f(g[i]) * sc, mv, vv, h);
    p[i] = from_f<PT>(pv);
    m[i] = mv;
    v[i] = vv;
    if (lp) lp[i] = (bf16)pv;
  }
}

// ---- multi-tensor chunk table ------------------------------------------------------------
// tensors: int64 [ntensors][6] = {p, g, m, v, lp, numel}
// chunks:  int64 [nchunks][2]  = {tensor index, start element}
constexpr int kChunk = 16384;

template <typename PT, typename GT>
__global__ __launch_bounds__(256) void adam_multi(const int64_t* __restrict__ tensors,
                                                  const int64_t* __restrict__ chunks, AdamHP h, float gscale,
                                                  const float* __restrict__ dev_scale,
                                                  const int* __restrict__ found_inf) {
  if (found_inf && *found_inf) return;
  const float sc = load_scale(gscale, dev_scale);
  const int64_t ti = chunks[blockIdx.x * 2], start = chunks[blockIdx.x * 2 + 1];
  const int64_t* t = tensors + ti * 6;
  PT* p = (PT*)t[0];
  const GT* g = (const GT*)t[1];
  float* m = (float*)t[2];
  float* v = (float*)t[3];
  bf16* lp = (bf16*)t[4];
  const int64_t n = t[5];
  const int64_t end = start + kChunk < n ? start + kChunk : n;
  // vector path when the chunk (and therefore all addresses) is 8-element aligned
  const bool vec_ok = ((end - start) % 8 == 0) && (((uintptr_t)p | (uintptr_t)g) % 16 == 0);
  if (vec_ok) {
    for (int64_t i = start + threadIdx.x * 8; i < end; i += 256 * 8) {
      float pv[8], gv[8], mv[8], vv[8];
      Vec8<PT>::load(p + i, pv);
      Vec8<GT>::load(g + i, gv);
      Vec8<float>::load(m + i, mv);
      Vec8<float>::load(v + i, vv);
#pragma unroll
      for (int j = 0; j < 8; ++j) adam_elem<PT, GT>(pv[j], gv[j] * sc, mv[j], vv[j], h);
      Vec8<PT>::store(p + i, pv);
      Vec8<float>::store(m + i, mv);
      Vec8<float>::store(v + i, vv);
      if (lp) Vec8<bf16>::store(lp + i, pv);
    }
  } else {
    for (int64_t i = start + threadIdx.x; i < end; i += 256) {
      float pv = to_f(p[i]), mv = m[i], vv = v[i];
      adam_elem<PT, GT>(pv, to_f(g[i]) * sc, mv, vv, h);
      p[i] = from_f<PT>(pv);
      m[i] = mv;
      v[i] = vv;
      if (lp) lp[i] = (bf16)pv;
    }
  }
}

// ---- Lion -------------------------------------------------------------------------------
template <typename PT, typename GT>
__global__ __launch_bounds__(256) void lion_flat(PT* __restrict__ p, const GT* __restrict__ g, float* __restrict__ m,
                                                 bf16* __restrict__ lp, int64_t n, float lr, float b1, float b2,
                                                 float wd, float gscale, const float* __restrict__ dev_scale,
                                                 const int* __restrict__ found_inf) {
  if (found_inf && *found_inf) return;
  const float sc = load_scale(gscale, dev_scale);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float pv = to_f(p[i]);
    const float gv = to_f(g[i]) * sc;
    float mv = m[i];
    const float c = b1 * mv + (1.f - b1) * gv;
    const float upd = (c > 0.f) ? 1.f : ((c < 0.f) ? -1.f : 0.f);
    pv = pv * (1.f - lr * wd) - lr * upd;
    mv = b2 * mv + (1.f - b2) * gv;
    p[i] = from_f<PT>(pv);
    m[i] = mv;
    if (lp) lp[i] = (bf16)pv;
  }
}

// ---- Adagrad ----------------------------------------------------------------------------
template <typename PT, typename GT>
__global__ __launch_bounds__(256) void adagrad_flat(PT* __restrict__ p, const GT* __restrict__ g,
                                                    float* __restrict__ s, bf16* __restrict__ lp, int64_t n, float lr,
                                                    float eps, float wd, float gscale,
                                                    const float* __restrict__ dev_scale,
                                                    const int* __restrict__ found_inf) {
  if (found_inf && *found_inf) return;
  const float sc = load_scale(gscale, dev_scale);
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    float pv = to_f(p[i]);
    float gv = to_f(g[i]) * sc + wd * pv;
    float sv = s[i] + gv * gv;
    pv -= lr * gv / (sqrtf(sv) + eps);
    p[i] = from_f<PT>(pv);
    s[i] = sv;
    if (lp) lp[i] = (bf16)pv;
  }
}

// ---- LAMB (per-tensor trust ratio over the multi-tensor table) ---------------------------
// phase 1: m, v update; u = mhat/(sqrt(vhat)+eps) + wd*p is recomputed in phase 2; accumulate
// ||p||^2 and ||u||^2 per tensor into norms[2*t], norms[2*t+1] (fp32 atomics, one per block).
template <typename PT, typename GT>
__global__ __launch_bounds__(256) void lamb_phase1(const int64_t* __restrict__ tensors,
                                                   const int64_t* __restrict__ chunks, AdamHP h, float gscale,
                                                   const float* __restrict__ dev_scale, float* __restrict__ norms,
                                                   const int* __restrict__ found_inf) {
  if (found_inf && *found_inf) return;
  __shared__ float red[4];
  const float sc = load_scale(gscale, dev_scale);
  const int64_t ti = chunks[blockIdx.x * 2], start = chunks[blockIdx.x * 2 + 1];
  const int64_t* t = tensors + ti * 6;
  const PT* p = (const PT*)t[0];
  const GT* g = (const GT*)t[1];
  float* m = (float*)t[2];
  float* v = (float*)t[3];
  const int64_t n = t[5];
  const int64_t end = start + kChunk < n ? start + kChunk : n;
  float pp = 0.f, uu = 0.f;
  for (int64_t i = start + threadIdx.x; i < end; i += 256) {
    const float pv = to_f(p[i]);
    const float gv = to_f(g[i]) * sc;
    const float mv = h.b1 * m[i] + (1.f - h.b1) * gv;
    const float vv = h.b2 * v[i] + (1.f - h.b2) * gv * gv;
    m[i] = mv;
    v[i] = vv;
    const float u = (mv / h.bc1) / (sqrtf(vv / h.bc2) + h.eps) + h.wd * pv;
    pp += pv * pv;
    uu += u * u;
  }
  pp = block_sum<256>(pp, red);
  uu = block_sum<256>(uu, red);
  if (threadIdx.x == 0) {
    atomicAdd(&norms[2 * ti], pp);
    atomicAdd(&norms[2 * ti + 1], uu);
  }
}

template <typename PT>
__global__ __launch_bounds__(256) void lamb_phase2(const int64_t* __restrict__ tensors,
                                                   const int64_t* __restrict__ chunks, AdamHP h,
                                                   const float* __restrict__ norms, float max_coeff, float min_coeff,
                                                   const int* __restrict__ found_inf) {
  if (found_inf && *found_inf) return;
  const int64_t ti = chunks[blockIdx.x * 2], start = chunks[blockIdx.x * 2 + 1];
  const int64_t* t = tensors + ti * 6;
  PT* p = (PT*)t[0];
  const float* m = (const float*)t[2];
  const float* v = (const float*)t[3];
  bf16* lp = (bf16*)t[4];
  const int64_t n = t[5];
  const int64_t end = start + kChunk < n ? start + kChunk : n;
  const float pn = sqrtf(norms[2 * ti]), un = sqrtf(norms[2 * ti + 1]);
  float trust = (pn > 0.f && un > 0.f) ? pn / un : 1.f;
  trust = fminf(fmaxf(trust, min_coeff), max_coeff);
  for (int64_t i = start + threadIdx.x; i < end; i += 256) {
    float pv = to_f(p[i]);
    const float u = (m[i] / h.bc1) / (sqrtf(v[i] / h.bc2) + h.eps) + h.wd * pv;
    pv -= h.lr * trust * u;
    p[i] = from_f<PT>(pv);
    if (lp) lp[i] = (bf16)pv;
  }
}

// ---- grad norm / overflow ------------------------------------------------------------------
// out[0] += sum(x^2) (fp32 atomics, one per block);  found_inf[0] |= any non-finite
template <typename T>
__global__ __launch_bounds__(256) void sumsq_kernel(const T* __restrict__ x, int64_t n, float* __restrict__ out,
                                                    int* __restrict__ found_inf) {
  __shared__ float red[4];
  float s = 0.f;
  int bad = 0;
  const int64_t nvec = n / 8;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < nvec; i += (int64_t)gridDim.x * 256) {
    float v[8];
    Vec8<T>::load(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s += v[j] * v[j];
      bad |= !isfinite(v[j]);
    }
  }
  for (int64_t i = nvec * 8 + (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
    const float v = to_f(x[i]);
    s += v * v;
    bad |= !isfinite(v);
  }
  s = block_sum<256>(s, red);
  const int anybad = __syncthreads_or(bad);
  if (threadIdx.x == 0) {
    atomicAdd(out, s);
    if (anybad && found_inf) atomicOr(found_inf, 1);
  }
}

// coef = min(1, max_norm / (sqrt(sumsq_total) + 1e-6)) * inv_scale  -> dev_scale[0]
__global__ void clip_coef_kernel(const float* __restrict__ sumsq, float max_norm, float inv_scale,
                                 float* __restrict__ coef, float* __restrict__ norm_out) {
  const float nrm = sqrtf(sumsq[0]) * inv_scale;
  if (norm_out) norm_out[0] = nrm;
  float c = inv_scale;
  if (max_norm > 0.f) {
    const float k = max_norm / (nrm + 1e-6f);
    if (k < 1.f) c *= k;
  }
  coef[0] = c;
}

}  // namespace

#define PG_SWITCH(pdtype, gdtype, BODY)                                                            \
  if (pdtype == kF32 && gdtype == kF32) {                                                          \
    typedef float PT;                                                                              \
    typedef float GT;                                                                              \
    BODY;                                                                                          \
  } else if (pdtype == kF32 && gdtype == kBF16) {                                                  \
    typedef float PT;                                                                              \
    typedef bf16 GT;                                                                               \
    BODY;                                                                                          \
  } else if (pdtype == kBF16 && gdtype == kBF16) {                                                 \
    typedef bf16 PT;                                                                               \
    typedef bf16 GT;                                                                               \
    BODY;                                                                                          \
  } else if (pdtype == kBF16 && gdtype == kF32) {                                                  \
    typedef bf16 PT;                                                                               \
    typedef float GT;                                                                              \
    BODY;                                                                                          \
  } else if (pdtype == kF32 && gdtype == kF16) {                                                   \
    typedef float PT;                                                                              \
    typedef _Float16 GT;                                                                           \
    BODY;                                                                                          \
  } else {                                                                                         \
    return hipErrorInvalidValue;                                                                   \
  }

HDS_EXPORT int hds_adam_flat(int pdtype, int gdtype, void* p, const void* g, float* m, float* v, void* lp, int64_t n,
                             float lr, float b1, float b2, float eps, float wd, float bc1, float bc2, int adamw,
                             float gscale, const float* dev_scale, const int* found_inf, hipStream_t st) {
  AdamHP h{lr, b1, b2, eps, wd, bc1, bc2, adamw};
  dim3 grid(stream_grid(n / 8 + 1, 256, 4096)), block(256);
  static const int nt = [] {
    const char* e = getenv("HDS_ADAM_NT");
    return e ? atoi(e) : 0;
  }();
  if (nt && pdtype == kF32) {  // fp32 master: the training configuration
    PG_SWITCH(pdtype, gdtype,
              hipLaunchKernelGGL((adam_flat<PT, GT, true>), grid, block, 0, st, (PT*)p, (const GT*)g, m, v,
                                 (bf16*)lp, n, h, gscale, dev_scale, found_inf));
  } else {
    PG_SWITCH(pdtype, gdtype,
              hipLaunchKernelGGL((adam_flat<PT, GT>), grid, block, 0, st, (PT*)p, (const GT*)g, m, v, (bf16*)lp, n,
                                 h, gscale, dev_scale, found_inf));
  }
  return hipGetLastError();
}

HDS_EXPORT int hds_multi_chunk_size() { return kChunk; }

HDS_EXPORT int hds_adam_multi(int pdtype, int gdtype, const int64_t* tensors, const int64_t* chunks, int nchunks,
                              float lr, float b1, float b2, float eps, float wd, float bc1, float bc2, int adamw,
                              float gscale, const float* dev_scale, const int* found_inf, hipStream_t st) {
  if (nchunks <= 0) return 0;
  AdamHP h{lr, b1, b2, eps, wd, bc1, bc2, adamw};
  PG_SWITCH(pdtype, gdtype,
            hipLaunchKernelGGL((adam_multi<PT, GT>), dim3(nchunks), dim3(256), 0, st, tensors, chunks, h, gscale,
                               dev_scale, found_inf));
  return hipGetLastError();
}

HDS_EXPORT int hds_lion_flat(int pdtype, int gdtype, void* p, const void* g, float* m, void* lp, int64_t n, float lr,
                             float b1, float b2, float wd, float gscale, const float* dev_scale, const int* found_inf,
                             hipStream_t st) {
  dim3 grid(stream_grid(n, 256, 4096)), block(256);
  PG_SWITCH(pdtype, gdtype,
            hipLaunchKernelGGL((lion_flat<PT, GT>), grid, block, 0, st, (PT*)p, (const GT*)g, m, (bf16*)lp, n, lr, b1,
                               b2, wd, gscale, dev_scale, found_inf));
  return hipGetLastError();
}

HDS_EXPORT int hds_adagrad_flat(int pdtype, int gdtype, void* p, const void* g, float* s, void* lp, int64_t n,
                                float lr, float eps, float wd, float gscale, const float* dev_scale,
                                const int* found_inf, hipStream_t st) {
  dim3 grid(stream_grid(n, 256, 4096)), block(256);
  PG_SWITCH(pdtype, gdtype,
            hipLaunchKernelGGL((adagrad_flat<PT, GT>), grid, block, 0, st, (PT*)p, (const GT*)g, s, (bf16*)lp, n, lr,
                               eps, wd, gscale, dev_scale, found_inf));
  return hipGetLastError();
}

HDS_EXPORT int hds_lamb_multi(int pdtype, int gdtype, const int64_t* tensors, const int64_t* chunks, int nchunks,
                              float* norms, float lr, float b1, float b2, float eps, float wd, float bc1, float bc2,
                              float max_coeff, float min_coeff, float gscale, const float* dev_scale,
                              const int* found_inf, hipStream_t st) {
  if (nchunks <= 0) return 0;
  AdamHP h{lr, b1, b2, eps, wd, bc1, bc2, 1};
  PG_SWITCH(pdtype, gdtype, {
    hipLaunchKernelGGL((lamb_phase1<PT, GT>), dim3(nchunks), dim3(256), 0, st, tensors, chunks, h, gscale, dev_scale,
                       norms, found_inf);
    hipLaunchKernelGGL((lamb_phase2<PT>), dim3(nchunks), dim3(256), 0, st, tensors, chunks, h, norms, max_coeff,
                       min_coeff, found_inf);
  });
  return hipGetLastError();
}

HDS_EXPORT int hds_sumsq(int dtype, const void* x, int64_t n, float* out, int* found_inf, hipStream_t st) {
  dim3 grid(stream_grid(n / 8 + 1, 256, 1024)), block(256);
  if (dtype == kF32)
    hipLaunchKernelGGL(sumsq_kernel<float>, grid, block, 0, st, (const float*)x, n, out, found_inf);
  else if (dtype == kBF16)
    hipLaunchKernelGGL(sumsq_kernel<bf16>, grid, block, 0, st, (const bf16*)x, n, out, found_inf);
  else if (dtype == kF16)
    hipLaunchKernelGGL(sumsq_kernel<_Float16>, grid, block, 0, st, (const _Float16*)x, n, out, found_inf);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

HDS_EXPORT int hds_clip_coef(const float* sumsq, float max_norm, float inv_scale, float* coef, float* norm_out,
                             hipStream_t st) {
  hipLaunchKernelGGL(clip_coef_kernel, dim3(1), dim3(1), 0, st, sumsq, max_norm, inv_scale, coef, norm_out);
  return hipGetLastError();
}
