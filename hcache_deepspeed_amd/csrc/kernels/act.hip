// Gated activations (SwiGLU / GeGLU / ReGLU) and plain bias+activation, forward and backward.
//
// Capability parity: reference deepspeed/inference/v2/kernels/core_ops/gated_activations
// (`gated_activation_kernel`), bias_activations (K28), and the training
// GeLU of csrc/transformer/gelu_kernels.cu (K6). The reference has no training SwiGLU; the
// Llama/Mixtral training path here needs fwd+bwd.
//
// Layout: gate/up are the two halves of ONE fused GEMM output row [T, 2I] (gate first), so
// the MLP runs one GEMM for W1|W3 and this kernel reads both halves with 16-byte loads.
// Backward writes dgate|dup into the same [T, 2I] layout, which is what the fused GEMM's
// backward consumes, so no cat/split copies exist anywhere in the MLP.
#include <cstdlib>

#include "hds_common.h"

using namespace hds;

namespace {

enum Act : int { kSilu = 0, kGeluTanh = 1, kRelu = 2, kGeluErf = 3, kIdentity = 4 };

template <int A>
__device__ __forceinline__ float act_f(float x) {
  if constexpr (A == kSilu) return x * __builtin_amdgcn_rcpf(1.f + __expf(-x));
  if constexpr (A == kGeluTanh) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    return 0.5f * x * (1.f + tanhf(k0 * (x + k1 * x * x * x)));
  }
  if constexpr (A == kRelu) return fmaxf(x, 0.f);
  if constexpr (A == kGeluErf) return 0.5f * x * (1.f + erff(x * 0.7071067811865476f));
  return x;
}
template <int A>
__device__ __forceinline__ float act_grad(float x) {
  if constexpr (A == kSilu) {
    const float s = __builtin_amdgcn_rcpf(1.f + __expf(-x));
    return s * (1.f + x * (1.f - s));
  }
  if constexpr (A == kGeluTanh) {
    const float k0 = 0.7978845608028654f, k1 = 0.044715f;
    const float inner = k0 * (x + k1 * x * x * x);
    const float t = tanhf(inner);
    return 0.5f * (1.f + t) + 0.5f * x * (1.f - t * t) * k0 * (1.f + 3.f * k1 * x * x);
  }
  if constexpr (A == kRelu) return x > 0.f ? 1.f : 0.f;
  if constexpr (A == kGeluErf) {
    const float cdf = 0.5f * (1.f + erff(x * 0.7071067811865476f));
    const float pdf = 0.3989422804014327f * __expf(-0.5f * x * x);
    return cdf + x * pdf;
  }
  return 1.f;
}

// act(x) and act'(x) together: SiLU shares one exp + one v_rcp between value and derivative (the
// backward is VALU-bound at Llama MLP sizes, so the precise-division sigmoid was the hot spot).
template <int A>
__device__ __forceinline__ void act_val_grad(float x, float& a, float& g) {
  if constexpr (A == kSilu) {
    const float s = __builtin_amdgcn_rcpf(1.f + __expf(-x));
    a = x * s;
    g = s * (1.f + x * (1.f - s));
  } else {
    a = act_f<A>(x);
    g = act_grad<A>(x);
  }
}

// Flat vector index -> (row, column) with 32-bit division when the problem fits (the 64-bit
// division is a ~40-instruction software sequence per 8 elements).
__device__ __forceinline__ void split_idx(int64_t idx, int vpr, bool small, int64_t& r, int& c) {
  if (small) {
    const unsigned q = (unsigned)idx / (unsigned)vpr;
    r = q;
    c = (int)((unsigned)idx - q * (unsigned)vpr) * 8;
  } else {
    r = idx / vpr;
    c = (int)(idx - r * vpr) * 8;
  }
}

// y[t, i] = act(g[t, i]) * u[t, i]     g = gu[t, 0:I], u = gu[t, I:2I]
template <typename T, int A>
__global__ __launch_bounds__(256) void glu_fwd(const T* __restrict__ gu, T* __restrict__ y, int64_t rows, int I) {
  const int vpr = I / 8;
  const int64_t total = rows * vpr;
  const bool small = total < (int64_t)0x7fffffff;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    int64_t r;
    int c;
    split_idx(idx, vpr, small, r, c);
    float g[8], u[8], o[8];
    Vec8<T>::load(gu + r * 2 * I + c, g);
    Vec8<T>::load(gu + r * 2 * I + I + c, u);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = act_f<A>(g[j]) * u[j];
    Vec8<T>::store(y + r * I + c, o);
  }
}

template <typename T, int A>
__global__ __launch_bounds__(256) void glu_bwd(const T* __restrict__ dy, const T* __restrict__ gu,
                                               T* __restrict__ dgu, int64_t rows, int I) {
  const int vpr = I / 8;
  const int64_t total = rows * vpr;
  const bool small = total < (int64_t)0x7fffffff;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    int64_t r;
    int c;
    split_idx(idx, vpr, small, r, c);
    float g[8], u[8], d[8], dg[8], du[8];
    Vec8<T>::load(gu + r * 2 * I + c, g);
    Vec8<T>::load(gu + r * 2 * I + I + c, u);
    Vec8<T>::load(dy + r * I + c, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      float a, ga;
      act_val_grad<A>(g[j], a, ga);
      du[j] = d[j] * a;
      dg[j] = d[j] * u[j] * ga;
    }
    Vec8<T>::store(dgu + r * 2 * I + c, dg);
    Vec8<T>::store(dgu + r * 2 * I + I + c, du);
  }
}

// v2 of the gated kernels: two independent 16-B vectors per thread per grid-stride iteration, every load of both
// issued before any math (twice the bytes in flight per wave: the v1 loop is one dependent load -> math -> store
// chain per iteration and sat at ~5.1-5.4 TB/s). `total` vectors of 8; the tail iteration guards the second vector.
template <typename T, int A>
__global__ __launch_bounds__(256) void glu_fwd2(const T* __restrict__ gu, T* __restrict__ y, int64_t rows, int I) {
  const int vpr = I / 8;
  const int64_t total = rows * vpr;
  const bool small = total < (int64_t)0x7fffffff;
  const int64_t stride = (int64_t)gridDim.x * 512;
  for (int64_t i0 = (int64_t)blockIdx.x * 512 + threadIdx.x; i0 < total; i0 += stride) {
    const int64_t i1 = i0 + 256;
    const bool has1 = i1 < total;
    int64_t r0, r1;
    int c0, c1;
    split_idx(i0, vpr, small, r0, c0);
    split_idx(has1 ? i1 : i0, vpr, small, r1, c1);
    float g0[8], u0[8], g1[8], u1[8], o[8];
    Vec8<T>::load(gu + r0 * 2 * I + c0, g0);
    Vec8<T>::load(gu + r0 * 2 * I + I + c0, u0);
    Vec8<T>::load(gu + r1 * 2 * I + c1, g1);
    Vec8<T>::load(gu + r1 * 2 * I + I + c1, u1);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = act_f<A>(g0[j]) * u0[j];
    Vec8<T>::store(y + r0 * I + c0, o);
    if (has1) {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = act_f<A>(g1[j]) * u1[j];
      Vec8<T>::store(y + r1 * I + c1, o);
    }
  }
}

template <typename T, int A>
__global__ __launch_bounds__(256) void glu_bwd2(const T* __restrict__ dy, const T* __restrict__ gu,
                                                T* __restrict__ dgu, int64_t rows, int I) {
  const int vpr = I / 8;
  const int64_t total = rows * vpr;
  const bool small = total < (int64_t)0x7fffffff;
  const int64_t stride = (int64_t)gridDim.x * 512;
  for (int64_t i0 = (int64_t)blockIdx.x * 512 + threadIdx.x; i0 < total; i0 += stride) {
    const int64_t i1 = i0 + 256;
    const bool has1 = i1 < total;
    int64_t r[2];
    int c[2];
    split_idx(i0, vpr, small, r[0], c[0]);
    split_idx(has1 ? i1 : i0, vpr, small, r[1], c[1]);
    float g[2][8], u[2][8], d[2][8];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      Vec8<T>::load(gu + r[k] * 2 * I + c[k], g[k]);
      Vec8<T>::load(gu + r[k] * 2 * I + I + c[k], u[k]);
      Vec8<T>::load(dy + r[k] * I + c[k], d[k]);
    }
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      if (k == 1 && !has1) break;
      float dg[8], du[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a, ga;
        act_val_grad<A>(g[k][j], a, ga);
        du[j] = d[k][j] * a;
        dg[j] = d[k][j] * u[k][j] * ga;
      }
      Vec8<T>::store(dgu + r[k] * 2 * I + c[k], dg);
      Vec8<T>::store(dgu + r[k] * 2 * I + I + c[k], du);
    }
  }
}

// SwiGLU-family backward that ALSO writes the transposed gradient dguT [2I, rows] (bf16): the gate|up weight
// gradient runs hipBLASLt's NT form on dguT (ops/gemm.wgrad "nt"), which otherwise needs a separate HBM transpose of
// the [rows, 2I] gradient (read + write of 2 x rows x I x 2 B). Block = 64 rows x 128 columns of I: the dg / du tiles
// go to HBM row-major as in glu_bwd and through LDS (16-B writes, 8-B reads + v_perm, as transpose.hip v2) to their
// transposed rows i and I + i. rows % 8 == 0, I % 8 == 0.
constexpr int GT_R = 64, GT_C = 128;

template <int A>
__global__ __launch_bounds__(256) void glu_bwd_t(const bf16* __restrict__ dy, const bf16* __restrict__ gu,
                                                 bf16* __restrict__ dgu, bf16* __restrict__ dgut, int rows, int I) {
  __shared__ __attribute__((aligned(16))) bf16 tile[2][GT_R * GT_C];
  const int r0 = blockIdx.y * GT_R, c0 = blockIdx.x * GT_C;
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int v = tid + 256 * k, rr = v >> 4, cc = (v & 15) * 8;
    const int r = r0 + rr, c = c0 + cc;
    float dg[8], du[8];
    if (r < rows && c < I) {  // I % 8 == 0: a vector is all in or all out
      float g[8], u[8], d[8];
      Vec8<bf16>::load(gu + (int64_t)r * 2 * I + c, g);
      Vec8<bf16>::load(gu + (int64_t)r * 2 * I + I + c, u);
      Vec8<bf16>::load(dy + (int64_t)r * I + c, d);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        float a, ga;
        act_val_grad<A>(g[j], a, ga);
        du[j] = d[j] * a;
        dg[j] = d[j] * u[j] * ga;
      }
      Vec8<bf16>::store(dgu + (int64_t)r * 2 * I + c, dg);
      Vec8<bf16>::store(dgu + (int64_t)r * 2 * I + I + c, du);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) dg[j] = du[j] = 0.f;
    }
    Vec8<bf16>::store(&tile[0][rr * GT_C + cc], dg);
    Vec8<bf16>::store(&tile[1][rr * GT_C + cc], du);
  }
  __syncthreads();
  const int lr = tid >> 5, lc = tid & 31;
  const int r = r0 + 8 * lr;
  if (r >= rows) return;
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    u32x2 v[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const u32x2*>(&tile[h][(8 * lr + j) * GT_C + 4 * lc]);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int c = c0 + 4 * lc + i;
      if (c >= I) break;
      const uint32_t sel = (i & 1) ? 0x07060302u : 0x05040100u;
      u32x4 y;
#pragma unroll
      for (int k = 0; k < 4; ++k) y[k] = __builtin_amdgcn_perm(v[2 * k + 1][i >> 1], v[2 * k][i >> 1], sel);
      *reinterpret_cast<u32x4*>(dgut + (int64_t)(h * I + c) * rows + r) = y;
    }
  }
}

// Gated forward that ALSO writes the transposed output yT [I, rows] (bf16): the down projection saves yT instead of
// y for its weight gradient (hipBLASLt NT form), so the backward's [rows, I] transpose disappears. Same tiling as
// glu_bwd_t.
template <int A>
__global__ __launch_bounds__(256) void glu_fwd_t(const bf16* __restrict__ gu, bf16* __restrict__ y,
                                                 bf16* __restrict__ yt, int rows, int I) {
  __shared__ __attribute__((aligned(16))) bf16 tile[GT_R * GT_C];
  const int r0 = blockIdx.y * GT_R, c0 = blockIdx.x * GT_C;
  const int tid = threadIdx.x;
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int v = tid + 256 * k, rr = v >> 4, cc = (v & 15) * 8;
    const int r = r0 + rr, c = c0 + cc;
    float o[8];
    if (r < rows && c < I) {
      float g[8], u[8];
      Vec8<bf16>::load(gu + (int64_t)r * 2 * I + c, g);
      Vec8<bf16>::load(gu + (int64_t)r * 2 * I + I + c, u);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = act_f<A>(g[j]) * u[j];
      Vec8<bf16>::store(y + (int64_t)r * I + c, o);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = 0.f;
    }
    Vec8<bf16>::store(&tile[rr * GT_C + cc], o);
  }
  __syncthreads();
  const int lr = tid >> 5, lc = tid & 31;
  const int r = r0 + 8 * lr;
  if (r >= rows) return;
  u32x2 v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const u32x2*>(&tile[(8 * lr + j) * GT_C + 4 * lc]);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = c0 + 4 * lc + i;
    if (c >= I) break;
    const uint32_t sel = (i & 1) ? 0x07060302u : 0x05040100u;
    u32x4 w;
#pragma unroll
    for (int k = 0; k < 4; ++k) w[k] = __builtin_amdgcn_perm(v[2 * k + 1][i >> 1], v[2 * k][i >> 1], sel);
    *reinterpret_cast<u32x4*>(yt + (int64_t)c * rows + r) = w;
  }
}

// y = act(x + bias)   (bias optional, [C])
template <typename T, int A>
__global__ __launch_bounds__(256) void bias_act_fwd(const T* __restrict__ x, const T* __restrict__ bias,
                                                    T* __restrict__ y, int64_t rows, int C) {
  const int vpr = C / 8;
  const int64_t total = rows * vpr;
  const bool small = total < (int64_t)0x7fffffff;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    int64_t r;
    int c;
    split_idx(idx, vpr, small, r, c);
    float v[8], b[8] = {0, 0, 0, 0, 0, 0, 0, 0}, o[8];
    Vec8<T>::load(x + r * C + c, v);
    if (bias) Vec8<T>::load(bias + c, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = act_f<A>(v[j] + b[j]);
    Vec8<T>::store(y + r * C + c, o);
  }
}

// dx = dy * act'(x + bias)
template <typename T, int A>
__global__ __launch_bounds__(256) void bias_act_bwd(const T* __restrict__ dy, const T* __restrict__ x,
                                                    const T* __restrict__ bias, T* __restrict__ dx, int64_t rows,
                                                    int C) {
  const int vpr = C / 8;
  const int64_t total = rows * vpr;
  const bool small = total < (int64_t)0x7fffffff;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    int64_t r;
    int c;
    split_idx(idx, vpr, small, r, c);
    float v[8], b[8] = {0, 0, 0, 0, 0, 0, 0, 0}, d[8], o[8];
    Vec8<T>::load(x + r * C + c, v);
    Vec8<T>::load(dy + r * C + c, d);
    if (bias) Vec8<T>::load(bias + c, b);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = d[j] * act_grad<A>(v[j] + b[j]);
    Vec8<T>::store(dx + r * C + c, o);
  }
}

}  // namespace

#define ACT_SWITCH(act, KERN, T, ...)                                                   \
  switch (act) {                                                                        \
    case kSilu: hipLaunchKernelGGL((KERN<T, kSilu>), __VA_ARGS__); break;               \
    case kGeluTanh: hipLaunchKernelGGL((KERN<T, kGeluTanh>), __VA_ARGS__); break;       \
    case kRelu: hipLaunchKernelGGL((KERN<T, kRelu>), __VA_ARGS__); break;               \
    case kGeluErf: hipLaunchKernelGGL((KERN<T, kGeluErf>), __VA_ARGS__); break;         \
    default: hipLaunchKernelGGL((KERN<T, kIdentity>), __VA_ARGS__); break;              \
  }

#define DT_SWITCH(dtype, BODY)                 \
  if (dtype == kBF16) {                        \
    typedef bf16 T;                            \
    BODY;                                      \
  } else if (dtype == kF32) {                  \
    typedef float T;                           \
    BODY;                                      \
  } else if (dtype == kF16) {                  \
    typedef _Float16 T;                        \
    BODY;                                      \
  } else {                                     \
    return hipErrorInvalidValue;               \
  }

// HDS_GLU_VAR selects the kernel generation (2 = default, 1 = one vector per iteration); read once per process
static int glu_variant() {
  static const int v = [] {
    const char* e = getenv("HDS_GLU_VAR");
    return e ? atoi(e) : 2;
  }();
  return v;
}

HDS_EXPORT int hds_glu_fwd(int dtype, int act, const void* gu, void* y, int64_t rows, int I, hipStream_t st) {
  if (I % 8) return hipErrorInvalidValue;
  if (glu_variant() == 2) {
    dim3 grid(stream_grid(rows * (I / 8), 512)), block(256);
    DT_SWITCH(dtype, ACT_SWITCH(act, glu_fwd2, T, grid, block, 0, st, (const T*)gu, (T*)y, rows, I));
  } else {
    dim3 grid(stream_grid(rows * (I / 8), 256)), block(256);
    DT_SWITCH(dtype, ACT_SWITCH(act, glu_fwd, T, grid, block, 0, st, (const T*)gu, (T*)y, rows, I));
  }
  return hipGetLastError();
}

HDS_EXPORT int hds_glu_bwd(int dtype, int act, const void* dy, const void* gu, void* dgu, int64_t rows, int I,
                           hipStream_t st) {
  if (I % 8) return hipErrorInvalidValue;
  if (glu_variant() == 2) {
    dim3 grid(stream_grid(rows * (I / 8), 512)), block(256);
    DT_SWITCH(dtype, ACT_SWITCH(act, glu_bwd2, T, grid, block, 0, st, (const T*)dy, (const T*)gu, (T*)dgu, rows, I));
  } else {
    dim3 grid(stream_grid(rows * (I / 8), 256)), block(256);
    DT_SWITCH(dtype, ACT_SWITCH(act, glu_bwd, T, grid, block, 0, st, (const T*)dy, (const T*)gu, (T*)dgu, rows, I));
  }
  return hipGetLastError();
}

#define GLU_T_SWITCH(act, KERN, ...)                                                 \
  switch (act) {                                                                     \
    case kSilu: hipLaunchKernelGGL((KERN<kSilu>), __VA_ARGS__); break;               \
    case kGeluTanh: hipLaunchKernelGGL((KERN<kGeluTanh>), __VA_ARGS__); break;       \
    case kRelu: hipLaunchKernelGGL((KERN<kRelu>), __VA_ARGS__); break;               \
    case kGeluErf: hipLaunchKernelGGL((KERN<kGeluErf>), __VA_ARGS__); break;         \
    default: hipLaunchKernelGGL((KERN<kIdentity>), __VA_ARGS__); break;              \
  }

// bf16 only: y [rows, I] and its transpose yt [I, rows] in one pass
HDS_EXPORT int hds_glu_fwd_t(int act, const void* gu, void* y, void* yt, int rows, int I, hipStream_t st) {
  if (I % 8 || rows % 8 || rows <= 0 || I <= 0) return hipErrorInvalidValue;
  if (((uintptr_t)gu | (uintptr_t)y | (uintptr_t)yt) & 15) return hipErrorInvalidValue;
  dim3 grid((I + GT_C - 1) / GT_C, (rows + GT_R - 1) / GT_R), block(256);
  GLU_T_SWITCH(act, glu_fwd_t, grid, block, 0, st, (const bf16*)gu, (bf16*)y, (bf16*)yt, rows, I);
  return hipGetLastError();
}

// bf16 only: dgu [rows, 2I] and its transpose dgut [2I, rows] in one pass
HDS_EXPORT int hds_glu_bwd_t(int act, const void* dy, const void* gu, void* dgu, void* dgut, int rows, int I,
                             hipStream_t st) {
  if (I % 8 || rows % 8 || rows <= 0 || I <= 0) return hipErrorInvalidValue;
  if (((uintptr_t)dy | (uintptr_t)gu | (uintptr_t)dgu | (uintptr_t)dgut) & 15) return hipErrorInvalidValue;
  dim3 grid((I + GT_C - 1) / GT_C, (rows + GT_R - 1) / GT_R), block(256);
  GLU_T_SWITCH(act, glu_bwd_t, grid, block, 0, st, (const bf16*)dy, (const bf16*)gu, (bf16*)dgu, (bf16*)dgut, rows,
               I);
  return hipGetLastError();
}

HDS_EXPORT int hds_bias_act_fwd(int dtype, int act, const void* x, const void* bias, void* y, int64_t rows, int C,
                                hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  dim3 grid(stream_grid(rows * (C / 8), 256)), block(256);
  DT_SWITCH(dtype, ACT_SWITCH(act, bias_act_fwd, T, grid, block, 0, st, (const T*)x, (const T*)bias, (T*)y, rows, C));
  return hipGetLastError();
}

HDS_EXPORT int hds_bias_act_bwd(int dtype, int act, const void* dy, const void* x, const void* bias, void* dx,
                                int64_t rows, int C, hipStream_t st) {
  if (C % 8) return hipErrorInvalidValue;
  dim3 grid(stream_grid(rows * (C / 8), 256)), block(256);
  DT_SWITCH(dtype, ACT_SWITCH(act, bias_act_bwd, T, grid, block, 0, st, (const T*)dy, (const T*)x, (const T*)bias,
                              (T*)dx, rows, C));
  return hipGetLastError();
}
