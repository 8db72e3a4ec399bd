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

HDS_EXPORT int hds_glu_fwd(int dtype, int act, const void* gu, void* y, int64_t rows, int I, hipStream_t st) {
  if (I % 8) return hipErrorInvalidValue;
  dim3 grid(stream_grid(rows * (I / 8), 256)), block(256);
  DT_SWITCH(dtype, ACT_SWITCH(act, glu_fwd, T, grid, block, 0, st, (const T*)gu, (T*)y, rows, I));
  return hipGetLastError();
}

HDS_EXPORT int hds_glu_bwd(int dtype, int act, const void* dy, const void* gu, void* dgu, int64_t rows, int I,
                           hipStream_t st) {
  if (I % 8) return hipErrorInvalidValue;
  dim3 grid(stream_grid(rows * (I / 8), 256)), block(256);
  DT_SWITCH(dtype, ACT_SWITCH(act, glu_bwd, T, grid, block, 0, st, (const T*)dy, (const T*)gu, (T*)dgu, rows, I));
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
