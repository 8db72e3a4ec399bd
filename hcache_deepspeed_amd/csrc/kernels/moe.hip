// Mixture-of-Experts token routing: dispatch (permute into expert/capacity slots) and combine
// (weighted un-permute), forward and backward.
//
// Capability parity: deepspeed/inference/v2/kernels/ragged_ops/moe_scatter (`moe_scatter_kernel`, K35) and
// moe_gather (`moe_gather_kernel`, K36), plus the training dispatch/combine einsums of
// moe/sharded_moe.py (`MOELayer` :449-677, '[E, C, M]' dispatched tensor :96-109). The reference training
// path builds dense [T, E, C] masks and runs einsums; here every token row moves once with 16-byte
// vectors and the capacity slot of each (token, choice) is precomputed (deterministic cumsum).
//
// Slot layout: expert-major [E * C, H]; slot(t, j) = expert[t, j] * C + pos[t, j], dropped if pos >= C.
#include "hds_common.h"

using namespace hds;

namespace {

template <typename T>
__global__ __launch_bounds__(256) void dispatch_kernel(const T* __restrict__ x, const int* __restrict__ expert,
                                                       const int* __restrict__ pos, T* __restrict__ out, int n_tok,
                                                       int k, int H, int C) {
  const int t = blockIdx.x;
  for (int j = 0; j < k; ++j) {
    const int p = pos[t * k + j];
    if (p < 0 || p >= C) continue;
    const int64_t slot = (int64_t)expert[t * k + j] * C + p;
    for (int c = threadIdx.x * 8; c < H; c += 256 * 8) {
      float v[8];
      Vec8<T>::load(x + (int64_t)t * H + c, v);
      Vec8<T>::store(out + slot * H + c, v);
    }
  }
}

// dx[t] = sum_j dout[slot(t, j)]
template <typename T>
__global__ __launch_bounds__(256) void dispatch_bwd_kernel(const T* __restrict__ dout, const int* __restrict__ expert,
                                                           const int* __restrict__ pos, T* __restrict__ dx, int n_tok,
                                                           int k, int H, int C) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x * 8; c < H; c += 256 * 8) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const int p = pos[t * k + j];
      if (p < 0 || p >= C) continue;
      const int64_t slot = (int64_t)expert[t * k + j] * C + p;
      float v[8];
      Vec8<T>::load(dout + slot * H + c, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += v[i];
    }
    Vec8<T>::store(dx + (int64_t)t * H + c, acc);
  }
}

// out[t] = sum_j w[t, j] * y[slot(t, j)]
template <typename T>
__global__ __launch_bounds__(256) void combine_kernel(const T* __restrict__ y, const int* __restrict__ expert,
                                                      const int* __restrict__ pos, const float* __restrict__ w,
                                                      T* __restrict__ out, int n_tok, int k, int H, int C) {
  const int t = blockIdx.x;
  for (int c = threadIdx.x * 8; c < H; c += 256 * 8) {
    float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    for (int j = 0; j < k; ++j) {
      const int p = pos[t * k + j];
      if (p < 0 || p >= C) continue;
      const int64_t slot = (int64_t)expert[t * k + j] * C + p;
      const float wj = w[t * k + j];
      float v[8];
      Vec8<T>::load(y + slot * H + c, v);
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] += wj * v[i];
    }
    Vec8<T>::store(out + (int64_t)t * H + c, acc);
  }
}

// dy[slot(t, j)] = w[t, j] * dout[t] ; dw[t, j] = <dout[t], y[slot(t, j)]>
template <typename T>
__global__ __launch_bounds__(256) void combine_bwd_kernel(const T* __restrict__ dout, const T* __restrict__ y,
                                                          const int* __restrict__ expert, const int* __restrict__ pos,
                                                          const float* __restrict__ w, T* __restrict__ dy,
                                                          float* __restrict__ dw, int n_tok, int k, int H, int C) {
  __shared__ float red[4];
  const int t = blockIdx.x;
  for (int j = 0; j < k; ++j) {
    const int p = pos[t * k + j];
    const bool kept = p >= 0 && p < C;
    const int64_t slot = kept ? (int64_t)expert[t * k + j] * C + p : 0;
    const float wj = w[t * k + j];
    float dot = 0.f;
    if (kept) {
      for (int c = threadIdx.x * 8; c < H; c += 256 * 8) {
        float d[8], v[8], o[8];
        Vec8<T>::load(dout + (int64_t)t * H + c, d);
        Vec8<T>::load(y + slot * H + c, v);
#pragma unroll
        for (int i = 0; i < 8; ++i) {
          dot += d[i] * v[i];
          o[i] = wj * d[i];
        }
        Vec8<T>::store(dy + slot * H + c, o);
      }
    }
    dot = block_sum<256>(dot, red);
    if (threadIdx.x == 0) dw[t * k + j] = kept ? dot : 0.f;
  }
}

}  // namespace

HDS_EXPORT int hds_moe_dispatch(int dtype, const void* x, const int* expert, const int* pos, void* out, int n_tok,
                                int k, int H, int C, hipStream_t st) {
  if (H % 8 || n_tok <= 0) return n_tok <= 0 ? 0 : hipErrorInvalidValue;
  if (dtype == kBF16)
    hipLaunchKernelGGL(dispatch_kernel<bf16>, dim3(n_tok), dim3(256), 0, st, (const bf16*)x, expert, pos, (bf16*)out,
                       n_tok, k, H, C);
  else if (dtype == kF32)
    hipLaunchKernelGGL(dispatch_kernel<float>, dim3(n_tok), dim3(256), 0, st, (const float*)x, expert, pos,
                       (float*)out, n_tok, k, H, C);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

HDS_EXPORT int hds_moe_dispatch_bwd(int dtype, const void* dout, const int* expert, const int* pos, void* dx, int n_tok,
                                    int k, int H, int C, hipStream_t st) {
  if (H % 8 || n_tok <= 0) return n_tok <= 0 ? 0 : hipErrorInvalidValue;
  if (dtype == kBF16)
    hipLaunchKernelGGL(dispatch_bwd_kernel<bf16>, dim3(n_tok), dim3(256), 0, st, (const bf16*)dout, expert, pos,
                       (bf16*)dx, n_tok, k, H, C);
  else if (dtype == kF32)
    hipLaunchKernelGGL(dispatch_bwd_kernel<float>, dim3(n_tok), dim3(256), 0, st, (const float*)dout, expert, pos,
                       (float*)dx, n_tok, k, H, C);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

HDS_EXPORT int hds_moe_combine(int dtype, const void* y, const int* expert, const int* pos, const float* w, void* out,
                               int n_tok, int k, int H, int C, hipStream_t st) {
  if (H % 8 || n_tok <= 0) return n_tok <= 0 ? 0 : hipErrorInvalidValue;
  if (dtype == kBF16)
    hipLaunchKernelGGL(combine_kernel<bf16>, dim3(n_tok), dim3(256), 0, st, (const bf16*)y, expert, pos, w,
                       (bf16*)out, n_tok, k, H, C);
  else if (dtype == kF32)
    hipLaunchKernelGGL(combine_kernel<float>, dim3(n_tok), dim3(256), 0, st, (const float*)y, expert, pos, w,
                       (float*)out, n_tok, k, H, C);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

HDS_EXPORT int hds_moe_combine_bwd(int dtype, const void* dout, const void* y, const int* expert, const int* pos,
                                   const float* w, void* dy, float* dw, int n_tok, int k, int H, int C,
                                   hipStream_t st) {
  if (H % 8 || n_tok <= 0) return n_tok <= 0 ? 0 : hipErrorInvalidValue;
  if (dtype == kBF16)
    hipLaunchKernelGGL(combine_bwd_kernel<bf16>, dim3(n_tok), dim3(256), 0, st, (const bf16*)dout, (const bf16*)y,
                       expert, pos, w, (bf16*)dy, dw, n_tok, k, H, C);
  else if (dtype == kF32)
    hipLaunchKernelGGL(combine_bwd_kernel<float>, dim3(n_tok), dim3(256), 0, st, (const float*)dout, (const float*)y,
                       expert, pos, w, (float*)dy, dw, n_tok, k, H, C);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
