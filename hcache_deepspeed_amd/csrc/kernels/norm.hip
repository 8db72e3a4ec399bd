// RMSNorm / LayerNorm forward + backward with fused residual add, gfx950.
//
// Capability parity: the reference's inference-only norms
// (deepspeed/inference/v2/kernels/core_ops/cuda_rms_norm/rms_norm_cuda.cu `rms_norm`/`pre_rms_norm`,
//  cuda_layer_norm/layer_norm_cuda.cu `fused_ln`/`fused_residual_ln`)
// and the training LayerNorm of csrc/transformer/normalize_kernels.cu (K4). Here both
// forward AND backward exist for both norms, because the training engine uses them.
//
// Design (MI355X-first):
//   * one wave64 per row; the row lives in registers (NV 16-byte vectors per lane,
//     NV = H/512 for bf16), so x is read from HBM exactly once in forward;
//   * residual add + norm + store of the new residual happen in one pass
//     (pre-norm transformer: h = x + r; y = norm(h)) -- one read of x and r,
//     one write of h and y, instead of three kernels;
//   * backward keeps dgamma/dbeta partials in registers across the rows a wave
//     owns, reduces across the block's waves in LDS and writes one fp32 partial
//     row per block; a second tiny kernel reduces the partials (deterministic,
//     no float atomics).
#include "hds_common.h"

using namespace hds;

namespace {

constexpr int kRowsPerBlock = 4;  // 4 waves per block, one row each per iteration

// ---------------------------------------------------------------------------------
// forward
// ---------------------------------------------------------------------------------
template <typename T, typename WT, int NV, bool LN>
__global__ __launch_bounds__(256) void norm_fwd_kernel(const T* __restrict__ x, const T* __restrict__ res,
                                                       T* __restrict__ res_out, const WT* __restrict__ w,
                                                       const WT* __restrict__ b, T* __restrict__ y,
                                                       float* __restrict__ stat_mean, float* __restrict__ stat_rstd,
                                                       int rows, int cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int row = blockIdx.x * kRowsPerBlock + wid;
  if (row >= rows) return;
  const T* xr = x + (int64_t)row * cols;
  float v[NV][8];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 8;
    Vec8<T>::load(xr + c, v[i]);
  }
  if (res != nullptr) {
    const T* rr = res + (int64_t)row * cols;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 8;
      float r[8];
      Vec8<T>::load(rr + c, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[i][j] = to_f(from_f<T>(v[i][j] + r[j]));  // round like the unfused add
    }
    if (res_out != nullptr) {
      T* ro = res_out + (int64_t)row * cols;
#pragma unroll
      for (int i = 0; i < NV; ++i) Vec8<T>::store(ro + (i * 64 + lane) * 8, v[i]);
    }
  }
  float mean = 0.f;
  if constexpr (LN) {
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i)
#pragma unroll
      for (int j = 0; j < 8; ++j) s += v[i][j];
    mean = wave_sum(s) / (float)cols;
  }
  float ss = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float d = v[i][j] - mean;
      ss += d * d;
    }
  const float rstd = rsqrtf(wave_sum(ss) / (float)cols + eps);
  T* yr = y + (int64_t)row * cols;
#pragma unroll
  for (int i = 0; i < NV; ++i) {
    const int c = (i * 64 + lane) * 8;
    float wv[8], o[8];
    Vec8<WT>::load(w + c, wv);
    if constexpr (LN) {
      float bv[8];
      if (b != nullptr) Vec8<WT>::load(b + c, bv);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = (v[i][j] - mean) * rstd * wv[j] + (b != nullptr ? bv[j] : 0.f);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = v[i][j] * rstd * wv[j];
    }
    Vec8<T>::store(yr + c, o);
  }
  if (lane == 0) {
    stat_rstd[row] = rstd;
    if constexpr (LN) stat_mean[row] = mean;
  }
}

// Generic-width forward (cols % 8 == 0, any cols): two passes over the row (second hits L1/L2).
template <typename T, typename WT, bool LN>
__global__ __launch_bounds__(256) void norm_fwd_generic(const T* __restrict__ x, const T* __restrict__ res,
                                                        T* __restrict__ res_out, const WT* __restrict__ w,
                                                        const WT* __restrict__ b, T* __restrict__ y,
                                                        float* __restrict__ stat_mean, float* __restrict__ stat_rstd,
                                                        int rows, int cols, float eps) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * kRowsPerBlock + (threadIdx.x >> 6);
  if (row >= rows) return;
  const T* xr = x + (int64_t)row * cols;
  const T* rr = res ? res + (int64_t)row * cols : nullptr;
  T* ro = res_out ? res_out + (int64_t)row * cols : nullptr;
  float s = 0.f, ss = 0.f;
  for (int c = lane * 8; c < cols; c += 512) {
    float v[8];
    Vec8<T>::load(xr + c, v);
    if (rr) {
      float r[8];
      Vec8<T>::load(rr + c, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = to_f(from_f<T>(v[j] + r[j]));
      if (ro) Vec8<T>::store(ro + c, v);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s += v[j];
      ss += v[j] * v[j];
    }
  }
  s = wave_sum(s);
  ss = wave_sum(ss);
  const float mean = LN ? s / cols : 0.f;
  const float var = LN ? fmaxf(ss / cols - mean * mean, 0.f) : ss / cols;
  const float rstd = rsqrtf(var + eps);
  T* yr = y + (int64_t)row * cols;
  for (int c = lane * 8; c < cols; c += 512) {
    float v[8], wv[8], o[8];
    Vec8<T>::load(xr + c, v);
    if (rr) {
      float r[8];
      Vec8<T>::load(rr + c, r);
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = to_f(from_f<T>(v[j] + r[j]));
    }
    Vec8<WT>::load(w + c, wv);
    float bv[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    if (LN && b) Vec8<WT>::load(b + c, bv);
#pragma unroll
    for (int j = 0; j < 8; ++j) o[j] = (v[j] - mean) * rstd * wv[j] + bv[j];
    Vec8<T>::store(yr + c, o);
  }
  if (lane == 0) {
    stat_rstd[row] = rstd;
    if (LN) stat_mean[row] = mean;
  }
}

// ---------------------------------------------------------------------------------
// backward:  h = norm input (after the fused residual add), dy = dL/dy,
//            dres = gradient arriving at h through the residual stream (optional).
// dx = rstd * (w*dy - xhat * mean(w*dy*xhat) [- mean(w*dy) for LN]) + dres
// dw_part[block] = sum_rows dy * xhat ; db_part[block] = sum_rows dy
// ---------------------------------------------------------------------------------
template <typename T, typename WT, int NV, bool LN>
__global__ __launch_bounds__(256) void norm_bwd_kernel(const T* __restrict__ dy, const T* __restrict__ h,
                                                       const T* __restrict__ dres, const WT* __restrict__ w,
                                                       const float* __restrict__ stat_mean,
                                                       const float* __restrict__ stat_rstd, T* __restrict__ dx,
                                                       float* __restrict__ dw_part, float* __restrict__ db_part,
                                                       int rows, int cols) {
  typedef T vec8 __attribute__((ext_vector_type(8)));
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  float accw[NV][8], accb[LN ? NV : 1][8];
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) accw[i][j] = 0.f;
#pragma unroll
  for (int i = 0; i < (LN ? NV : 1); ++i)
#pragma unroll
    for (int j = 0; j < 8; ++j) accb[i][j] = 0.f;

  for (int row = blockIdx.x * kRowsPerBlock + wid; row < rows; row += gridDim.x * kRowsPerBlock) {
    const int64_t base = (int64_t)row * cols;
    const float rstd = stat_rstd[row];
    const float mean = LN ? stat_mean[row] : 0.f;
    vec8 hv[NV], dv[NV], rv[NV];  // packed in the activation dtype: 4 VGPRs per vector for bf16
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 8;
      hv[i] = *reinterpret_cast<const vec8*>(h + base + c);
      dv[i] = *reinterpret_cast<const vec8*>(dy + base + c);
    }
    // the residual gradient is issued with the row's other loads, so its latency hides behind the reduction
    if (dres != nullptr) {
#pragma unroll
      for (int i = 0; i < NV; ++i) rv[i] = *reinterpret_cast<const vec8*>(dres + base + (i * 64 + lane) * 8);
    }
    float sum_gx = 0.f, sum_g = 0.f;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      float wv[8];
      Vec8<WT>::load(w + (i * 64 + lane) * 8, wv);  // L1/L2 resident across rows
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (to_f(hv[i][j]) - mean) * rstd;
        const float d = to_f(dv[i][j]);
        const float g = d * wv[j];
        sum_gx += g * xh;
        sum_g += g;
        accw[i][j] += d * xh;
        if constexpr (LN) accb[i][j] += d;
      }
    }
    sum_gx = wave_sum(sum_gx) / (float)cols;
    if (LN) sum_g = wave_sum(sum_g) / (float)cols;
#pragma unroll
    for (int i = 0; i < NV; ++i) {
      const int c = (i * 64 + lane) * 8;
      float wv[8], o[8];
      Vec8<WT>::load(w + c, wv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (to_f(hv[i][j]) - mean) * rstd;
        const float g = to_f(dv[i][j]) * wv[j];
        const float d = rstd * (g - xh * sum_gx - (LN ? sum_g : 0.f));
        o[j] = d + (dres != nullptr ? to_f(rv[i][j]) : 0.f);
      }
      Vec8<T>::store(dx + base + c, o);
    }
  }
  // block reduction of the weight-gradient partials through LDS (one fp32 row per block)
  __shared__ float red[kRowsPerBlock][512];
#pragma unroll
  for (int i = 0; i < NV; ++i) {
#pragma unroll
    for (int j = 0; j < 8; ++j) red[wid][lane * 8 + j] = accw[i][j];
    __syncthreads();
    for (int e = threadIdx.x; e < 512; e += 256) {
      const int col = i * 512 + (e / 8) * 8 + (e % 8);  // = i*512 + e
      dw_part[(int64_t)blockIdx.x * cols + col] = red[0][e] + red[1][e] + red[2][e] + red[3][e];
    }
    __syncthreads();
    if constexpr (LN) {
#pragma unroll
      for (int j = 0; j < 8; ++j) red[wid][lane * 8 + j] = accb[i][j];
      __syncthreads();
      for (int e = threadIdx.x; e < 512; e += 256)
        db_part[(int64_t)blockIdx.x * cols + i * 512 + e] = red[0][e] + red[1][e] + red[2][e] + red[3][e];
      __syncthreads();
    }
  }
}

// generic-width backward: per-row two passes, partial weight grads via atomics into
// the block's own partial row (no cross-block contention; order fixed per block).
template <typename T, typename WT, bool LN>
__global__ __launch_bounds__(256) void norm_bwd_generic(const T* __restrict__ dy, const T* __restrict__ h,
                                                        const T* __restrict__ dres, const WT* __restrict__ w,
                                                        const float* __restrict__ stat_mean,
                                                        const float* __restrict__ stat_rstd, T* __restrict__ dx,
                                                        float* __restrict__ dw_part, float* __restrict__ db_part,
                                                        int rows, int cols) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  // zero this block's partial rows
  for (int c = threadIdx.x; c < cols; c += 256) {
    dw_part[(int64_t)blockIdx.x * cols + c] = 0.f;
    if (LN) db_part[(int64_t)blockIdx.x * cols + c] = 0.f;
  }
  __syncthreads();
  for (int row = blockIdx.x * kRowsPerBlock + wid; row < rows; row += gridDim.x * kRowsPerBlock) {
    const int64_t base = (int64_t)row * cols;
    const float rstd = stat_rstd[row];
    const float mean = LN ? stat_mean[row] : 0.f;
    float sgx = 0.f, sg = 0.f;
    for (int c = lane * 8; c < cols; c += 512) {
      float hv[8], dv[8], wv[8];
      Vec8<T>::load(h + base + c, hv);
      Vec8<T>::load(dy + base + c, dv);
      Vec8<WT>::load(w + c, wv);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (hv[j] - mean) * rstd;
        const float g = dv[j] * wv[j];
        sgx += g * xh;
        sg += g;
        atomicAdd(&dw_part[(int64_t)blockIdx.x * cols + c + j], dv[j] * xh);
        if (LN) atomicAdd(&db_part[(int64_t)blockIdx.x * cols + c + j], dv[j]);
      }
    }
    sgx = wave_sum(sgx) / cols;
    sg = LN ? wave_sum(sg) / cols : 0.f;
    for (int c = lane * 8; c < cols; c += 512) {
      float hv[8], dv[8], wv[8], o[8], dr[8];
      Vec8<T>::load(h + base + c, hv);
      Vec8<T>::load(dy + base + c, dv);
      Vec8<WT>::load(w + c, wv);
      if (dres) Vec8<T>::load(dres + base + c, dr);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float xh = (hv[j] - mean) * rstd;
        o[j] = rstd * (dv[j] * wv[j] - xh * sgx - sg) + (dres ? dr[j] : 0.f);
      }
      Vec8<T>::store(dx + base + c, o);
    }
  }
}

// partial [nparts, cols] fp32 -> out[cols] (dtype WT), optionally accumulated into out.
// Block = 64 columns x 4 part-groups: coalesced 256-B rows per wave, LDS combine of the 4 groups.
template <typename WT>
__global__ __launch_bounds__(256) void reduce_parts_kernel(const float* __restrict__ part, WT* __restrict__ out,
                                                           int nparts, int cols, int accumulate) {
  __shared__ float red[4][64];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int pg = threadIdx.x >> 6;
  float s = 0.f;
  if (c < cols)
    for (int p = pg; p < nparts; p += 4) s += part[(int64_t)p * cols + c];
  red[pg][threadIdx.x & 63] = s;
  __syncthreads();
  if (pg == 0 && c < cols) {
    float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    if (accumulate) t += to_f(out[c]);
    out[c] = from_f<WT>(t);
  }
}

template <typename T, typename WT, bool LN>
hipError_t launch_fwd(const void* x, const void* res, void* res_out, const void* w, const void* b, void* y,
                      float* mean, float* rstd, int rows, int cols, float eps, hipStream_t st) {
  dim3 grid((rows + kRowsPerBlock - 1) / kRowsPerBlock), block(256);
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, block, 0, st, (const T*)x, (const T*)res, (T*)res_out, (const WT*)w,
                       (const WT*)b, (T*)y, mean, rstd, rows, cols, eps);
  };
  switch (cols) {
    case 512: args(norm_fwd_kernel<T, WT, 1, LN>); break;
    case 1024: args(norm_fwd_kernel<T, WT, 2, LN>); break;
    case 2048: args(norm_fwd_kernel<T, WT, 4, LN>); break;
    case 3072: args(norm_fwd_kernel<T, WT, 6, LN>); break;
    case 4096: args(norm_fwd_kernel<T, WT, 8, LN>); break;
    case 5120: args(norm_fwd_kernel<T, WT, 10, LN>); break;
    case 6144: args(norm_fwd_kernel<T, WT, 12, LN>); break;
    case 8192: args(norm_fwd_kernel<T, WT, 16, LN>); break;
    default: args(norm_fwd_generic<T, WT, LN>); break;
  }
  return hipGetLastError();
}

template <typename T, typename WT, bool LN>
hipError_t launch_bwd(const void* dy, const void* h, const void* dres, const void* w, const float* mean,
                      const float* rstd, void* dx, float* dw_part, float* db_part, int nparts, void* dw, void* db,
                      int accumulate, int rows, int cols, hipStream_t st) {
  dim3 grid(nparts), block(256);
  auto args = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, block, 0, st, (const T*)dy, (const T*)h, (const T*)dres, (const WT*)w, mean,
                       rstd, (T*)dx, dw_part, db_part, rows, cols);
  };
  switch (cols) {
    case 512: args(norm_bwd_kernel<T, WT, 1, LN>); break;
    case 1024: args(norm_bwd_kernel<T, WT, 2, LN>); break;
    case 2048: args(norm_bwd_kernel<T, WT, 4, LN>); break;
    case 3072: args(norm_bwd_kernel<T, WT, 6, LN>); break;
    case 4096: args(norm_bwd_kernel<T, WT, 8, LN>); break;
    case 5120: args(norm_bwd_kernel<T, WT, 10, LN>); break;
    case 6144: args(norm_bwd_kernel<T, WT, 12, LN>); break;
    case 8192: args(norm_bwd_kernel<T, WT, 16, LN>); break;
    default: args(norm_bwd_generic<T, WT, LN>); break;
  }
  dim3 rg((cols + 63) / 64);
  if (dw) hipLaunchKernelGGL(reduce_parts_kernel<WT>, rg, block, 0, st, dw_part, (WT*)dw, nparts, cols, accumulate);
  if (LN && db) hipLaunchKernelGGL(reduce_parts_kernel<WT>, rg, block, 0, st, db_part, (WT*)db, nparts, cols, accumulate);
  return hipGetLastError();
}

}  // namespace

// dtype: activation dtype code; wdtype: weight dtype code (DType enum)
#define HDS_DISPATCH2(dtype, wdtype, LN, FN, ...)                                              \
  do {                                                                                         \
    if (dtype == kBF16 && wdtype == kBF16) return FN<bf16, bf16, LN>(__VA_ARGS__);             \
    if (dtype == kBF16 && wdtype == kF32) return FN<bf16, float, LN>(__VA_ARGS__);             \
    if (dtype == kF32 && wdtype == kF32) return FN<float, float, LN>(__VA_ARGS__);             \
    if (dtype == kF16 && wdtype == kF16) return FN<_Float16, _Float16, LN>(__VA_ARGS__);       \
    if (dtype == kF16 && wdtype == kF32) return FN<_Float16, float, LN>(__VA_ARGS__);          \
    return hipErrorInvalidValue;                                                               \
  } while (0)

HDS_EXPORT int hds_norm_fwd(int is_ln, int dtype, int wdtype, const void* x, const void* res, void* res_out,
                            const void* w, const void* b, void* y, float* mean, float* rstd, int rows, int cols,
                            float eps, hipStream_t st) {
  if (cols % 8) return hipErrorInvalidValue;
  if (is_ln) HDS_DISPATCH2(dtype, wdtype, true, launch_fwd, x, res, res_out, w, b, y, mean, rstd, rows, cols, eps, st);
  HDS_DISPATCH2(dtype, wdtype, false, launch_fwd, x, res, res_out, w, b, y, mean, rstd, rows, cols, eps, st);
}

static int g_norm_bwd_max_parts = 512;

// cap on the backward's workgroups = fp32 weight-gradient partial rows (A/B knob; 512 = 8 waves per CU)
HDS_EXPORT int hds_norm_bwd_set_max_parts(int n) {
  if (n < 1 || n > 8192) return hipErrorInvalidValue;
  g_norm_bwd_max_parts = n;
  return 0;
}

HDS_EXPORT int hds_norm_bwd_nparts(int rows) {
  int n = (rows + kRowsPerBlock - 1) / kRowsPerBlock;
  return n < g_norm_bwd_max_parts ? (n < 1 ? 1 : n) : g_norm_bwd_max_parts;
}

HDS_EXPORT int hds_norm_bwd(int is_ln, int dtype, int wdtype, const void* dy, const void* h, const void* dres,
                            const void* w, const float* mean, const float* rstd, void* dx, float* dw_part,
                            float* db_part, int nparts, void* dw, void* db, int accumulate, int rows, int cols,
                            hipStream_t st) {
  if (cols % 8) return hipErrorInvalidValue;
  if (is_ln)
    HDS_DISPATCH2(dtype, wdtype, true, launch_bwd, dy, h, dres, w, mean, rstd, dx, dw_part, db_part, nparts, dw, db,
                  accumulate, rows, cols, st);
  HDS_DISPATCH2(dtype, wdtype, false, launch_bwd, dy, h, dres, w, mean, rstd, dx, dw_part, db_part, nparts, dw, db,
                accumulate, rows, cols, st);
}
