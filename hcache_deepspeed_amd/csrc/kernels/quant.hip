// Group-wise quantization: INT8 / INT4 (symmetric or asymmetric) and FP8 (OCP e4m3 / e5m2 via the
// gfx950 conversion instructions), dequantization, and the ZeRO++ qgZ "dequantize + reduce" of the
// chunks received from every rank in a quantized reduce-scatter.
//
// Capability parity: csrc/quantization/quantize.cu (`cached_quantization`, K16), dequantize.cu /
// quantize_intX.cu (K17), quant_reduce.cu (`dequant_reduce`, K19), csrc/fp_quantizer/fp_quantize.cu
// (`apply_quantization` / `apply_dequantization`, K21). One wave64 owns one group (group_size up to
// 8192 elements, a multiple of 8): 16-byte vector loads, wave-level absmax / min-max through
// __shfl_xor, scales kept in fp32. INT4 packs two values per byte (low nibble = even element).
#include <algorithm>

#include "hds_common.h"

using namespace hds;

namespace {

constexpr int kWaves = 4;  // groups per 256-thread block

__device__ __forceinline__ float wave_min(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fminf(v, __shfl_xor(v, o));
  return v;
}

template <typename T, int BITS, bool SYM>
__global__ __launch_bounds__(256) void quant_int_kernel(const T* __restrict__ x, int8_t* __restrict__ q,
                                                        float* __restrict__ scales, float* __restrict__ mins,
                                                        int64_t n_groups, int group_size) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (g >= n_groups) return;
  const T* xg = x + g * group_size;
  float amax = 0.f, vmin = 3.4e38f, vmax = -3.4e38f;
  for (int c = lane * 8; c < group_size; c += 64 * 8) {
    float v[8];
    Vec8<T>::load(xg + c, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      amax = fmaxf(amax, fabsf(v[i]));
      vmin = fminf(vmin, v[i]);
      vmax = fmaxf(vmax, v[i]);
    }
  }
  constexpr float qmax = (float)((1 << (BITS - 1)) - 1);       // 127 / 7
  constexpr float qrange = (float)((1 << BITS) - 1);           // 255 / 15
  float scale, lo = 0.f;
  if (SYM) {
    amax = wave_max(amax);
    scale = amax > 0.f ? amax / qmax : 1.f;
  } else {
    vmin = wave_min(vmin);
    vmax = wave_max(vmax);
    scale = vmax > vmin ? (vmax - vmin) / qrange : 1.f;
    lo = vmin;
  }
  const float inv = 1.f / scale;
  if (lane == 0) {
    scales[g] = scale;
    if (!SYM) mins[g] = lo;
  }
  for (int c = lane * 8; c < group_size; c += 64 * 8) {
    float v[8];
    Vec8<T>::load(xg + c, v);
    int qi[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      if (SYM) {
        qi[i] = (int)fminf(fmaxf(rintf(v[i] * inv), -qmax - 1.f), qmax);
      } else {
        qi[i] = (int)fminf(fmaxf(rintf((v[i] - lo) * inv), 0.f), qrange);
      }
    }
    if (BITS == 8) {
      uint32_t w0 = (qi[0] & 0xff) | ((qi[1] & 0xff) << 8) | ((qi[2] & 0xff) << 16) | ((uint32_t)(qi[3] & 0xff) << 24);
      uint32_t w1 = (qi[4] & 0xff) | ((qi[5] & 0xff) << 8) | ((qi[6] & 0xff) << 16) | ((uint32_t)(qi[7] & 0xff) << 24);
      *reinterpret_cast<uint2*>(q + g * group_size + c) = make_uint2(w0, w1);
    } else {
      uint32_t w = 0;
#pragma unroll
      for (int i = 0; i < 8; ++i) w |= (uint32_t)(qi[i] & 0xf) << (4 * i);
      *reinterpret_cast<uint32_t*>(q + (g * group_size + c) / 2) = w;
    }
  }
}

// Element-parallel: thread i dequantizes elements [8i, 8i+8) (one 8-B int8 / 4-B int4 load, one 16-B bf16 store),
// its group is 8i / group_size, so every lane is busy whatever the group size (a wave-per-group layout leaves 3/4
// of the lanes idle at the common 128-element weight groups).
template <typename T, int BITS, bool SYM>
__global__ __launch_bounds__(256) void dequant_int_kernel(const int8_t* __restrict__ q, const float* __restrict__ scales,
                                                          const float* __restrict__ mins, T* __restrict__ y,
                                                          int64_t n_groups, int group_size) {
  const int64_t n8 = n_groups * group_size / 8;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t g = i * 8 / group_size;
    const float s = scales[g];
    const float lo = SYM ? 0.f : mins[g];
    float v[8];
    if (BITS == 8) {
      const uint2 w = *reinterpret_cast<const uint2*>(q + i * 8);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int a = SYM ? (int)(int8_t)((w.x >> (8 * k)) & 0xff) : (int)((w.x >> (8 * k)) & 0xff);
        const int b = SYM ? (int)(int8_t)((w.y >> (8 * k)) & 0xff) : (int)((w.y >> (8 * k)) & 0xff);
        v[k] = a * s + lo;
        v[4 + k] = b * s + lo;
      }
    } else {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(q + i * 4);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        int n = (w >> (4 * k)) & 0xf;
        if (SYM) n = (n ^ 8) - 8;  // sign-extend the nibble
        v[k] = n * s + lo;
      }
    }
    Vec8<T>::store(y + i * 8, v);
  }
}

// ---- FP8 (OCP e4m3 / e5m2) -----------------------------------------------------------------
template <typename T, bool E5M2>
__global__ __launch_bounds__(256) void quant_fp8_kernel(const T* __restrict__ x, uint8_t* __restrict__ q,
                                                        float* __restrict__ scales, int64_t n_groups, int group_size) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (g >= n_groups) return;
  const T* xg = x + g * group_size;
  float amax = 0.f;
  for (int c = lane * 8; c < group_size; c += 64 * 8) {
    float v[8];
    Vec8<T>::load(xg + c, v);
#pragma unroll
    for (int i = 0; i < 8; ++i) amax = fmaxf(amax, fabsf(v[i]));
  }
  amax = wave_max(amax);
  constexpr float fmax = E5M2 ? 57344.f : 448.f;
  const float scale = amax > 0.f ? amax / fmax : 1.f;
  const float inv = 1.f / scale;
  if (lane == 0) scales[g] = scale;
  for (int c = lane * 8; c < group_size; c += 64 * 8) {
    float v[8];
    Vec8<T>::load(xg + c, v);
    int w0, w1;
    if (E5M2) {
      w0 = __builtin_amdgcn_cvt_pk_bf8_f32(v[0] * inv, v[1] * inv, 0, false);
      w0 = __builtin_amdgcn_cvt_pk_bf8_f32(v[2] * inv, v[3] * inv, w0, true);
      w1 = __builtin_amdgcn_cvt_pk_bf8_f32(v[4] * inv, v[5] * inv, 0, false);
      w1 = __builtin_amdgcn_cvt_pk_bf8_f32(v[6] * inv, v[7] * inv, w1, true);
    } else {
      w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[0] * inv, v[1] * inv, 0, false);
      w0 = __builtin_amdgcn_cvt_pk_fp8_f32(v[2] * inv, v[3] * inv, w0, true);
      w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[4] * inv, v[5] * inv, 0, false);
      w1 = __builtin_amdgcn_cvt_pk_fp8_f32(v[6] * inv, v[7] * inv, w1, true);
    }
    *reinterpret_cast<int2*>(q + g * group_size + c) = make_int2(w0, w1);
  }
}

template <bool E5M2>
__device__ __forceinline__ float fp8_to_f32(int w, int sel) {
  switch (sel) {
    case 0: return E5M2 ? __builtin_amdgcn_cvt_f32_bf8(w, 0) : __builtin_amdgcn_cvt_f32_fp8(w, 0);
    case 1: return E5M2 ? __builtin_amdgcn_cvt_f32_bf8(w, 1) : __builtin_amdgcn_cvt_f32_fp8(w, 1);
    case 2: return E5M2 ? __builtin_amdgcn_cvt_f32_bf8(w, 2) : __builtin_amdgcn_cvt_f32_fp8(w, 2);
    default: return E5M2 ? __builtin_amdgcn_cvt_f32_bf8(w, 3) : __builtin_amdgcn_cvt_f32_fp8(w, 3);
  }
}

template <typename T, bool E5M2>
__global__ __launch_bounds__(256) void dequant_fp8_kernel(const uint8_t* __restrict__ q,
                                                          const float* __restrict__ scales, T* __restrict__ y,
                                                          int64_t n_groups, int group_size) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (g >= n_groups) return;
  const float s = scales[g];
  for (int c = lane * 8; c < group_size; c += 64 * 8) {
    const int2 w = *reinterpret_cast<const int2*>(q + g * group_size + c);
    float v[8];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[i] = fp8_to_f32<E5M2>(w.x, i) * s;
      v[4 + i] = fp8_to_f32<E5M2>(w.y, i) * s;
    }
    Vec8<T>::store(y + g * group_size + c, v);
  }
}

// ---- qgZ dequantize + reduce ------------------------------------------------------------------
// q: [world][n] symmetric int8/int4 chunks received from every rank, scales [world][n/group];
// out[i] (+)= sum_r dequant(q[r][i]).  One wave per group of the OUTPUT chunk.
template <typename TO, int BITS>
__global__ __launch_bounds__(256) void dequant_reduce_kernel(const int8_t* __restrict__ q,
                                                             const float* __restrict__ scales, TO* __restrict__ out,
                                                             int world, int64_t n, int group_size, int accumulate) {
  const int lane = threadIdx.x & 63;
  const int64_t groups = n / group_size;
  const int64_t g = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (g >= groups) return;
  for (int c = lane * 8; c < group_size; c += 64 * 8) {
    float acc[8];
    if (accumulate) {
      Vec8<TO>::load(out + g * group_size + c, acc);
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    }
    for (int r = 0; r < world; ++r) {
      const float s = scales[(int64_t)r * groups + g];
      const int64_t e = (int64_t)r * n + g * group_size + c;
      if (BITS == 8) {
        const uint2 w = *reinterpret_cast<const uint2*>(q + e);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          acc[i] += (float)(int8_t)((w.x >> (8 * i)) & 0xff) * s;
          acc[4 + i] += (float)(int8_t)((w.y >> (8 * i)) & 0xff) * s;
        }
      } else {
        const uint32_t w = *reinterpret_cast<const uint32_t*>(q + e / 2);
#pragma unroll
        for (int i = 0; i < 8; ++i) acc[i] += (float)((((int)(w >> (4 * i)) & 0xf) ^ 8) - 8) * s;
      }
    }
    Vec8<TO>::store(out + g * group_size + c, acc);
  }
}

inline dim3 grid_for(int64_t groups) { return dim3((unsigned)((groups + kWaves - 1) / kWaves)); }

// ---- weight-only INT8 / INT4 GEMV for decode (reference K37 mixed-input GEMM, inference/quantization) ------------
// y[m, n] = sum_k x[m, k] * q[n, k] * scale[n, k / G] for a symmetric group-quantized weight [N, K] (groups along k,
// the layout of quant_int_kernel on W.reshape(-1)). One wave owns R = 4 output features; each lane takes 16
// consecutive k per step: it loads its x fragment for all M rows ONCE (bf16, registers) and reuses it for the R
// weight rows (one 16-B int8 / 8-B int4 load each), so x traffic is amortised over R rows instead of being
// re-read per row (which made M = 8 L2-bound). fp32 accumulators [R][M], one wave reduction per output at the end.
// The weight stream is 2x (int8) / 4x (int4) smaller than bf16 and nothing is dequantized to HBM.
template <int BITS, int MAXM, int R>
__global__ __launch_bounds__(256) void int_gemv_kernel(const bf16* __restrict__ x, const int8_t* __restrict__ q,
                                                       const float* __restrict__ scales, bf16* __restrict__ y, int M,
                                                       int N, int K, int G) {
  const int lane = threadIdx.x & 63;
  const int n0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (n0 >= N) return;
  float acc[R][MAXM];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < MAXM; ++m) acc[r][m] = 0.f;
  for (int k0 = 16 * lane; k0 < K; k0 += 16 * 64) {
    bf16x8 xa[MAXM], xb[MAXM];
#pragma unroll
    for (int m = 0; m < MAXM; ++m) {
      if (m < M) {
        xa[m] = *reinterpret_cast<const bf16x8*>(x + (int64_t)m * K + k0);
        xb[m] = *reinterpret_cast<const bf16x8*>(x + (int64_t)m * K + k0 + 8);
      }
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const int n = n0 + r;
      if (n >= N) break;
      const float s = scales[(int64_t)n * (K / G) + k0 / G];
      float wv[16];
      if (BITS == 8) {
        const uint4 d = *reinterpret_cast<const uint4*>(q + (int64_t)n * K + k0);
        const uint32_t dw[4] = {d.x, d.y, d.z, d.w};
#pragma unroll
        for (int j = 0; j < 16; ++j) wv[j] = (float)(int8_t)((dw[j >> 2] >> (8 * (j & 3))) & 0xff);
      } else {
        const uint2 d = *reinterpret_cast<const uint2*>(q + ((int64_t)n * K + k0) / 2);
        const uint32_t dw[2] = {d.x, d.y};
#pragma unroll
        for (int j = 0; j < 16; ++j) wv[j] = (float)((int)((dw[j >> 3] >> (4 * (j & 7))) & 0xf) ^ 8) - 8.f;
      }
#pragma unroll
      for (int m = 0; m < MAXM; ++m) {
        if (m < M) {
          float a = 0.f;
#pragma unroll
          for (int j = 0; j < 8; ++j) a += (float)xa[m][j] * wv[j] + (float)xb[m][j] * wv[8 + j];
          acc[r][m] += a * s;  // group scale applied once per 16 weights
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < MAXM; ++m) {
      if (m < M && n0 + r < N) {
        const float v = wave_sum(acc[r][m]);
        if (lane == 0) y[(int64_t)m * N + n0 + r] = (bf16)v;
      }
    }
}

}  // namespace

#define HDS_QDISPATCH(KERNEL, T, ...)                                                  \
  do {                                                                                 \
    if (bits == 8 && sym) hipLaunchKernelGGL((KERNEL<T, 8, true>), __VA_ARGS__);       \
    else if (bits == 8) hipLaunchKernelGGL((KERNEL<T, 8, false>), __VA_ARGS__);        \
    else if (bits == 4 && sym) hipLaunchKernelGGL((KERNEL<T, 4, true>), __VA_ARGS__);  \
    else if (bits == 4) hipLaunchKernelGGL((KERNEL<T, 4, false>), __VA_ARGS__);        \
    else return hipErrorInvalidValue;                                                  \
  } while (0)

HDS_EXPORT int hds_quant_int(int dtype, const void* x, void* q, float* scales, float* mins, int64_t n_groups,
                             int group_size, int bits, int sym, hipStream_t st) {
  if (group_size % 8 || n_groups <= 0) return n_groups <= 0 ? 0 : hipErrorInvalidValue;
  const dim3 grid = grid_for(n_groups);
  if (dtype == kBF16)
    HDS_QDISPATCH(quant_int_kernel, bf16, grid, dim3(256), 0, st, (const bf16*)x, (int8_t*)q, scales, mins, n_groups,
                  group_size);
  else if (dtype == kF16)
    HDS_QDISPATCH(quant_int_kernel, _Float16, grid, dim3(256), 0, st, (const _Float16*)x, (int8_t*)q, scales, mins, n_groups,
                  group_size);
  else
    HDS_QDISPATCH(quant_int_kernel, float, grid, dim3(256), 0, st, (const float*)x, (int8_t*)q, scales, mins,
                  n_groups, group_size);
  return hipGetLastError();
}

HDS_EXPORT int hds_dequant_int(int dtype, const void* q, const float* scales, const float* mins, void* y,
                               int64_t n_groups, int group_size, int bits, int sym, hipStream_t st) {
  if (group_size % 8 || n_groups <= 0) return n_groups <= 0 ? 0 : hipErrorInvalidValue;
  const int64_t n8 = n_groups * group_size / 8;
  const dim3 grid((unsigned)std::min<int64_t>((n8 + 255) / 256, 256 * 64));
  if (dtype == kBF16)
    HDS_QDISPATCH(dequant_int_kernel, bf16, grid, dim3(256), 0, st, (const int8_t*)q, scales, mins, (bf16*)y,
                  n_groups, group_size);
  else if (dtype == kF16)
    HDS_QDISPATCH(dequant_int_kernel, _Float16, grid, dim3(256), 0, st, (const int8_t*)q, scales, mins, (_Float16*)y,
                  n_groups, group_size);
  else
    HDS_QDISPATCH(dequant_int_kernel, float, grid, dim3(256), 0, st, (const int8_t*)q, scales, mins, (float*)y,
                  n_groups, group_size);
  return hipGetLastError();
}

HDS_EXPORT int hds_quant_fp8(int dtype, const void* x, void* q, float* scales, int64_t n_groups, int group_size,
                             int e5m2, hipStream_t st) {
  if (group_size % 8 || n_groups <= 0) return n_groups <= 0 ? 0 : hipErrorInvalidValue;
  const dim3 grid = grid_for(n_groups);
#define HDS_F8(T)                                                                                                   \
  if (e5m2)                                                                                                         \
    hipLaunchKernelGGL((quant_fp8_kernel<T, true>), grid, dim3(256), 0, st, (const T*)x, (uint8_t*)q, scales,       \
                       n_groups, group_size);                                                                       \
  else                                                                                                              \
    hipLaunchKernelGGL((quant_fp8_kernel<T, false>), grid, dim3(256), 0, st, (const T*)x, (uint8_t*)q, scales,      \
                       n_groups, group_size);
  if (dtype == kBF16) {
    HDS_F8(bf16)
  } else if (dtype == kF16) {
    HDS_F8(_Float16)
  } else {
    HDS_F8(float)
  }
#undef HDS_F8
  return hipGetLastError();
}

HDS_EXPORT int hds_dequant_fp8(int dtype, const void* q, const float* scales, void* y, int64_t n_groups,
                               int group_size, int e5m2, hipStream_t st) {
  if (group_size % 8 || n_groups <= 0) return n_groups <= 0 ? 0 : hipErrorInvalidValue;
  const dim3 grid = grid_for(n_groups);
#define HDS_F8(T)                                                                                                   \
  if (e5m2)                                                                                                         \
    hipLaunchKernelGGL((dequant_fp8_kernel<T, true>), grid, dim3(256), 0, st, (const uint8_t*)q, scales, (T*)y,     \
                       n_groups, group_size);                                                                       \
  else                                                                                                              \
    hipLaunchKernelGGL((dequant_fp8_kernel<T, false>), grid, dim3(256), 0, st, (const uint8_t*)q, scales, (T*)y,    \
                       n_groups, group_size);
  if (dtype == kBF16) {
    HDS_F8(bf16)
  } else if (dtype == kF16) {
    HDS_F8(_Float16)
  } else {
    HDS_F8(float)
  }
#undef HDS_F8
  return hipGetLastError();
}

HDS_EXPORT int hds_dequant_reduce(int out_dtype, const void* q, const float* scales, void* out, int world, int64_t n,
                                  int group_size, int bits, int accumulate, hipStream_t st) {
  if (group_size % 8 || n % group_size || n <= 0) return n <= 0 ? 0 : hipErrorInvalidValue;
  const dim3 grid = grid_for(n / group_size);
#define HDS_DR(TO)                                                                                               \
  if (bits == 8)                                                                                                 \
    hipLaunchKernelGGL((dequant_reduce_kernel<TO, 8>), grid, dim3(256), 0, st, (const int8_t*)q, scales, (TO*)out, \
                       world, n, group_size, accumulate);                                                        \
  else if (bits == 4)                                                                                            \
    hipLaunchKernelGGL((dequant_reduce_kernel<TO, 4>), grid, dim3(256), 0, st, (const int8_t*)q, scales, (TO*)out, \
                       world, n, group_size, accumulate);                                                        \
  else                                                                                                           \
    return hipErrorInvalidValue;
  if (out_dtype == kF32) {
    HDS_DR(float)
  } else if (out_dtype == kBF16) {
    HDS_DR(bf16)
  } else {
    HDS_DR(_Float16)
  }
#undef HDS_DR
  return hipGetLastError();
}

// x [M, K] bf16 (M <= 8), q int8/int4-packed [N, K], scales [N, K / G] -> y [M, N] bf16
HDS_EXPORT int hds_int_gemv(const void* x, const void* q, const float* scales, void* y, int M, int N, int K, int G,
                            int bits, hipStream_t st) {
  if (M <= 0 || M > 8 || K % 16 || G % 16 || K % G || (bits != 8 && bits != 4)) return hipErrorInvalidValue;
  // R = 4 rows per wave when that still gives >= 1024 blocks (x reuse), else one row per wave (parallelism)
#define HDS_IG(B, MM, RR)                                                                                           \
  hipLaunchKernelGGL((int_gemv_kernel<B, MM, RR>), dim3((N + 4 * RR - 1) / (4 * RR)), dim3(256), 0, st,           \
                     (const bf16*)x, (const int8_t*)q, scales, (bf16*)y, M, N, K, G)
#define HDS_IGM(B, RR)                                                                                             \
  if (M == 1) HDS_IG(B, 1, RR); else if (M <= 2) HDS_IG(B, 2, RR); else if (M <= 4) HDS_IG(B, 4, RR);              \
  else HDS_IG(B, 8, RR);
  const bool wide = N >= 16 * 1024;
  if (bits == 8) {
    if (wide) { HDS_IGM(8, 4) } else { HDS_IGM(8, 1) }
  } else {
    if (wide) { HDS_IGM(4, 4) } else { HDS_IGM(4, 1) }
  }
#undef HDS_IGM
#undef HDS_IG
  return hipGetLastError();
}
