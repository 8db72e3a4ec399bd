// Group-wise quantization: INT8 / INT4 (symmetric or asymmetric) and FP8 (OCP e4m3 / e5m2 via the
// gfx950 conversion instructions), dequantization, and the ZeRO++ qgZ "dequantize + reduce" of the
// chunks received from every rank in a quantized reduce-scatter.
//
// Capability parity: csrc/quantization/quantize.cu (`cached_quantization`, K16), dequantize.cu /
// quantize_intX.cu (K17), quant_reduce.cu (`dequant_reduce`, K19), csrc/fp_quantizer/fp_quantize.cu
// (`apply_quantization` / `apply_dequantization`, K21). One wave64 owns one group (group_size up to
// 8192 elements, a multiple of 8): 16-byte vector loads, wave-level absmax / min-max through
// __shfl_xor, scales kept in fp32. INT4 packs two values per byte (low nibble = even element).
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

template <typename T, int BITS, bool SYM>
__global__ __launch_bounds__(256) void dequant_int_kernel(const int8_t* __restrict__ q, const float* __restrict__ scales,
                                                          const float* __restrict__ mins, T* __restrict__ y,
                                                          int64_t n_groups, int group_size) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * kWaves + (threadIdx.x >> 6);
  if (g >= n_groups) return;
  const float s = scales[g];
  const float lo = SYM ? 0.f : mins[g];
  for (int c = lane * 8; c < group_size; c += 64 * 8) {
    float v[8];
    if (BITS == 8) {
      const uint2 w = *reinterpret_cast<const uint2*>(q + g * group_size + c);
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int a = SYM ? (int)(int8_t)((w.x >> (8 * i)) & 0xff) : (int)((w.x >> (8 * i)) & 0xff);
        const int b = SYM ? (int)(int8_t)((w.y >> (8 * i)) & 0xff) : (int)((w.y >> (8 * i)) & 0xff);
        v[i] = a * s + lo;
        v[4 + i] = b * s + lo;
      }
    } else {
      const uint32_t w = *reinterpret_cast<const uint32_t*>(q + (g * group_size + c) / 2);
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        int n = (w >> (4 * i)) & 0xf;
        if (SYM) n = (n ^ 8) - 8;  // sign-extend the nibble
        v[i] = n * s + lo;
      }
    }
    Vec8<T>::store(y + g * group_size + c, v);
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
  const dim3 grid = grid_for(n_groups);
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
