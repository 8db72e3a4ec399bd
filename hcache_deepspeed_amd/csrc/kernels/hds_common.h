// Shared device helpers for the gfx950 (CDNA4) kernels of hcache_deepspeed_amd.
//
// Everything here is written for wave64 / MI355X only:
//   * 16-byte vector I/O (8 x bf16 per lane) for every memory-bound kernel,
//   * wave reductions with __shfl_xor over 64 lanes,
//   * bf16 <-> f32 conversions through the native __bf16 type (gfx950 has
//     v_cvt_pk_bf16_f32, the compiler emits it for the casts below).
//
// Replaces the role of csrc/includes/{reduction_utils.h,memory_access_utils.h,
// conversion_utils.h} of the reference -- not a translation:
// there is no warp-size abstraction and no cooperative-groups layer here.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HDS_EXPORT extern "C" __attribute__((visibility("default")))

namespace hds {

constexpr int kWave = 64;

typedef __bf16 bf16;
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));

// dtype codes shared with python (hcache_deepspeed_amd/ops/native.py)
enum DType : int { kF32 = 0, kBF16 = 1, kF16 = 2 };

__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
__device__ __forceinline__ float to_f(_Float16 x) { return (float)x; }
template <typename T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }
template <> __device__ __forceinline__ _Float16 from_f<_Float16>(float x) { return (_Float16)x; }

// 8-element vector load/store in f32 registers. For bf16/f16 this is ONE
// 16-byte global access per lane; for f32 two 16-byte accesses.
template <typename T> struct Vec8;
template <> struct Vec8<bf16> {
  __device__ __forceinline__ static void load(const bf16* p, float (&v)[8]) {
    bf16x8 r = *reinterpret_cast<const bf16x8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)r[i];
  }
  __device__ __forceinline__ static void store(bf16* p, const float (&v)[8]) {
    bf16x8 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = (bf16)v[i];
    *reinterpret_cast<bf16x8*>(p) = r;
  }
};
template <> struct Vec8<_Float16> {
  typedef _Float16 h8 __attribute__((ext_vector_type(8)));
  __device__ __forceinline__ static void load(const _Float16* p, float (&v)[8]) {
    h8 r = *reinterpret_cast<const h8*>(p);
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = (float)r[i];
  }
  __device__ __forceinline__ static void store(_Float16* p, const float (&v)[8]) {
    h8 r;
#pragma unroll
    for (int i = 0; i < 8; ++i) r[i] = (_Float16)v[i];
    *reinterpret_cast<h8*>(p) = r;
  }
};
template <> struct Vec8<float> {
  __device__ __forceinline__ static void load(const float* p, float (&v)[8]) {
    f32x4 a = *reinterpret_cast<const f32x4*>(p);
    f32x4 b = *reinterpret_cast<const f32x4*>(p + 4);
    v[0] = a[0]; v[1] = a[1]; v[2] = a[2]; v[3] = a[3];
    v[4] = b[0]; v[5] = b[1]; v[6] = b[2]; v[7] = b[3];
  }
  __device__ __forceinline__ static void store(float* p, const float (&v)[8]) {
    f32x4 a = {v[0], v[1], v[2], v[3]}, b = {v[4], v[5], v[6], v[7]};
    *reinterpret_cast<f32x4*>(p) = a;
    *reinterpret_cast<f32x4*>(p + 4) = b;
  }
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}

// Block-wide sum for blockDim.x == NT (multiple of 64). `red` must hold NT/64 floats.
template <int NT>
__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = 0.f;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r += red[i];
  __syncthreads();
  return r;
}
template <int NT>
__device__ __forceinline__ float block_max(float v, float* red) {
  v = wave_max(v);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float r = -INFINITY;
#pragma unroll
  for (int i = 0; i < NT / 64; ++i) r = fmaxf(r, red[i]);
  __syncthreads();
  return r;
}

// Grid size for a memory-bound grid-stride kernel: enough blocks to fill
// 256 CUs several times over without paying launch cost for millions of blocks.
__host__ inline int stream_grid(int64_t work_items, int per_block, int cap = 2048) {
  int64_t g = (work_items + per_block - 1) / per_block;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace hds
