// Single-query (decode) attention over a contiguous per-sequence KV cache -- the inference-v1 "softmax_context"
// path for HF-style caches [B, Hkv, S, D] (reference csrc/transformer/inference/csrc/pt_binding.cpp:1969-2036
// ds_softmax_context + the KV-cache attention kernels).
//
//   o[b, h, :] = softmax(scale * q[b, h] . K[b, h / G]^T + bias[b, :] + alibi[h] * (j - (S - 1))) . V[b, h / G]
//
// Decode is a pure K/V stream (2 * S * D bytes per (b, kv-head)), so the kernel is built for bandwidth:
//   * grid (splits, Hkv, B); a workgroup (4 waves) owns one (b, kv head) and a contiguous key range, and serves
//     ALL G = H / Hkv query heads of that kv head from one read of K and V (no repeat_interleave copies);
//   * a wave reads 64 / LPK keys per instruction, LPK = D / 8 lanes per key, 16 B (8 bf16) per lane; the q . k
//     partial dot products reduce over the LPK lanes of a key with xor-shuffles;
//   * online softmax per (lane group, head), P . V accumulated in registers (o[G][8] per lane);
//   * lane groups, waves and key splits are merged by max / rescale -- splits through fp32 partials and a small
//     combine kernel (split-K "flash decoding"), chosen so B * Hkv * splits fills the 256 CUs.
#include "hds_common.h"

using namespace hds;

namespace {

constexpr int kGMax = 8;  // query heads per kv head served by one workgroup

struct DecodeParams {
  const bf16* q;      // [B, H, D] (strides sqb, sqh)
  const bf16* k;      // [B, Hkv, S, D] (strides skb, skh, sks)
  const bf16* v;
  const float* bias;  // [B, S] additive (may be null)
  const float* alibi; // [H] slopes (may be null)
  bf16* o;            // [B, H, D] contiguous
  float* part_o;      // [B, H, splits, D]
  float* part_ml;     // [B, H, splits, 2]
  int64_t sqb, sqh, skb, skh, sks, svb, svh, svs, sbias;
  int B, H, Hkv, S, splits, keys_per_split;
  float scale;
  const int* lens;  // [B] valid keys per sequence, read on the device (may be null: S); HIP-graph decode
  int window;       // > 0: only the last `window` valid keys attend
};

template <int D>
__global__ __launch_bounds__(256) void decode_attn_kernel(DecodeParams p) {
  constexpr int LPK = D / 8;        // lanes per key
  constexpr int KPW = 64 / LPK;     // keys per wave step
  __shared__ float red[4][kGMax][2 + D];

  const int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int G = p.H / p.Hkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kl = lane / LPK, c = lane % LPK;  // key slot in the wave step, 8-element chunk of the row
  // valid key range [jb, Se): the cache buffer holds S slots, the sequence fills the first lens[b] of them
  const int Se = p.lens ? min(p.S, p.lens[b]) : p.S;
  const int jb = p.window > 0 ? max(0, Se - p.window) : 0;
  const int j0 = split * p.keys_per_split;
  const int j1 = min(Se, j0 + p.keys_per_split);

  float qv[kGMax][8];
#pragma unroll
  for (int g = 0; g < kGMax; ++g) {
    if (g < G) {
      Vec8<bf16>::load(p.q + b * p.sqb + (int64_t)(hk * G + g) * p.sqh + c * 8, qv[g]);
#pragma unroll
      for (int e = 0; e < 8; ++e) qv[g][e] *= p.scale;
    }
  }
  float slope[kGMax];
#pragma unroll
  for (int g = 0; g < kGMax; ++g) slope[g] = (p.alibi && g < G) ? p.alibi[hk * G + g] : 0.f;

  float m[kGMax], l[kGMax], acc[kGMax][8];
#pragma unroll
  for (int g = 0; g < kGMax; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[g][e] = 0.f;
  }
  const bf16* kb = p.k + b * p.skb + hk * p.skh + c * 8;
  const bf16* vb = p.v + b * p.svb + hk * p.svh + c * 8;
  for (int j = j0 + w * KPW + kl; j - kl < j1; j += 4 * KPW) {
    const bool ok = j < j1 && j >= jb;
    float kv[8] = {}, vv[8] = {};  // masked lanes still run the (e_s = 0) update: keep NaN bits out of acc
    if (ok) {
      Vec8<bf16>::load(kb + (int64_t)j * p.sks, kv);
      Vec8<bf16>::load(vb + (int64_t)j * p.svs, vv);
    }
    const float bj = (ok && p.bias) ? p.bias[b * p.sbias + j] : 0.f;
#pragma unroll
    for (int g = 0; g < kGMax; ++g) {
      if (g >= G) break;
      float s = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) s += qv[g][e] * kv[e];
#pragma unroll
      for (int off = LPK / 2; off >= 1; off >>= 1) s += __shfl_xor(s, off, 64);
      s = ok ? s + bj + slope[g] * (float)(j - (Se - 1)) : -INFINITY;
      const float mn = fmaxf(m[g], s);
      const bool none = mn == -INFINITY;  // nothing valid yet for this lane group (selects keep lanes converged)
      const float a = none ? 1.f : __expf(m[g] - mn), e_s = none ? 0.f : __expf(s - mn);
      l[g] = l[g] * a + e_s;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[g][e] = acc[g][e] * a + e_s * vv[e];
      m[g] = mn;
    }
  }
  // merge the KPW lane groups of the wave (lanes with the same chunk c)
#pragma unroll
  for (int g = 0; g < kGMax; ++g) {
    if (g >= G) break;
#pragma unroll
    for (int off = LPK; off < 64; off <<= 1) {
      const float mo = __shfl_xor(m[g], off, 64), lo = __shfl_xor(l[g], off, 64);
      const float mn = fmaxf(m[g], mo);
      const float a = mn == -INFINITY ? 0.f : __expf(m[g] - mn), ao = mn == -INFINITY ? 0.f : __expf(mo - mn);
      l[g] = l[g] * a + lo * ao;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[g][e] = acc[g][e] * a + __shfl_xor(acc[g][e], off, 64) * ao;
      m[g] = mn;
    }
  }
  // merge the 4 waves through LDS (lanes 0..LPK-1 of each wave hold the wave's result)
  if (kl == 0) {
#pragma unroll
    for (int g = 0; g < kGMax; ++g) {
      if (g >= G) break;
      if (c == 0) {
        red[w][g][0] = m[g];
        red[w][g][1] = l[g];
      }
#pragma unroll
      for (int e = 0; e < 8; ++e) red[w][g][2 + c * 8 + e] = acc[g][e];
    }
  }
  __syncthreads();
  // thread t < G * D/8 ... finalise one (g, chunk)
  for (int t = threadIdx.x; t < G * LPK; t += 256) {
    const int g = t / LPK, cc = t % LPK;
    float mm = -INFINITY;
    for (int ww = 0; ww < 4; ++ww) mm = fmaxf(mm, red[ww][g][0]);
    float ll = 0.f, oo[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int ww = 0; ww < 4; ++ww) {
      const float a = mm == -INFINITY ? 0.f : __expf(red[ww][g][0] - mm);
      ll += red[ww][g][1] * a;
#pragma unroll
      for (int e = 0; e < 8; ++e) oo[e] += red[ww][g][2 + cc * 8 + e] * a;
    }
    const int h = hk * G + g;
    if (p.splits == 1) {
      const float inv = ll > 0.f ? 1.f / ll : 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) oo[e] *= inv;
      Vec8<bf16>::store(p.o + ((int64_t)b * p.H + h) * D + cc * 8, oo);
    } else {
      float* po = p.part_o + (((int64_t)b * p.H + h) * p.splits + split) * D + cc * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) po[e] = oo[e];
      if (cc == 0) {
        float* pm = p.part_ml + (((int64_t)b * p.H + h) * p.splits + split) * 2;
        pm[0] = mm;
        pm[1] = ll;
      }
    }
  }
}

template <int D>
__global__ __launch_bounds__(256) void decode_combine_kernel(DecodeParams p) {
  // one workgroup per (b, h): threads over D
  const int bh = blockIdx.x;
  const float* pm = p.part_ml + (int64_t)bh * p.splits * 2;
  float mm = -INFINITY;
  for (int s = 0; s < p.splits; ++s) mm = fmaxf(mm, pm[2 * s]);
  for (int d = threadIdx.x; d < D; d += blockDim.x) {
    float ll = 0.f, oo = 0.f;
    for (int s = 0; s < p.splits; ++s) {
      const float a = mm == -INFINITY ? 0.f : __expf(pm[2 * s] - mm);
      ll += pm[2 * s + 1] * a;
      oo += p.part_o[((int64_t)bh * p.splits + s) * D + d] * a;
    }
    p.o[(int64_t)bh * D + d] = (bf16)(ll > 0.f ? oo / ll : 0.f);
  }
}

}  // namespace

HDS_EXPORT int hds_decode_attn_supported(int D, int G) { return (D == 64 || D == 128 || D == 256) && G >= 1 && G <= kGMax; }

// Returns the number of key splits to use (the caller sizes the fp32 partial buffers from it).
HDS_EXPORT int hds_decode_attn_splits(int B, int Hkv, int S) {
  const int groups = B * Hkv;
  int splits = (512 + groups - 1) / groups;          // >= 2 workgroups per CU overall
  // >= 32 keys per split: a split's waves walk their keys with one dependent K/V load per step, so at short
  // contexts (a few hundred keys, B * Hkv = 8) the HBM latency of those steps, not bandwidth, sets the time
  const int max_by_len = (S + 31) / 32;
  splits = splits < max_by_len ? splits : max_by_len;
  return splits < 1 ? 1 : (splits > 64 ? 64 : splits);
}

// ``lens`` (device [B] int32, or null) bounds each sequence's keys inside the S-slot cache on the device, so one
// launch shape serves every decode step (HIP-graph replay); ``window`` > 0 keeps only the last window keys.
HDS_EXPORT int hds_decode_attn_len(const void* q, int64_t sqb, int64_t sqh, const void* k, int64_t skb,
                                   int64_t skh, int64_t sks, const void* v, int64_t svb, int64_t svh, int64_t svs,
                                   const float* bias, int64_t sbias, const float* alibi, void* o, float* part_o,
                                   float* part_ml, int B, int H, int Hkv, int S, int D, int splits, float scale,
                                   const int* lens, int window, hipStream_t st) {
  if (B <= 0 || S <= 0 || Hkv <= 0 || H % Hkv || !hds_decode_attn_supported(D, H / Hkv) || splits < 1 ||
      (splits > 1 && (!part_o || !part_ml)) || window < 0)
    return (int)hipErrorInvalidValue;
  const int kps = (S + splits - 1) / splits;
  DecodeParams p{(const bf16*)q, (const bf16*)k, (const bf16*)v, bias, alibi, (bf16*)o, part_o, part_ml,
                 sqb, sqh, skb, skh, sks, svb, svh, svs, sbias, B, H, Hkv, S, splits, kps, scale, lens, window};
  const dim3 grid(splits, Hkv, B);
  switch (D) {
    case 64:
      hipLaunchKernelGGL(decode_attn_kernel<64>, grid, dim3(256), 0, st, p);
      if (splits > 1) hipLaunchKernelGGL(decode_combine_kernel<64>, dim3(B * H), dim3(64), 0, st, p);
      break;
    case 128:
      hipLaunchKernelGGL(decode_attn_kernel<128>, grid, dim3(256), 0, st, p);
      if (splits > 1) hipLaunchKernelGGL(decode_combine_kernel<128>, dim3(B * H), dim3(128), 0, st, p);
      break;
    default:
      hipLaunchKernelGGL(decode_attn_kernel<256>, grid, dim3(256), 0, st, p);
      if (splits > 1) hipLaunchKernelGGL(decode_combine_kernel<256>, dim3(B * H), dim3(256), 0, st, p);
  }
  return (int)hipGetLastError();
}

HDS_EXPORT int hds_decode_attn(const void* q, int64_t sqb, int64_t sqh, const void* k, int64_t skb, int64_t skh,
                               int64_t sks, const void* v, int64_t svb, int64_t svh, int64_t svs, const float* bias,
                               int64_t sbias, const float* alibi, void* o, float* part_o, float* part_ml, int B,
                               int H, int Hkv, int S, int D, int splits, float scale, hipStream_t st) {
  return hds_decode_attn_len(q, sqb, sqh, k, skb, skh, sks, v, svb, svh, svs, bias, sbias, alibi, o, part_o, part_ml,
                             B, H, Hkv, S, D, splits, scale, nullptr, 0, st);
}

// ---------------------------------------------------------------------------------------------------------------
// KV append for the HIP-graph decode step: K and V of one new token per sequence written into cache slot
// cur[0] (read on the device) of [B, Hkv, S, D] caches, one launch for both tensors (two index_copy kernels
// before). Workgroup = one (b, kv head), 16-B vectors along D.
// ---------------------------------------------------------------------------------------------------------------
namespace {
__global__ __launch_bounds__(64) void kv_append_kernel(const bf16* __restrict__ k, int64_t skb, int64_t skh,
                                                       const bf16* __restrict__ v, int64_t svb, int64_t svh,
                                                       bf16* __restrict__ kc, int64_t ckb, int64_t ckh,
                                                       int64_t cks, bf16* __restrict__ vc, int64_t cvb, int64_t cvh,
                                                       int64_t cvs, const int64_t* __restrict__ cur, int Hkv, int D) {
  const int b = blockIdx.x / Hkv, h = blockIdx.x % Hkv;
  const int64_t s = cur[0];
  for (int c = threadIdx.x * 8; c < D; c += 64 * 8) {
    *reinterpret_cast<bf16x8*>(kc + b * ckb + h * ckh + s * cks + c) =
        *reinterpret_cast<const bf16x8*>(k + b * skb + h * skh + c);
    *reinterpret_cast<bf16x8*>(vc + b * cvb + h * cvh + s * cvs + c) =
        *reinterpret_cast<const bf16x8*>(v + b * svb + h * svh + c);
  }
}
}  // namespace

HDS_EXPORT int hds_kv_append(const void* k, int64_t skb, int64_t skh, const void* v, int64_t svb, int64_t svh, void* kc,
                             int64_t ckb, int64_t ckh, int64_t cks, void* vc, int64_t cvb, int64_t cvh, int64_t cvs,
                             const int64_t* cur, int B, int Hkv, int D, hipStream_t st) {
  if (B <= 0 || Hkv <= 0 || D % 8 || !cur) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(kv_append_kernel, dim3(B * Hkv), dim3(64), 0, st, (const bf16*)k, skb, skh, (const bf16*)v, svb,
                     svh, (bf16*)kc, ckb, ckh, cks, (bf16*)vc, cvb, cvh, cvs, cur, Hkv, D);
  return (int)hipGetLastError();
}
