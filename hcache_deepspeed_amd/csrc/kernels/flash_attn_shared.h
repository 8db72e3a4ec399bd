// Shared by the FlashAttention translation units (flash_attn.hip, flash_attn_w64.hip): launch parameters,
// sequence / mask helpers and the LDS read wrappers. Anonymous namespace: every TU has its own copy; the
// parameter block crosses TUs only as bytes of this one definition (hds_attn_fwd_w64_launch).
#pragma once
// A/B experiment build of the FlashAttention units (ops/build.py build_kernels_diag): 1 adds the earlier forward
// schedules, the cycle-stamp builds and the timing-only (wrong-result) diagnostics to a separate library. The shipped
// library is built without it and carries none of them.
#ifndef HDS_FA_DIAG
#define HDS_FA_DIAG 0
#endif
#include <type_traits>
#include <utility>

#include "attn_common.h"

namespace {
using namespace hds;
using namespace hds::attn;

constexpr int BN = 64;   // keys per LDS tile (fwd, dq) / query rows per tile (dkdv)
// query rows per workgroup (fwd, dq) = 32 * NW ; keys per workgroup (dkdv) = 32 * NW
constexpr float kLog2e = 1.4426950408889634f;

struct AttnParams {
  const bf16* q;
  const bf16* k;
  const bf16* v;
  bf16* o;
  float* lse;  // [Hq][total_tokens], natural-log units of (scale * q.k)
  const bf16* dout;
  bf16* dq;
  bf16* dk;
  bf16* dv;
  float* delta;  // [Hq][total_tokens]
  float* lse2;   // [Hq][total_tokens] lse * log2(e), written by the delta pre-kernel (null: not wanted)
  int64_t sq, sk, sv, so, sdo, sdq, sdk, sdv;  // token strides (elements)
  const int* cu_seqlens;                       // [B+1] or null
  const int* seq_lens;                         // [B] valid lengths of a right-padded batch (null: all seq_len)
  int seq_len;                                 // when cu_seqlens is null
  int total_tokens;
  int batch, hq, hkv;
  float scale;
  int causal;
  int window;  // >0: sliding window (keys in (q - window, q])
  // Evoformer (EVO kernels only): additive biases and their gradients, batch = B * evo_n sequences of seq_len
  const void* b1;  // [B*N][L]        (bf16 or fp32, bias_f32)
  const void* b2;  // [B][H][L][L]
  int bias_f32;
  float* db1;      // [B*N][L]  fp32, accumulated
  float* db2;      // [B][H][L][L] fp32, accumulated
  int evo_n;
};

__device__ __forceinline__ float ld_bias(const AttnParams& p, const void* base, int64_t i) {
  return p.bias_f32 ? reinterpret_cast<const float*>(base)[i] : (float)reinterpret_cast<const bf16*>(base)[i];
}

// Evoformer pair / mask bias of (sequence bn, head h, query q, key) (indices clamped; masked() zeroes padding)
__device__ __forceinline__ float evo_bias(const AttnParams& p, int bn, int h, int q, int key) {
  const int L = p.seq_len;
  q = q < L ? q : L - 1;
  key = key < L ? key : L - 1;
  float x = 0.f;
  if (p.b1) x += ld_bias(p, p.b1, (int64_t)bn * L + key);
  if (p.b2) x += ld_bias(p, p.b2, ((int64_t)((bn / p.evo_n) * p.hq + h) * L + q) * L + key);
  return x;
}

__device__ __forceinline__ void seq_bounds(const AttnParams& p, int b, int& start, int& len) {
  if (p.cu_seqlens) {
    start = p.cu_seqlens[b];
    len = p.cu_seqlens[b + 1] - start;
  } else {
    start = b * p.seq_len;
    len = p.seq_lens ? p.seq_lens[b] : p.seq_len;
  }
}

// Launch grids are (blocks-per-sequence, heads, batch); reinterpret the linear workgroup id so the
// block index within a sequence varies SLOWEST: the dispatcher then starts every (head, batch)'s
// heaviest causal block before any lighter one (longest-processing-time-first across 256 CUs).
__device__ __forceinline__ void lpt_ids(int& blk, int& head, int& b) {
  const int heads = gridDim.y, nb = gridDim.z;
  const int lid = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);
  blk = lid / (heads * nb);
  const int rem = lid - blk * heads * nb;
  head = rem % heads;
  b = rem / heads;
}

// The per-element mask as an interval test (two compares, no branches): the keys a query may see, or the queries
// that may see a key, form [lo, hi] (empty when lo > hi). Same predicate as masked() below.
__device__ __forceinline__ void key_span(const AttnParams& p, int qi, int len, int& lo, int& hi) {
  lo = p.window > 0 ? max(0, qi - p.window + 1) : 0;
  hi = p.causal ? min(qi, len - 1) : len - 1;
  if (qi >= len) lo = 1, hi = 0;
}
__device__ __forceinline__ void query_span(const AttnParams& p, int kj, int len, int& lo, int& hi) {
  lo = p.causal ? kj : 0;
  hi = p.window > 0 ? min(len - 1, kj + p.window - 1) : len - 1;
  if (kj >= len) lo = 1, hi = 0;
}
__device__ __forceinline__ bool outside(int i, int lo, int hi) { return i < lo || i > hi; }

__device__ __forceinline__ bool masked(const AttnParams& p, int qi, int kj, int len) {
  if (kj >= len || qi >= len) return true;
  if (p.causal && kj > qi) return true;
  if (p.window > 0 && kj <= qi - p.window) return true;
  return false;
}

// =====================================================================================
// forward
// =====================================================================================
// VAR bit 0: static s_setprio(1) for the second-dispatched half of the waves (guide T5 static form);
// VAR bit 1: deferred running-max update -- the max (and the O / l rescale) only moves when some row of the
//            wave grew by more than kDeferThr (log2 units), so P stays <= 2^kDeferThr (guide T13).
constexpr float kDeferThr = 8.f;

template <int IMM>
__device__ __forceinline__ bf16x8 lds_b128(uint32_t a) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(a), "n"(IMM) : "memory");
  return r;
}
template <int IMM>
__device__ __forceinline__ bf16x8 lds_tr8(uint32_t a0, uint32_t a1) {
  bf16x4 lo, hi;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(a0), "n"(IMM) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(a1), "n"(IMM) : "memory");
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
template <int... I, typename F>
__device__ __forceinline__ void static_for_impl(std::integer_sequence<int, I...>, F&& f) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  static_for_impl(std::make_integer_sequence<int, N>{}, f);
}

// one LDS-DMA piece of K or V tile through a buffer descriptor built from plain scalars (the descriptor type does not
// exist in the host pass, so no lambda may hold one): base = the tile's first row of this kv head, records = the bytes
// up to the end of the tile's last row inside the sequence -- the range check zero-fills the pieces of rows past it
struct TileSrc {
  const char* base;
  int bytes;
};
template <int D>
__device__ __forceinline__ TileSrc tile_src(const bf16* base, int64_t stride, int start, int kt, int hk, int len) {
  const int rows = min(BN, len - kt * BN);
  return {(const char*)(base + (int64_t)(start + kt * BN) * stride + (int64_t)hk * D),
          (int)(((int64_t)(rows - 1) * stride + D) * 2)};
}
__device__ __forceinline__ void tile_dma(const TileSrc& t, void* lds, int32_t off) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(__builtin_amdgcn_make_buffer_rsrc((void*)t.base, (short)0, t.bytes, 0x00020000),
                                           (lds_void*)lds, 16, off, 0, 0, 0);
}

}  // namespace
