// Serving kernels over the paged (blocked) KV cache: fused RoPE + KV scatter, and ragged
// prefill/decode attention that reads K/V through per-sequence block tables.
//
// Capability parity: deepspeed/inference/v2/kernels/ragged_ops/linear_blocked_kv_rotary
// (`kv_rotary_pos_kernel`, SURVEY §2.11 K31 -- also the only kernel the HCache `restore_kv`
// path runs) and blocked_flash (`run_mha_fwd` over AttentionAtoms, K32, a prebuilt NVIDIA-only
// library in the reference).
//
// Cache layout per layer (same as the reference BlockedKVCache): [num_blocks, block_size, 2, Hkv, D]
// (K then V for each slot). Any block_size works: every staged tile row computes its own
// (block, slot) address, and LDS-DMA takes a per-lane global source address.
//
// Head dims: every multiple of 16 up to 256 that flash_attn.hip instantiates (HDS_PAGED_DIMS below), via the
// generic tile helpers of attn_common.h. The RoPE scatter takes any head_dim % 4 == 0 with a rotary prefix
// of rot_dim (% 8 == 0) dims -- partial rotary (Phi, GPT-NeoX) rotates the prefix and copies the rest.
//
// Attention work unit ("atom"): (sequence, kv head, 128 packed rows). Rows pack the G = Hq/Hkv
// query heads that share a kv head with the tokens of the chunk (row = token * G + head_in_group),
// so K/V of a kv head are read ONCE for all of its query heads -- for decode (1 token) one wave
// serves the whole GQA group from a single pass over the sequence's KV blocks.
#include "attn_common.h"

using namespace hds;
using namespace hds::attn;

namespace {

constexpr int BN = 64;
constexpr float kLog2e = 1.4426950408889634f;

// ------------------------------------------------------------------------------------------
// fused RoPE (q in place, k rotated into the cache) + V copy into the cache
// ------------------------------------------------------------------------------------------
template <typename T>
struct Vec4 {  // 4 x 16-bit elements = one 8-byte access
  typedef uint32_t u2 __attribute__((ext_vector_type(2)));
  __device__ __forceinline__ static void load(const T* p, float (&v)[4]) {
    const u2 r = *reinterpret_cast<const u2*>(p);
    const T* e = reinterpret_cast<const T*>(&r);
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = (float)e[i];
  }
  __device__ __forceinline__ static void store(T* p, const float (&v)[4]) {
    u2 r;
    T* e = reinterpret_cast<T*>(&r);
#pragma unroll
    for (int i = 0; i < 4; ++i) e[i] = (T)v[i];
    *reinterpret_cast<u2*>(p) = r;
  }
};

// per head: rot/8 rotation groups of 4 pairs (i, i + rot/2), then (D - rot)/4 plain 4-element chunks. 4-element
// granularity covers every rotary prefix the HF families use (Phi partial_rotary 0.4 / 0.5 of 80 -> 32 / 40).
template <typename T>
__global__ __launch_bounds__(256) void kv_rope_scatter_kernel(T* __restrict__ qkv, int64_t sq, T* __restrict__ cache,
                                                              const int* __restrict__ tok_seq,
                                                              const int* __restrict__ tok_pos,
                                                              const int* __restrict__ block_tables, int max_blocks,
                                                              const float* __restrict__ cos_t,
                                                              const float* __restrict__ sin_t, int n_tok, int hq,
                                                              int hkv, int D, int rot, int block_size, int rotate_q,
                                                              int do_rope) {
  const int half = rot / 2;
  const int nrot = rot / 8;
  const int gph = nrot + (D - rot) / 4;
  const int heads = hq + 2 * hkv;
  const int64_t total = (int64_t)n_tok * heads * gph;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int t = (int)(idx / (heads * gph));
    const int rem = (int)(idx - (int64_t)t * heads * gph);
    const int h = rem / gph, g = rem - h * gph;
    if (h < hq && !rotate_q) continue;
    const int pos = tok_pos[t];
    T* src = qkv + (int64_t)t * sq + (int64_t)h * D;
    T* dst = nullptr;
    if (h >= hq) {
      const int kv = (h < hq + hkv) ? 0 : 1;
      const int hk = h - hq - kv * hkv;
      const int seq = tok_seq[t];
      const int blk = block_tables[(int64_t)seq * max_blocks + pos / block_size];
      const int slot = pos % block_size;
      dst = cache + ((((int64_t)blk * block_size + slot) * 2 + kv) * hkv + hk) * D;
    }
    if (g >= nrot) {  // un-rotated tail (and every V chunk past the rotary prefix)
      if (dst == nullptr) continue;
      const int c0 = rot + (g - nrot) * 4;
      float a[4];
      Vec4<T>::load(src + c0, a);
      Vec4<T>::store(dst + c0, a);
      continue;
    }
    float a[4], b[4];
    Vec4<T>::load(src + g * 4, a);
    Vec4<T>::load(src + half + g * 4, b);
    if (h < hq + hkv && do_rope) {
      const f32x4 c = *reinterpret_cast<const f32x4*>(cos_t + (int64_t)pos * half + g * 4);
      const f32x4 sn = *reinterpret_cast<const f32x4*>(sin_t + (int64_t)pos * half + g * 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float oa = a[j] * c[j] - b[j] * sn[j];
        const float ob = b[j] * c[j] + a[j] * sn[j];
        a[j] = oa;
        b[j] = ob;
      }
    }
    T* out = dst != nullptr ? dst : src;  // q rotates in place
    Vec4<T>::store(out + g * 4, a);
    Vec4<T>::store(out + half + g * 4, b);
  }
}

// ------------------------------------------------------------------------------------------
// paged attention (ragged prefill + decode)
// ------------------------------------------------------------------------------------------
struct PagedParams {
  const bf16* q;  // [T, Hq, D] rows with token stride sq
  int64_t sq;
  const bf16* cache;  // layer base: [num_blocks, block_size, 2, Hkv, D]
  bf16* o;            // [T, Hq, D] contiguous
  const int* atoms;   // [n_atoms][3] = {seq, kv_head, row_start}
  const int* seq_meta;  // [n_seqs][3] = {q_start, n_new, seen}
  const int* block_tables;
  int max_blocks;
  int block_size;
  int hq, hkv;
  float scale;
  int window;
};

template <int D, int NW>
__global__ __launch_bounds__(64 * NW) void paged_attn_kernel(PagedParams p) {
  constexpr int KS = Dim<D>::KS, DT = Dim<D>::DT, TL = Dim<D>::TILE;
  __shared__ __attribute__((aligned(16))) char smem[4 * TL];  // K[2], V[2]
  const int* at = p.atoms + blockIdx.x * 3;
  const int seq = at[0], hk = at[1], row_start = at[2];
  const int q_start = p.seq_meta[seq * 3], n_new = p.seq_meta[seq * 3 + 1], seen = p.seq_meta[seq * 3 + 2];
  const int G = p.hq / p.hkv;
  const int n_rows = n_new * G;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int myrow = row_start + 32 * w + (lane & 31);
  const bool row_ok = myrow < n_rows;
  const int rr = row_ok ? myrow : n_rows - 1;
  const int tok = rr / G, head = hk * G + rr % G;
  const int qpos = seen + tok;  // absolute position of this row's query
  const float c = p.scale * kLog2e;
  const int* table = p.block_tables + (int64_t)seq * p.max_blocks;
  const int64_t kv_row = 2LL * p.hkv * D;  // elements between consecutive slots

  bf16x8 qf[KS];
  {
    const bf16* qp = p.q + (int64_t)(q_start + tok) * p.sq + (int64_t)head * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
  }
  // last query position covered by this workgroup (rows are token-major)
  const int last_row = min(row_start + 32 * NW, n_rows) - 1;
  const int wg_qpos_max = seen + last_row / G;
  const int ctx = wg_qpos_max + 1;
  const int kt_end = (ctx + BN - 1) / BN;
  int kt_begin = 0;
  if (p.window > 0) {
    const int first = seen + (row_start / G) - p.window + 1;
    kt_begin = first > 0 ? first / BN : 0;
  }
  auto rowp = [&](int kt, int kv) {
    return [=](int row) {
      int pos = kt * BN + row;
      pos = pos < ctx ? pos : ctx - 1;
      const int blk = table[pos / p.block_size];
      return p.cache + ((int64_t)blk * p.block_size + pos % p.block_size) * kv_row + (int64_t)kv * p.hkv * D +
             (int64_t)hk * D;
    };
  };
  const int w_row_lo = row_start + 32 * w;
  const int w_qpos_lo = seen + min(w_row_lo, n_rows - 1) / G;
  const int w_qpos_hi = seen + min(w_row_lo + 31, n_rows - 1) / G;
  const bool wave_active = w_row_lo < n_rows;

  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = f32x16{};
  float m = -INFINITY, l = 0.f;

  stage_tile_d<NW, D>(smem, rowp(kt_begin, 0));
  stage_tile_d<NW, D>(smem + 2 * TL, rowp(kt_begin, 1));
  __syncthreads();
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const int buf = (kt - kt_begin) & 1;
    const char* Kt = smem + buf * TL;
    const char* Vt = smem + 2 * TL + buf * TL;
    if (kt + 1 < kt_end) {
      stage_tile_d<NW, D>(smem + (buf ^ 1) * TL, rowp(kt + 1, 0));
      stage_tile_d<NW, D>(smem + 2 * TL + (buf ^ 1) * TL, rowp(kt + 1, 1));
    }
    const int k0 = kt * BN;
    bool skip = !wave_active || k0 > w_qpos_hi;
    if (p.window > 0 && k0 + BN - 1 <= w_qpos_lo - p.window) skip = true;
    if (!skip) {
      f32x16 s[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        s[t] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) s[t] = mfma(rows_d(Kt, 32 * t, ks), qf[ks], s[t]);
      }
      float tmax = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int kp = k0 + 32 * t + acc_row(r, h);
          float x = s[t][r] * c;
          if (kp > qpos || !row_ok || (p.window > 0 && kp <= qpos - p.window)) x = -INFINITY;
          s[t][r] = x;
          tmax = fmaxf(tmax, x);
        }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
      const float mnew = fmaxf(m, tmax);
      const float muse = (mnew == -INFINITY) ? 0.f : mnew;
      const float alpha = fast_exp2(m - muse);
      float rs = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = fast_exp2(s[t][r] - muse);
          s[t][r] = e;
          rs += e;
        }
      rs += __shfl_xor(rs, 32, 64);
      l = l * alpha + rs;
      m = mnew;
      if (__any(alpha != 1.f)) {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
      }
      const bf16x8 pb[4] = {acc_to_b<0>(s[0]), acc_to_b<1>(s[0]), acc_to_b<0>(s[1]), acc_to_b<1>(s[1])};
#pragma unroll
      for (int dt = 0; dt < DT; ++dt)
#pragma unroll
        for (int st = 0; st < 4; ++st) o[dt] = mfma(tr_d(Vt, st, dt), pb[st], o[dt]);
    }
    __syncthreads();
  }
  if (row_ok) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16* op = p.o + ((int64_t)(q_start + tok) * p.hq + head) * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) store_row_block<D>(op, o[dt], dt, h, inv);
  }
}

// ------------------------------------------------------------------------------------------
// decode-only batches: split-K ("flash decoding") over the paged cache
// ------------------------------------------------------------------------------------------
// One new token per sequence: the atom kernel above would run one 4-wave workgroup per (sequence, kv head) --
// 8 workgroups for a single Llama-3-8B sequence, each walking the whole context on a mostly empty 128-row MFMA tile
// (35 us per layer at 540 keys, profiles/r3). Decode is a K/V stream, so this kernel is built like decode_attn.hip:
// grid (splits, Hkv, n_seqs), a workgroup serves all G query heads of its kv head from ONE read of its key range,
// 16-B loads with LPK = D / 8 lanes per key, online softmax in registers, lane groups and waves merged by
// max / rescale, splits merged by a combine kernel through fp32 partials. The key range comes from the device-side
// sequence metadata (seen + 1 keys), so one launch shape serves every step of a HIP-graph decode.
constexpr int kDecGMax = 8;

struct PagedDecodeParams {
  const bf16* q;  // [T, Hq, D] rows with token stride sq
  int64_t sq;
  const bf16* cache;  // [num_blocks, block_size, 2, Hkv, D]
  bf16* o;            // [T, Hq, D]
  float* part_o;      // [n_seqs, Hq, splits, D]
  float* part_ml;     // [n_seqs, Hq, splits, 2]
  const int* seq_meta;  // [n_seqs][3] = {q_start, n_new (1), seen}
  const int* block_tables;
  int max_blocks, block_size, hq, hkv, splits;
  float scale;
  int window;
  // splits > 1: one int per (sequence, kv head), zero between launches. Non-null: the last workgroup of a
  // (sequence, kv head) to finish merges the splits itself (no combine launch) and resets its counter to 0, so a
  // HIP-graph replay finds it zeroed again.
  int* counters;
};

template <int D>
__device__ __forceinline__ void decode_merge_splits(const PagedDecodeParams& p, int b, int h, int d, int q_start) {
  const float* pm = p.part_ml + ((int64_t)b * p.hq + h) * p.splits * 2;
  float mm = -INFINITY;
  for (int s = 0; s < p.splits; ++s) mm = fmaxf(mm, pm[2 * s]);
  float ll = 0.f, oo = 0.f;
  for (int s = 0; s < p.splits; ++s) {
    const float a = mm == -INFINITY ? 0.f : __expf(pm[2 * s] - mm);
    ll += pm[2 * s + 1] * a;
    oo += p.part_o[(((int64_t)b * p.hq + h) * p.splits + s) * D + d] * a;
  }
  p.o[((int64_t)q_start * p.hq + h) * D + d] = (bf16)(ll > 0.f ? oo / ll : 0.f);
}

template <int D>
__global__ __launch_bounds__(256) void paged_decode_kernel(PagedDecodeParams p) {
  constexpr int LPK = D / 8, KPW = 64 / LPK;
  __shared__ float red[4][kDecGMax][2 + D];
  const int split = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int G = p.hq / p.hkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int kl = lane / LPK, c = lane % LPK;
  const int q_start = p.seq_meta[3 * b], ctx = p.seq_meta[3 * b + 2] + 1;
  const int jb = p.window > 0 ? max(0, ctx - p.window) : 0;
  const int kps = (ctx + p.splits - 1) / p.splits;
  const int j0 = split * kps, j1 = min(ctx, j0 + kps);
  const int* table = p.block_tables + (int64_t)b * p.max_blocks;
  const int64_t kv_row = 2LL * p.hkv * D;

  float qv[kDecGMax][8];
#pragma unroll
  for (int g = 0; g < kDecGMax; ++g) {
    if (g < G) {
      Vec8<bf16>::load(p.q + (int64_t)q_start * p.sq + (int64_t)(hk * G + g) * D + c * 8, qv[g]);
#pragma unroll
      for (int e = 0; e < 8; ++e) qv[g][e] *= p.scale;
    }
  }
  float m[kDecGMax], l[kDecGMax], acc[kDecGMax][8];
#pragma unroll
  for (int g = 0; g < kDecGMax; ++g) {
    m[g] = -INFINITY;
    l[g] = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) acc[g][e] = 0.f;
  }
  for (int j = j0 + w * KPW + kl; j - kl < j1; j += 4 * KPW) {
    const bool ok = j < j1 && j >= jb;
    float kv[8] = {}, vv[8] = {};
    if (ok) {
      const int blk = table[j / p.block_size];
      const bf16* kb = p.cache + ((int64_t)blk * p.block_size + j % p.block_size) * kv_row + (int64_t)hk * D + c * 8;
      Vec8<bf16>::load(kb, kv);
      Vec8<bf16>::load(kb + (int64_t)p.hkv * D, vv);
    }
#pragma unroll
    for (int g = 0; g < kDecGMax; ++g) {
      if (g >= G) break;
      float sc = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) sc += qv[g][e] * kv[e];
#pragma unroll
      for (int off = LPK / 2; off >= 1; off >>= 1) sc += __shfl_xor(sc, off, 64);
      sc = ok ? sc : -INFINITY;
      const float mn = fmaxf(m[g], sc);
      const bool none = mn == -INFINITY;
      const float a = none ? 1.f : __expf(m[g] - mn), e_s = none ? 0.f : __expf(sc - mn);
      l[g] = l[g] * a + e_s;
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[g][e] = acc[g][e] * a + e_s * vv[e];
      m[g] = mn;
    }
  }
#pragma unroll
  for (int g = 0; g < kDecGMax; ++g) {
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
  if (kl == 0) {
#pragma unroll
    for (int g = 0; g < kDecGMax; ++g) {
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
      Vec8<bf16>::store(p.o + ((int64_t)q_start * p.hq + h) * D + cc * 8, oo);
    } else {
      float* po = p.part_o + (((int64_t)b * p.hq + h) * p.splits + split) * D + cc * 8;
#pragma unroll
      for (int e = 0; e < 8; ++e) po[e] = oo[e];
      if (cc == 0) {
        float* pm = p.part_ml + (((int64_t)b * p.hq + h) * p.splits + split) * 2;
        pm[0] = mm;
        pm[1] = ll;
      }
    }
  }
  if (p.splits > 1 && p.counters != nullptr) {
    // release this split's partials (device scope: the splits run on every XCD), count it in; the last one in
    // acquires all of them and merges
    __shared__ int s_last;
    __threadfence();
    __syncthreads();
    if (threadIdx.x == 0) s_last = atomicAdd(p.counters + b * p.hkv + hk, 1) == p.splits - 1;
    __syncthreads();
    if (!s_last) return;
    __threadfence();
    for (int t = threadIdx.x; t < G * D; t += 256) decode_merge_splits<D>(p, b, hk * G + t / D, t % D, q_start);
    if (threadIdx.x == 0) p.counters[b * p.hkv + hk] = 0;
  }
}

// One workgroup of D threads per (sequence, q head): the split maxima / sums are loaded once, one per thread, into LDS
// (one memory round trip instead of a dependent walk over the splits), then every thread merges its output column
// over the splits from partial-o values it requested before the barrier (splits <= 64 <= D).
template <int D>
__global__ __launch_bounds__(D) void paged_decode_combine_kernel(PagedDecodeParams p) {
  __shared__ float s_m[64], s_l[64];
  const int bh = blockIdx.x, b = bh / p.hq, h = bh % p.hq;
  const int d = threadIdx.x;
  // every load is issued before the barrier: the partial-o column (its addresses need no split stat) and the output
  // row overlap the stats' round trip instead of following it
  const float* po = p.part_o + (int64_t)bh * p.splits * D + d;
  float pov[64];
#pragma unroll
  for (int s = 0; s < 64; ++s) pov[s] = s < p.splits ? po[(int64_t)s * D] : 0.f;
  const int row = p.seq_meta[3 * b];
  const float* pm = p.part_ml + (int64_t)bh * p.splits * 2;
  if (d < p.splits) {
    s_m[d] = pm[2 * d];
    s_l[d] = pm[2 * d + 1];
  }
  __syncthreads();
  float mm = -INFINITY;
  for (int s = 0; s < p.splits; ++s) mm = fmaxf(mm, s_m[s]);
  float ll = 0.f, oo = 0.f;
#pragma unroll
  for (int s = 0; s < 64; ++s) {
    if (s < p.splits) {
      const float a = mm == -INFINITY ? 0.f : __expf(s_m[s] - mm);
      ll += s_l[s] * a;
      oo += pov[s] * a;
    }
  }
  p.o[((int64_t)row * p.hq + h) * D + d] = (bf16)(ll > 0.f ? oo / ll : 0.f);
}

}  // namespace

#define HDS_PAGED_DIMS(X) X(32) X(48) X(64) X(80) X(96) X(112) X(128) X(160) X(192) X(256)

// rot_dim: rotary prefix (0 = the whole head); cos/sin tables are [pos][rot_dim / 2]
HDS_EXPORT int hds_kv_rope_scatter(int dtype, void* qkv, int64_t sq, void* cache, const int* tok_seq,
                                   const int* tok_pos, const int* block_tables, int max_blocks, const float* cos_t,
                                   const float* sin_t, int n_tok, int hq, int hkv, int head_dim, int rot_dim,
                                   int block_size, int rotate_q, int do_rope, hipStream_t st) {
  if (n_tok <= 0) return 0;
  const int rot = (rot_dim <= 0 || rot_dim > head_dim) ? head_dim : rot_dim;
  if (head_dim % 4 || rot % 8 || (head_dim - rot) % 4) return hipErrorInvalidValue;
  const int64_t work = (int64_t)n_tok * (hq + 2 * hkv) * (rot / 8 + (head_dim - rot) / 4);
  dim3 grid(stream_grid(work, 256, 4096)), block(256);
  if (dtype == kBF16)
    hipLaunchKernelGGL(kv_rope_scatter_kernel<bf16>, grid, block, 0, st, (bf16*)qkv, sq, (bf16*)cache, tok_seq, tok_pos,
                       block_tables, max_blocks, cos_t, sin_t, n_tok, hq, hkv, head_dim, rot, block_size, rotate_q,
                       do_rope);
  else if (dtype == kF16)
    hipLaunchKernelGGL(kv_rope_scatter_kernel<_Float16>, grid, block, 0, st, (_Float16*)qkv, sq, (_Float16*)cache,
                       tok_seq, tok_pos, block_tables, max_blocks, cos_t, sin_t, n_tok, hq, hkv, head_dim, rot,
                       block_size, rotate_q, do_rope);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}

// atoms: device int32 [n_atoms][3]; seq_meta: device int32 [n_seqs][3]
HDS_EXPORT int hds_paged_attn(const void* q, int64_t sq, const void* cache, void* o, const int* atoms, int n_atoms,
                              const int* seq_meta, const int* block_tables, int max_blocks, int block_size, int hq,
                              int hkv, int head_dim, float scale, int window, hipStream_t st) {
  if (hq % hkv) return hipErrorInvalidValue;
  if (n_atoms <= 0) return 0;
  PagedParams p{(const bf16*)q, sq, (const bf16*)cache, (bf16*)o, atoms, seq_meta, block_tables, max_blocks,
                block_size, hq, hkv, scale, window};
#define HDS_CASE(d)                                                                          \
  if (head_dim == d) {                                                                       \
    hipLaunchKernelGGL((paged_attn_kernel<d, 4>), dim3(n_atoms), dim3(256), 0, st, p);       \
    return hipGetLastError();                                                                \
  }
  HDS_PAGED_DIMS(HDS_CASE)
#undef HDS_CASE
  return hipErrorInvalidValue;
}

HDS_EXPORT int hds_paged_rows_per_atom() { return 128; }

// decode-only batches (every sequence has exactly one new token)
HDS_EXPORT int hds_paged_decode_supported(int head_dim, int G) {
  return (head_dim == 64 || head_dim == 128 || head_dim == 256) && G >= 1 && G <= kDecGMax;
}

// key splits for n_seqs sequences of at most max_ctx keys: >= 2 workgroups per CU overall, >= 32 keys per split
HDS_EXPORT int hds_paged_decode_splits(int n_seqs, int hkv, int max_ctx) {
  const int groups = n_seqs * hkv;
  int splits = (512 + groups - 1) / groups;
  const int by_len = (max_ctx + 31) / 32;
  splits = splits < by_len ? splits : by_len;
  return splits < 1 ? 1 : (splits > 64 ? 64 : splits);
}

// counters: null -> the splits are merged by a second (combine) launch; else n_seqs * hkv zeroed ints and the last
// workgroup of each (sequence, kv head) merges them in the same launch (see paged_decode_kernel)
HDS_EXPORT int hds_paged_decode(const void* q, int64_t sq, const void* cache, void* o, float* part_o, float* part_ml,
                                const int* seq_meta, const int* block_tables, int max_blocks, int block_size,
                                int n_seqs, int hq, int hkv, int head_dim, int splits, float scale, int window,
                                int* counters, hipStream_t st) {
  if (n_seqs <= 0) return 0;
  if (hq % hkv || !hds_paged_decode_supported(head_dim, hq / hkv) || splits < 1 || splits > 64 ||
      (splits > 1 && (!part_o || !part_ml)))  // <= 64: the combine kernel stages the split stats in LDS
    return hipErrorInvalidValue;
  PagedDecodeParams p{(const bf16*)q, sq, (const bf16*)cache, (bf16*)o, part_o, part_ml, seq_meta, block_tables,
                      max_blocks, block_size, hq, hkv, splits, scale, window, counters};
  const dim3 grid(splits, hkv, n_seqs);
  switch (head_dim) {
#define HDS_DEC(d)                                                                                            \
  case d:                                                                                                     \
    hipLaunchKernelGGL(paged_decode_kernel<d>, grid, dim3(256), 0, st, p);                                    \
    if (splits > 1 && counters == nullptr)                                                                    \
      hipLaunchKernelGGL(paged_decode_combine_kernel<d>, dim3(n_seqs * hq), dim3(d), 0, st, p);               \
    break;
    HDS_DEC(64)
    HDS_DEC(128)
    HDS_DEC(256)
#undef HDS_DEC
  }
  return hipGetLastError();
}
