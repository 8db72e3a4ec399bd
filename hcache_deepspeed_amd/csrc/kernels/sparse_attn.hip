// Block-sparse FlashAttention forward + backward for gfx950 (64x64 layout blocks, head_dim 128, bf16 I/O).
//
// Capability parity: replaces the reference's Triton block-sparse SDD/DSD matmuls + block-sparse softmax
// (deepspeed/ops/sparse_attention/matmul.py, softmax.py). Instead of materialising the
// sparse score matrix in a compressed [nnz, block, block] format, the three passes are fused flash-style:
// each workgroup owns one 64-row query block (fwd, dQ) or one 64-key block (dK/dV) and walks ONLY the
// non-zero blocks of its layout row (CSR) or column (CSC); scores never leave registers.
//
// Structure (2 waves = 128 threads per workgroup, v_mfma_f32_32x32x16_bf16, layout block = 64 = one LDS tile):
//   fwd  : wave = 32 query rows; S^T = K.Q^T (query on the lane, lane-local online softmax), O^T += V^T.P^T;
//          the K/V tiles of the next non-zero block are LDS-DMA'd while the current block computes.
//   dq   : same walk; dS^T = P^T o (dP^T - delta), dQ += dS.K.
//   dkdv : wave = 32 keys (key on the lane); walks the CSC list of every q-head of the GQA group;
//          dK / dV stay in accumulators, no cross-workgroup reduction.
// The same MFMA/LDS building blocks (XOR-swizzled tiles, transposed reads) as flash_attn.hip (attn_common.h).
#include "attn_common.h"

using namespace hds;
using namespace hds::attn;

namespace {

constexpr int D = 128;
constexpr int BN = 64;  // layout block = query rows per workgroup = keys per tile
constexpr int NW = 2;
constexpr float kLog2e = 1.4426950408889634f;

struct SpParams {
  const bf16* q;
  const bf16* k;
  const bf16* v;
  bf16* o;
  float* lse;
  const bf16* dout;
  bf16* dq;
  bf16* dk;
  bf16* dv;
  float* delta;
  int64_t sq, sk, sv, so, sdo, sdq, sdk, sdv;
  const int* row_ptr;  // [Hl][nb + 1]
  const int* col_idx;  // [nnz] sorted within a row
  const int* col_ptr;  // [Hl][nb + 1]
  const int* row_idx;  // [nnz] sorted within a column
  int layout_heads;    // 1 (shared layout) or hq
  int nb;              // blocks per sequence
  int seq_len;
  int batch, hq, hkv;
  float scale;
  int causal;
};

__device__ __forceinline__ int layout_head(const SpParams& p, int hq) { return p.layout_heads == 1 ? 0 : hq; }

// ------------------------------------------------------------------------------------------------
// forward
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64 * NW) void bs_fwd_kernel(SpParams p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * 16384];  // K[2], V[2]
  const int qb = blockIdx.x, hq = blockIdx.y, b = blockIdx.z;
  const int start = b * p.seq_len;
  const int hk = hq / (p.hq / p.hkv);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int q0 = qb * BN;
  const int myq = q0 + 32 * w + (lane & 31);
  const float c = p.scale * kLog2e;
  const int* rp = p.row_ptr + (int64_t)layout_head(p, hq) * (p.nb + 1);
  const int e0 = rp[qb];
  int e1 = rp[qb + 1];
  if (p.causal) {  // rows are sorted: drop blocks strictly above the diagonal
    while (e1 > e0 && p.col_idx[e1 - 1] > qb) --e1;
  }

  bf16x8 qf[8];
  {
    const bf16* qp = p.q + (int64_t)(start + myq) * p.sq + (int64_t)hq * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
  }
  auto kptr = [&](int kt) {
    return [=](int row) { return p.k + (int64_t)(start + kt * BN + row) * p.sk + (int64_t)hk * D; };
  };
  auto vptr = [&](int kt) {
    return [=](int row) { return p.v + (int64_t)(start + kt * BN + row) * p.sv + (int64_t)hk * D; };
  };

  f32x16 o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = f32x16{};
  float m = -INFINITY, l = 0.f;

  if (e1 > e0) {
    const int kt = p.col_idx[e0];
    stage_tile64<NW>(smem + 0, kptr(kt));
    stage_tile64<NW>(smem + 2 * 16384, vptr(kt));
  }
  __syncthreads();
  for (int e = e0; e < e1; ++e) {
    const int buf = (e - e0) & 1;
    const char* Kt = smem + buf * 16384;
    const char* Vt = smem + 2 * 16384 + buf * 16384;
    const int kt = p.col_idx[e];
    if (e + 1 < e1) {
      const int kn = p.col_idx[e + 1];
      stage_tile64<NW>(smem + (buf ^ 1) * 16384, kptr(kn));
      stage_tile64<NW>(smem + 2 * 16384 + (buf ^ 1) * 16384, vptr(kn));
    }
    const int k0 = kt * BN;
    f32x16 s[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      s[t] = f32x16{};
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) s[t] = mfma(read_rows(Kt, 32 * t, ks), qf[ks], s[t]);
    }
    const bool diag = p.causal && kt == qb;
    float tmax = -INFINITY;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float x = s[t][r] * c;
        if (diag && k0 + 32 * t + acc_row(r, h) > myq) x = -INFINITY;
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
        const float ex = fast_exp2(s[t][r] - muse);
        s[t][r] = ex;
        rs += ex;
      }
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    m = mnew;
#pragma unroll
    for (int dt = 0; dt < 4; ++dt) o[dt] *= alpha;
    bf16x8 pb[4] = {acc_to_b<0>(s[0]), acc_to_b<1>(s[0]), acc_to_b<0>(s[1]), acc_to_b<1>(s[1])};
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int st = 0; st < 4; ++st) o[dt] = mfma(read_tr(Vt, st, dt), pb[st], o[dt]);
    __syncthreads();
  }

  const float inv = l > 0.f ? 1.f / l : 0.f;
  bf16* op = p.o + (int64_t)(start + myq) * p.so + (int64_t)hq * D;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 v4;
#pragma unroll
      for (int j = 0; j < 4; ++j) v4[j] = (bf16)(o[dt][4 * g + j] * inv);
      *reinterpret_cast<bf16x4*>(op + 32 * dt + 8 * g + 4 * h) = v4;
    }
  if (h == 0) {
    // rows without any key keep lse = +inf so the backward's exp2(s - lse) is exactly 0
    const float lse = (l > 0.f) ? (m + __log2f(l)) / kLog2e : INFINITY;
    p.lse[(int64_t)hq * p.batch * p.seq_len + start + myq] = lse;
  }
}

// delta[hq][t] = sum_d dO * O
__global__ __launch_bounds__(256) void bs_delta_kernel(SpParams p) {
  const int64_t total = (int64_t)p.batch * p.seq_len;
  const int64_t rows = total * p.hq;
  const int64_t row = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int sub = threadIdx.x & 15;
  float acc = 0.f;
  int64_t t = 0;
  int hq = 0;
  if (row < rows) {
    t = row / p.hq;
    hq = (int)(row - t * p.hq);
    float a[8], bb[8];
    Vec8<bf16>::load(p.o + t * p.so + (int64_t)hq * D + sub * 8, a);
    Vec8<bf16>::load(p.dout + t * p.sdo + (int64_t)hq * D + sub * 8, bb);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += a[j] * bb[j];
  }
#pragma unroll
  for (int off = 8; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 16);
  if (row < rows && sub == 0) p.delta[(int64_t)hq * total + t] = acc;
}

// ------------------------------------------------------------------------------------------------
// backward dQ (CSR walk)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64 * NW) void bs_dq_kernel(SpParams p) {
  __shared__ __attribute__((aligned(16))) char smem[4 * 16384];
  const int qb = blockIdx.x, hq = blockIdx.y, b = blockIdx.z;
  const int start = b * p.seq_len;
  const int64_t total = (int64_t)p.batch * p.seq_len;
  const int hk = hq / (p.hq / p.hkv);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int myq = qb * BN + 32 * w + (lane & 31);
  const float c = p.scale * kLog2e;
  const int* rp = p.row_ptr + (int64_t)layout_head(p, hq) * (p.nb + 1);
  const int e0 = rp[qb];
  int e1 = rp[qb + 1];
  if (p.causal) {
    while (e1 > e0 && p.col_idx[e1 - 1] > qb) --e1;
  }
  bf16x8 qf[8], df[8];
  {
    const bf16* qp = p.q + (int64_t)(start + myq) * p.sq + (int64_t)hq * D + 8 * h;
    const bf16* dp = p.dout + (int64_t)(start + myq) * p.sdo + (int64_t)hq * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
      df[ks] = *reinterpret_cast<const bf16x8*>(dp + 16 * ks);
    }
  }
  const float lse2 = p.lse[(int64_t)hq * total + start + myq] * kLog2e;
  const float dlt = p.delta[(int64_t)hq * total + start + myq];
  auto kptr = [&](int kt) {
    return [=](int row) { return p.k + (int64_t)(start + kt * BN + row) * p.sk + (int64_t)hk * D; };
  };
  auto vptr = [&](int kt) {
    return [=](int row) { return p.v + (int64_t)(start + kt * BN + row) * p.sv + (int64_t)hk * D; };
  };
  f32x16 dq[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dq[i] = f32x16{};
  if (e1 > e0) {
    const int kt = p.col_idx[e0];
    stage_tile64<NW>(smem + 0, kptr(kt));
    stage_tile64<NW>(smem + 2 * 16384, vptr(kt));
  }
  __syncthreads();
  for (int e = e0; e < e1; ++e) {
    const int buf = (e - e0) & 1;
    const char* Kt = smem + buf * 16384;
    const char* Vt = smem + 2 * 16384 + buf * 16384;
    const int kt = p.col_idx[e];
    if (e + 1 < e1) {
      const int kn = p.col_idx[e + 1];
      stage_tile64<NW>(smem + (buf ^ 1) * 16384, kptr(kn));
      stage_tile64<NW>(smem + 2 * 16384 + (buf ^ 1) * 16384, vptr(kn));
    }
    const int k0 = kt * BN;
    const bool diag = p.causal && kt == qb;
    f32x16 s[2], dp[2];
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      s[t] = f32x16{};
      dp[t] = f32x16{};
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) s[t] = mfma(read_rows(Kt, 32 * t, ks), qf[ks], s[t]);
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) dp[t] = mfma(read_rows(Vt, 32 * t, ks), df[ks], dp[t]);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float pr = fast_exp2(s[t][r] * c - lse2);
        if (diag && k0 + 32 * t + acc_row(r, h) > myq) pr = 0.f;
        s[t][r] = pr * (dp[t][r] - dlt);
      }
    const bf16x8 sb[4] = {acc_to_b<0>(s[0]), acc_to_b<1>(s[0]), acc_to_b<0>(s[1]), acc_to_b<1>(s[1])};
#pragma unroll
    for (int dt = 0; dt < 4; ++dt)
#pragma unroll
      for (int st = 0; st < 4; ++st) dq[dt] = mfma(read_tr(Kt, st, dt), sb[st], dq[dt]);
    __syncthreads();
  }
  bf16* qp = p.dq + (int64_t)(start + myq) * p.sdq + (int64_t)hq * D;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      bf16x4 v4;
#pragma unroll
      for (int j = 0; j < 4; ++j) v4[j] = (bf16)(dq[dt][4 * g + j] * p.scale);
      *reinterpret_cast<bf16x4*>(qp + 32 * dt + 8 * g + 4 * h) = v4;
    }
}

// ------------------------------------------------------------------------------------------------
// backward dK / dV (CSC walk over every q-head of the GQA group)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(64 * NW) void bs_dkdv_kernel(SpParams p) {
  // LDS: Q[2], dO[2] (16K each), lse[2][64], delta[2][64]
  __shared__ __attribute__((aligned(16))) char smem[4 * 16384 + 4 * 256];
  const int kb = blockIdx.x, hk = blockIdx.y, b = blockIdx.z;
  const int start = b * p.seq_len;
  const int64_t total_tok = (int64_t)p.batch * p.seq_len;
  const int G = p.hq / p.hkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int kw0 = kb * BN + 32 * w;
  const int myk = kw0 + (lane & 31);
  const float c = p.scale * kLog2e;

  bf16x8 kf[8], vf[8];
  {
    const bf16* kp = p.k + (int64_t)(start + myk) * p.sk + (int64_t)hk * D + 8 * h;
    const bf16* vp = p.v + (int64_t)(start + myk) * p.sv + (int64_t)hk * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      kf[ks] = *reinterpret_cast<const bf16x8*>(kp + 16 * ks);
      vf[ks] = *reinterpret_cast<const bf16x8*>(vp + 16 * ks);
    }
  }
  f32x16 dk[4], dv[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) dk[i] = dv[i] = f32x16{};

  // flattened walk over (g, e): e in the CSC column kb of q-head hk*G + g; causal drops q blocks < kb
  auto col_range = [&](int g, int& lo, int& hi) {
    const int* cp = p.col_ptr + (int64_t)layout_head(p, hk * G + g) * (p.nb + 1);
    lo = cp[kb];
    hi = cp[kb + 1];
    if (p.causal) {
      while (lo < hi && p.row_idx[lo] < kb) ++lo;
    }
  };
  auto advance = [&](int& g, int& e, int& hi) {  // move to the next valid (g, e); g == G when done
    ++e;
    while (g < G && e >= hi) {
      ++g;
      if (g < G) {
        int lo;
        col_range(g, lo, hi);
        e = lo;
      }
    }
  };
  auto stage = [&](int g, int e, int buf) {
    const int hq = hk * G + g;
    const int qt = p.row_idx[e];
    char* Qt = smem + buf * 16384;
    char* Ot = smem + 2 * 16384 + buf * 16384;
    float* Lt = reinterpret_cast<float*>(smem + 4 * 16384 + buf * 256);
    float* Dt = reinterpret_cast<float*>(smem + 4 * 16384 + 512 + buf * 256);
    stage_tile64<NW>(Qt, [=](int row) { return p.q + (int64_t)(start + qt * BN + row) * p.sq + (int64_t)hq * D; });
    stage_tile64<NW>(Ot,
                     [=](int row) { return p.dout + (int64_t)(start + qt * BN + row) * p.sdo + (int64_t)hq * D; });
    const float* src = (w == 0 ? p.lse : p.delta) + (int64_t)hq * total_tok + start + qt * BN + lane;
    __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(w == 0 ? Lt : Dt), 4, 0, 0);
  };

  int g = 0, e = 0, hi = 0;
  {
    int lo;
    col_range(0, lo, hi);
    e = lo - 1;
    advance(g, e, hi);
  }
  if (g < G) stage(g, e, 0);
  __syncthreads();
  int it = 0;
  while (g < G) {
    const int buf = it & 1;
    int g2 = g, e2 = e, hi2 = hi;
    advance(g2, e2, hi2);
    if (g2 < G) stage(g2, e2, buf ^ 1);
    const int qt = p.row_idx[e];
    const char* Qt = smem + buf * 16384;
    const char* Ot = smem + 2 * 16384 + buf * 16384;
    const float* Lt = reinterpret_cast<const float*>(smem + 4 * 16384 + buf * 256);
    const float* Dt = reinterpret_cast<const float*>(smem + 4 * 16384 + 512 + buf * 256);
    const int qbase = qt * BN;
    const bool diag = p.causal && qt == kb;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      f32x16 sacc = f32x16{}, dpacc = f32x16{};
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) sacc = mfma(read_rows(Qt, 32 * sub, ks), kf[ks], sacc);
#pragma unroll
      for (int ks = 0; ks < 8; ++ks) dpacc = mfma(read_rows(Ot, 32 * sub, ks), vf[ks], dpacc);
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int qr = 32 * sub + acc_row(r, h);
        float pr = fast_exp2(sacc[r] * c - Lt[qr] * kLog2e);
        if (diag && myk > qbase + qr) pr = 0.f;
        sacc[r] = pr;
        dpacc[r] = pr * (dpacc[r] - Dt[qr]);
      }
      const bf16x8 p0 = acc_to_b<0>(sacc), p1 = acc_to_b<1>(sacc);
      const bf16x8 s0 = acc_to_b<0>(dpacc), s1 = acc_to_b<1>(dpacc);
#pragma unroll
      for (int dt = 0; dt < 4; ++dt) {
        dv[dt] = mfma(read_tr(Ot, 2 * sub, dt), p0, dv[dt]);
        dv[dt] = mfma(read_tr(Ot, 2 * sub + 1, dt), p1, dv[dt]);
        dk[dt] = mfma(read_tr(Qt, 2 * sub, dt), s0, dk[dt]);
        dk[dt] = mfma(read_tr(Qt, 2 * sub + 1, dt), s1, dk[dt]);
      }
    }
    __syncthreads();
    g = g2;
    e = e2;
    hi = hi2;
    ++it;
  }
  bf16* kp = p.dk + (int64_t)(start + myk) * p.sdk + (int64_t)hk * D;
  bf16* vp = p.dv + (int64_t)(start + myk) * p.sdv + (int64_t)hk * D;
#pragma unroll
  for (int dt = 0; dt < 4; ++dt)
#pragma unroll
    for (int gg = 0; gg < 4; ++gg) {
      bf16x4 a4, b4;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        a4[j] = (bf16)(dk[dt][4 * gg + j] * p.scale);
        b4[j] = (bf16)(dv[dt][4 * gg + j]);
      }
      *reinterpret_cast<bf16x4*>(kp + 32 * dt + 8 * gg + 4 * h) = a4;
      *reinterpret_cast<bf16x4*>(vp + 32 * dt + 8 * gg + 4 * h) = b4;
    }
}

SpParams make_sp(const void* q, const void* k, const void* v, void* o, float* lse, const void* dout, void* dq, void* dk,
                 void* dv, float* delta, const int64_t* strides, const int* row_ptr, const int* col_idx,
                 const int* col_ptr, const int* row_idx, int layout_heads, int nb, int batch, int seq_len, int hq,
                 int hkv, float scale, int causal) {
  SpParams p;
  p.q = (const bf16*)q;
  p.k = (const bf16*)k;
  p.v = (const bf16*)v;
  p.o = (bf16*)o;
  p.lse = lse;
  p.dout = (const bf16*)dout;
  p.dq = (bf16*)dq;
  p.dk = (bf16*)dk;
  p.dv = (bf16*)dv;
  p.delta = delta;
  p.sq = strides[0];
  p.sk = strides[1];
  p.sv = strides[2];
  p.so = strides[3];
  p.sdo = strides[4];
  p.sdq = strides[5];
  p.sdk = strides[6];
  p.sdv = strides[7];
  p.row_ptr = row_ptr;
  p.col_idx = col_idx;
  p.col_ptr = col_ptr;
  p.row_idx = row_idx;
  p.layout_heads = layout_heads;
  p.nb = nb;
  p.seq_len = seq_len;
  p.batch = batch;
  p.hq = hq;
  p.hkv = hkv;
  p.scale = scale;
  p.causal = causal;
  return p;
}

bool sp_shapes_ok(int nb, int seq_len, int hq, int hkv, int head_dim, int layout_heads) {
  return head_dim == D && seq_len == nb * BN && hkv > 0 && hq % hkv == 0 && (layout_heads == 1 || layout_heads == hq);
}

}  // namespace

// q/k/v/o: [batch * seq_len, heads, 128] with token strides; lse: [hq][batch * seq_len] fp32.
// CSR (row_ptr/col_idx) of the 64-granular layout per layout head; seq_len must equal nb * 64.
HDS_EXPORT int hds_bsattn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, const int64_t* strides,
                              const int* row_ptr, const int* col_idx, int layout_heads, int nb, int batch, int seq_len,
                              int hq, int hkv, int head_dim, float scale, int causal, hipStream_t st) {
  if (!sp_shapes_ok(nb, seq_len, hq, hkv, head_dim, layout_heads)) return hipErrorInvalidValue;
  SpParams p = make_sp(q, k, v, o, lse, nullptr, nullptr, nullptr, nullptr, nullptr, strides, row_ptr, col_idx, nullptr,
                       nullptr, layout_heads, nb, batch, seq_len, hq, hkv, scale, causal);
  hipLaunchKernelGGL(bs_fwd_kernel, dim3(nb, hq, batch), dim3(64 * NW), 0, st, p);
  return hipGetLastError();
}

HDS_EXPORT int hds_bsattn_bwd(const void* q, const void* k, const void* v, const void* o, const float* lse,
                              const void* dout, void* dq, void* dk, void* dv, float* delta, const int64_t* strides,
                              const int* row_ptr, const int* col_idx, const int* col_ptr, const int* row_idx,
                              int layout_heads, int nb, int batch, int seq_len, int hq, int hkv, int head_dim,
                              float scale, int causal, hipStream_t st) {
  if (!sp_shapes_ok(nb, seq_len, hq, hkv, head_dim, layout_heads)) return hipErrorInvalidValue;
  SpParams p = make_sp(q, k, v, (void*)o, (float*)lse, dout, dq, dk, dv, delta, strides, row_ptr, col_idx, col_ptr,
                       row_idx, layout_heads, nb, batch, seq_len, hq, hkv, scale, causal);
  const int64_t rows = (int64_t)batch * seq_len * hq;
  hipLaunchKernelGGL(bs_delta_kernel, dim3((rows + 15) / 16), dim3(256), 0, st, p);
  hipLaunchKernelGGL(bs_dkdv_kernel, dim3(nb, hkv, batch), dim3(64 * NW), 0, st, p);
  hipLaunchKernelGGL(bs_dq_kernel, dim3(nb, hq, batch), dim3(64 * NW), 0, st, p);
  return hipGetLastError();
}
