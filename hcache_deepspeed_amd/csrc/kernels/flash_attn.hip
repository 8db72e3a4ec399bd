// FlashAttention forward + backward for gfx950 (causal / sliding-window / full, GQA, varlen),
// head_dim D in {32, 48, 64, 80, 96, 112, 128, 160, 192, 256} (any multiple of 16 up to 256 that is instantiated
// below), bf16 in/out, fp32 softmax statistics (LSE) exposed for FPDT / ring merges.
//
// Head-dim generality: tiles are stored as 128-column LDS sub-tiles (256-B rows, the XOR layout of
// attn_common.h); a D-wide tile is ceil(D/128) of them and only the first D/8 16-byte chunks of each row are
// staged. Q.K^T / dO.V^T contract over exactly D/16 k-steps; the P.V / dS.Q / dS.K products produce
// ceil(D/32) 32-column blocks whose columns >= D are never stored (they only see unstaged LDS columns, which
// cannot leak into valid columns: each MFMA output row depends on one A-operand row).
//
// Capability parity: replaces the reference's prebuilt NVIDIA-only `libblockedflash`
// (deepspeed/inference/v2/kernels/ragged_ops/blocked_flash), the `flash_attn`
// python dependency of sequence/fpdt_layer.py (§2.13) and the CUTLASS memory-efficient
// attention of csrc/deepspeed4science (K24) for the training path.
//
// Structure (all three kernels: 256 threads = 4 waves, v_mfma_f32_32x32x16_bf16):
//   fwd   : workgroup = 128 query rows of one (batch, q-head); wave = 32 rows; K/V tiles of 64
//           keys via LDS-DMA into a 2-deep LDS ring; S^T = K.Q^T puts the query on the lane so the
//           online softmax is lane-local; O^T += V^T.P^T reuses the S accumulators as the B
//           operand and reads V^T with ds_read_b64_tr_b16.  Heaviest causal blocks launch first.
//   dkdv  : workgroup = 128 keys of one (batch, kv-head); wave = 32 keys (key on the lane);
//           sweeps the GQA group's q-heads x 64-query tiles; dK and dV stay in accumulators
//           for the whole sweep, so no cross-workgroup reduction exists for them.
//   dq    : workgroup = 128 query rows of one (batch, q-head); sweeps key tiles; dQ in
//           accumulators. Deterministic (no float atomics anywhere).
// P is recomputed from the forward LSE; delta = rowsum(dO * O) comes from a tiny pre-kernel.
#include <type_traits>
#include <utility>

#include "attn_common.h"
#include "flash_attn_shared.h"

using namespace hds;
using namespace hds::attn;

// variant 9 lives in its own translation unit (flash_attn_w64.hip: built with the VGPR-form MFMA selection)
int hds_attn_fwd_w64_launch(const void* params, size_t params_bytes, int batch, int max_len, int hq, int mode,
                            hipStream_t st);
// one-wave-per-SIMD dQ (flash_attn_bwd_w64.hip)
int hds_attn_bwd_dq_w64_launch(const void* params, size_t params_bytes, int batch, int max_len, int hq,
                               hipStream_t st);

namespace {

template <int D, int NW, int VAR>
__global__ __launch_bounds__(64 * NW) void attn_fwd_kernel(AttnParams p) {
  constexpr int BM = 32 * NW;
  constexpr int KS = Dim<D>::KS, DT = Dim<D>::DT, TL = Dim<D>::TILE;
  __shared__ __attribute__((aligned(16))) char smem[4 * TL];  // K[2], V[2]
  int blk, hq, b;
  lpt_ids(blk, hq, b);
  int start, len;
  seq_bounds(p, b, start, len);
  const int nqb = (len + BM - 1) / BM;
  const int qb = p.causal ? (gridDim.x - 1 - blk) : blk;  // heaviest causal blocks first
  if (qb >= nqb || len == 0) return;
  const int hk = hq / (p.hq / p.hkv);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int q0 = qb * BM;
  const int myq = q0 + 32 * w + (lane & 31);
  const float c = p.scale * kLog2e;
  int klo, khi;
  key_span(p, myq, len, klo, khi);

  // Q fragments (B operand of S^T = K.Q^T): Q[myq][16ks + 8h .. +7]
  bf16x8 qf[KS];
  {
    const int qr = myq < len ? myq : len - 1;
    const bf16* qp = p.q + (int64_t)(start + qr) * p.sq + (int64_t)hq * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
  }

  // key-tile range
  int kt_end = (len + BN - 1) / BN;
  if (p.causal) {
    const int last = q0 + BM - 1 < len - 1 ? q0 + BM - 1 : len - 1;
    kt_end = last / BN + 1;
  }
  int kt_begin = 0;
  if (p.window > 0) {
    const int first = q0 - p.window + 1;
    kt_begin = first > 0 ? first / BN : 0;
  }

  auto kptr = [&](int kt) {
    return [=](int row) {
      int r = kt * BN + row;
      r = r < len ? r : len - 1;
      return p.k + (int64_t)(start + r) * p.sk + (int64_t)hk * D;
    };
  };
  auto vptr = [&](int kt) {
    return [=](int row) {
      int r = kt * BN + row;
      r = r < len ? r : len - 1;
      return p.v + (int64_t)(start + r) * p.sv + (int64_t)hk * D;
    };
  };

  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = f32x16{};
  float m = -INFINITY, l = 0.f;

  const int wq_lo = q0 + 32 * w, wq_hi = q0 + 32 * w + 31;

  stage_tile_d<NW, D>(smem + 0, kptr(kt_begin));
  stage_tile_d<NW, D>(smem + 2 * TL, vptr(kt_begin));
  __syncthreads();
  if constexpr ((VAR & 1) != 0 && NW == 8) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  }

  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const int buf = (kt - kt_begin) & 1;
    char* Kt = smem + buf * TL;
    char* Vt = smem + 2 * TL + buf * TL;
    if (kt + 1 < kt_end) {
      stage_tile_d<NW, D>(smem + (buf ^ 1) * TL, kptr(kt + 1));
      stage_tile_d<NW, D>(smem + 2 * TL + (buf ^ 1) * TL, vptr(kt + 1));
    }
    const int k0 = kt * BN;
    // wave-uniform skip of fully masked tiles
    bool skip = (k0 >= len) || (wq_lo >= len);
    if (p.causal && k0 > wq_hi) skip = true;
    if (p.window > 0 && k0 + BN - 1 <= wq_lo - p.window) skip = true;
    if (!skip) {
      f32x16 s[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        s[t] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) s[t] = mfma(rows_d(Kt, 32 * t, ks), qf[ks], s[t]);
      }
      const bool need_mask = (k0 + BN > len) || (p.causal && k0 + BN - 1 > wq_lo) ||
                             (p.window > 0 && k0 <= wq_hi - p.window) || (wq_hi >= len);
      // the max runs on the raw scores and the scale is folded into the exponent's FMA (c > 0), which saves a
      // multiply per score: the softmax VALU, not the MFMA pipe, bounds this loop
      float tmax = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (need_mask) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (outside(k0 + 32 * t + acc_row(r, h), klo, khi)) s[t][r] = -INFINITY;
        }
#pragma unroll
        for (int r = 0; r < 16; r += 2) tmax = max3_raw(tmax, s[t][r], s[t][r + 1]);
      }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * c;
      float alpha = 1.f, muse;
      if constexpr ((VAR & 2) != 0) {
        if (!__all(tmax <= m + kDeferThr)) {  // some row outgrew the stale max: move every row's max now
          const float mnew = fmaxf(m, tmax);
          alpha = (m == -INFINITY) ? 0.f : fast_exp2(m - mnew);
          m = mnew;
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
        }
        muse = (m == -INFINITY) ? 0.f : m;
      } else {
        const float mnew = fmaxf(m, tmax);
        muse = (mnew == -INFINITY) ? 0.f : mnew;
        alpha = fast_exp2(m - muse);
        m = mnew;
        if (__any(alpha != 1.f)) {  // running max moved for some row of this wave: rescale O
#pragma unroll
          for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
        }
      }
      float rs = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = fast_exp2(__builtin_fmaf(s[t][r], c, -muse));
          s[t][r] = e;
          rs += e;
        }
      rs += __shfl_xor(rs, 32, 64);
      l = l * alpha + rs;
      bf16x8 pb[4] = {acc_to_b<0>(s[0]), acc_to_b<1>(s[0]), acc_to_b<0>(s[1]), acc_to_b<1>(s[1])};
      if constexpr ((VAR & 2) != 0) {
        // V^T fragments by asm transposed reads (no compiler vmcnt(0) on the next tile's DMA in flight),
        // one 32-column block ahead of its MFMAs
        bf16x8 vf[2][4];
#pragma unroll
        for (int st = 0; st < 4; ++st) vf[0][st] = tr_d_asm(Vt, st, 0);
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          if (dt + 1 < DT) {
#pragma unroll
            for (int st = 0; st < 4; ++st) vf[(dt + 1) & 1][st] = tr_d_asm(Vt, st, dt + 1);
            lds_wait_tie<8>(vf[dt & 1][0], vf[dt & 1][1], vf[dt & 1][2], vf[dt & 1][3]);
          } else {
            lds_wait_tie<0>(vf[dt & 1][0], vf[dt & 1][1], vf[dt & 1][2], vf[dt & 1][3]);
          }
#pragma unroll
          for (int st = 0; st < 4; ++st) o[dt] = mfma(vf[dt & 1][st], pb[st], o[dt]);
        }
      } else {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int st = 0; st < 4; ++st) o[dt] = mfma(tr_d(Vt, st, dt), pb[st], o[dt]);
      }
    }
    __syncthreads();
  }

  // epilogue: O[myq][d] = o^T / l ; lse
  if (myq < len) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16* op = p.o + (int64_t)(start + myq) * p.so + (int64_t)hq * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) store_row_block<D>(op, o[dt], dt, h, inv);
    if (h == 0 && p.lse) {
      const float lse = (l > 0.f) ? (m + __log2f(l)) / kLog2e : -INFINITY;
      p.lse[(int64_t)hq * p.total_tokens + start + myq] = lse;
    }
  }
}

// =====================================================================================
// forward, staggered wave groups (D <= 128, 8 waves)
// =====================================================================================
// Every key tile is two SECTIONS separated by a raw barrier: S (S^T = K.Q^T, online softmax, O rescale) and P
// (O^T += V^T.P^T). Waves 4-7 run one barrier behind waves 0-3, so on every SIMD one wave's P-section MFMAs run
// beside its partner's S-section MFMAs + softmax VALU instead of both waves doing the same phase at once
// (MI355X_MICROARCH "Two waves per SIMD" item 9). The K/V ring stays two tiles deep; waves 0-3 stage K and
// waves 4-7 stage V, each during its S section, for the tile after next -- a buffer is restaged only after the
// lagging group's last read of it -- and each group retires its own DMA (vmcnt(0)) before the barrier that closes
// its P section, one section before the leading group first reads the tile.
template <int D>
__global__ __launch_bounds__(512) void attn_fwd_stg_kernel(AttnParams p) {
  constexpr int NW = 8, BM = 32 * NW;
  constexpr int KS = Dim<D>::KS, DT = Dim<D>::DT, TL = Dim<D>::TILE;
  static_assert(D <= 128, "staggered forward: head_dim <= 128");
  __shared__ __attribute__((aligned(16))) char smem[4 * TL];  // K[2], V[2]
  int blk, hq, b;
  lpt_ids(blk, hq, b);
  int start, len;
  seq_bounds(p, b, start, len);
  const int nqb = (len + BM - 1) / BM;
  const int qb = p.causal ? (gridDim.x - 1 - blk) : blk;
  if (qb >= nqb || len == 0) return;
  const int hk = hq / (p.hq / p.hkv);
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int grp = w >> 2;  // 0: leading group (stages K), 1: lagging group (stages V)
  const int q0 = qb * BM;
  const int myq = q0 + 32 * w + (lane & 31);
  const float c = p.scale * kLog2e;
  int klo, khi;
  key_span(p, myq, len, klo, khi);

  bf16x8 qf[KS];
  {
    const int qr = myq < len ? myq : len - 1;
    const bf16* qp = p.q + (int64_t)(start + qr) * p.sq + (int64_t)hq * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
  }
  int kt_end = (len + BN - 1) / BN;
  if (p.causal) {
    const int last = q0 + BM - 1 < len - 1 ? q0 + BM - 1 : len - 1;
    kt_end = last / BN + 1;
  }
  int kt_begin = 0;
  if (p.window > 0) {
    const int first = q0 - p.window + 1;
    kt_begin = first > 0 ? first / BN : 0;
  }
  auto rowp = [&](const bf16* base, int64_t stride, int kt) {
    return [=](int row) {
      int r = kt * BN + row;
      r = r < len ? r : len - 1;
      return base + (int64_t)(start + r) * stride + (int64_t)hk * D;
    };
  };

  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = f32x16{};
  float m = -INFINITY, l = 0.f;
  const int wq_lo = q0 + 32 * w, wq_hi = q0 + 32 * w + 31;

  // prologue: the first tile's K and V by every wave
  stage_tile_d<NW, D>(smem + 0, rowp(p.k, p.sk, kt_begin));
  stage_tile_d<NW, D>(smem + 2 * TL, rowp(p.v, p.sv, kt_begin));
  __syncthreads();
  if (grp == 1) __builtin_amdgcn_s_barrier();  // waves 4-7 start one section behind

  bf16x8 pb[4];
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const int buf = (kt - kt_begin) & 1;
    const char* Kt = smem + buf * TL;
    const char* Vt = smem + 2 * TL + buf * TL;
    const int k0 = kt * BN;
    bool skip = (k0 >= len) || (wq_lo >= len);
    if (p.causal && k0 > wq_hi) skip = true;
    if (p.window > 0 && k0 + BN - 1 <= wq_lo - p.window) skip = true;
    // ---- S section: stage the next tile's K (group 0) / V (group 1), S = K.Q^T, softmax ----
    if (kt + 1 < kt_end) {
      if (grp == 0)
        stage_tile_dw<4, D>(smem + (buf ^ 1) * TL, rowp(p.k, p.sk, kt + 1), w & 3);
      else
        stage_tile_dw<4, D>(smem + 2 * TL + (buf ^ 1) * TL, rowp(p.v, p.sv, kt + 1), w & 3);
    }
    if (!skip) {
      f32x16 s[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        s[t] = f32x16{};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) s[t] = mfma(rows_d(Kt, 32 * t, ks), qf[ks], s[t]);
      }
      const bool need_mask = (k0 + BN > len) || (p.causal && k0 + BN - 1 > wq_lo) ||
                             (p.window > 0 && k0 <= wq_hi - p.window) || (wq_hi >= len);
      float tmax = -INFINITY;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        if (need_mask) {
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (outside(k0 + 32 * t + acc_row(r, h), klo, khi)) s[t][r] = -INFINITY;
        }
#pragma unroll
        for (int r = 0; r < 16; r += 2) tmax = max3_raw(tmax, s[t][r], s[t][r + 1]);
      }
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * c;
      float alpha = 1.f;
      if (!__all(tmax <= m + kDeferThr)) {  // deferred running max (guide T13)
        const float mnew = fmaxf(m, tmax);
        alpha = (m == -INFINITY) ? 0.f : fast_exp2(m - mnew);
        m = mnew;
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
      }
      const float muse = (m == -INFINITY) ? 0.f : m;
      float rs = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float e = fast_exp2(__builtin_fmaf(s[t][r], c, -muse));
          s[t][r] = e;
          rs += e;
        }
      rs += __shfl_xor(rs, 32, 64);
      l = l * alpha + rs;
      pb[0] = acc_to_b<0>(s[0]);
      pb[1] = acc_to_b<1>(s[0]);
      pb[2] = acc_to_b<0>(s[1]);
      pb[3] = acc_to_b<1>(s[1]);
    }
    __builtin_amdgcn_s_barrier();
    // ---- P section: O^T += V^T.P^T (V^T fragments one 32-column block ahead of the MFMAs) ----
    if (!skip) {
      bf16x8 vf[2][4];
#pragma unroll
      for (int st = 0; st < 4; ++st) vf[0][st] = read_tr_asm(Vt, st, 0);
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        if (dt + 1 < DT) {
#pragma unroll
          for (int st = 0; st < 4; ++st) vf[(dt + 1) & 1][st] = read_tr_asm(Vt, st, dt + 1);
          // block dt's 8 reads are done, block dt+1's may still fly
          lds_wait_tie<8>(vf[dt & 1][0], vf[dt & 1][1], vf[dt & 1][2], vf[dt & 1][3]);
        } else {
          lds_wait_tie<0>(vf[dt & 1][0], vf[dt & 1][1], vf[dt & 1][2], vf[dt & 1][3]);
        }
#pragma unroll
        for (int st = 0; st < 4; ++st) o[dt] = mfma(vf[dt & 1][st], pb[st], o[dt]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this wave's DMA of the next tile has landed
    __builtin_amdgcn_s_barrier();
  }
  if (grp == 0) __builtin_amdgcn_s_barrier();  // rejoin

  if (myq < len) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16* op = p.o + (int64_t)(start + myq) * p.so + (int64_t)hq * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) store_row_block<D>(op, o[dt], dt, h, inv);
    if (h == 0 && p.lse) {
      const float lse = (l > 0.f) ? (m + __log2f(l)) / kLog2e : -INFINITY;
      p.lse[(int64_t)hq * p.total_tokens + start + myq] = lse;
    }
  }
}

// =====================================================================================
// forward, software-pipelined softmax (D = 128, 8 waves, 256 queries per workgroup)
// =====================================================================================
// The plain loop is a dependency chain per wave -- S = K.Q^T (16 MFMAs), then the softmax on the VALU, then
// O += V^T.P (16 MFMAs) -- so a wave's MFMAs and its own softmax never overlap. Here iteration kt computes the NEXT
// tile's scores while this tile's softmax runs: block A issues S_{kt+1} = K_{kt+1}.Q^T with the max / rescale /
// exponentials of S_kt between its MFMAs (independent work, interleaved by sched_group_barrier: a 32x32x16 MFMA
// leaves ~24 of its 32 issue cycles to VALU); block B issues O += V_kt^T.P_kt with the other half of the
// exponentials and the row sums beside it. The K ring runs one tile further ahead than V: at the top of iteration kt
// the wave retires V_kt and K_{kt+1} (vmcnt(0)), the barrier frees V_{kt-1} / K_kt, and the DMA of V_{kt+1} /
// K_{kt+2} goes into those slots -- one barrier per tile.
// Fixed per-tile VALU is removed as well (PMC: ~8 VALU per MFMA, the SIMD's issue port being the limit): the loop is
// unrolled by two so every LDS slot offset is a compile-time ds_read immediate on 16 per-lane address registers
// computed once (no address VALU per read), and a full tile's LDS-DMA source is a uniform base plus a per-lane
// 32-bit offset computed once (clamped per-row addressing only on the last, partial tile). Every wave runs every tile
// of the workgroup's causal range (a fully masked tile contributes exp(-inf) = 0), so the loop body has no
// wave-level branches that would split the interleaved blocks.

// SKIPW (variant 7): a wave whose queries all lie below a causal key tile skips that tile's math -- and every later
// one, which is masked too -- keeping only the workgroup's DMA staging and barrier (waves 0-5 of the last 1-3 tiles).
// NW4 (variant 8): 4 waves / 128 queries per workgroup, two workgroups per CU (64 KiB of LDS each, one wave per SIMD
// each) -- their barriers are independent, so one workgroup's MFMA phase can run beside the other's wait.
template <int D, bool FASTDMA = true, bool SKIPW = false, int NW = 8>
__global__ __launch_bounds__(64 * NW) __attribute__((amdgpu_waves_per_eu(2))) void attn_fwd_sp_kernel(AttnParams p) {
  constexpr int BM = 32 * NW, PW = 16 / NW;  // PW: 1-KiB tile pieces each wave stages
  constexpr int KS = Dim<D>::KS, DT = Dim<D>::DT, TL = Dim<D>::TILE;
  static_assert(D == 128, "software-pipelined forward: head_dim 128");
  __shared__ __attribute__((aligned(16))) char smem[4 * TL];  // K[2], V[2]
  int blk, hq, b;
  lpt_ids(blk, hq, b);
  int start, len;
  seq_bounds(p, b, start, len);
  const int nqb = (len + BM - 1) / BM;
  const int qb = p.causal ? (gridDim.x - 1 - blk) : blk;
  if (qb >= nqb || len == 0) return;
  const int hk = hq / (p.hq / p.hkv);
  const int lane = threadIdx.x & 63, h = lane >> 5;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int q0 = qb * BM;
  const int myq = q0 + 32 * w + (lane & 31);
  const float c = p.scale * kLog2e;
  int klo, khi;
  key_span(p, myq, len, klo, khi);
  if (NW == 8 && w >= 4) __builtin_amdgcn_s_setprio(1);  // static priority for the second-dispatched half (T5)

  bf16x8 qf[KS];
  {
    const int qr = myq < len ? myq : len - 1;
    const bf16* qp = p.q + (int64_t)(start + qr) * p.sq + (int64_t)hq * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
  }
  int kt_end = (len + BN - 1) / BN;
  if (p.causal) {
    const int last = q0 + BM - 1 < len - 1 ? q0 + BM - 1 : len - 1;
    kt_end = last / BN + 1;
  }
  int kt_begin = 0;
  if (p.window > 0) {
    const int first = q0 - p.window + 1;
    kt_begin = first > 0 ? first / BN : 0;
  }
  auto rowp = [&](const bf16* base, int64_t stride, int kt) {
    return [=](int row) {
      int r = kt * BN + row;
      r = r < len ? r : len - 1;
      return base + (int64_t)(start + r) * stride + (int64_t)hk * D;
    };
  };
  // LDS-DMA of a full tile: uniform tile base + per-lane byte offset (row 4n + lane/16, swizzled 16-B chunk)
  int32_t dk[PW], dv[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int row = 4 * (w * PW + i) + (lane >> 4);
    const int ch = (lane & 15) ^ swz(row);
    dk[i] = (int32_t)(((int64_t)row * p.sk + 8 * ch) * 2);
    dv[i] = (int32_t)(((int64_t)row * p.sv + 8 * ch) * 2);
  }
  auto stage = [&](char* dst, const bf16* base, int64_t stride, const int32_t* off, int kt) {
    if (FASTDMA && kt * BN + BN <= len) {
      const char* tb = (const char*)(base + (int64_t)(start + kt * BN) * stride + (int64_t)hk * D);
#pragma unroll
      for (int i = 0; i < PW; ++i)
        __builtin_amdgcn_global_load_lds((gbl_void*)(tb + off[i]), (lds_void*)(dst + (w * PW + i) * 1024), 16, 0, 0);
    } else {
      stage_tile_d<NW, D>(dst, rowp(base, stride, kt));
    }
  };
  const int wq_lo = q0 + 32 * w, wq_hi = q0 + 32 * w + 31;
  const uint32_t sbase = (uint32_t)(uintptr_t)smem;
  uint32_t ak[KS], av0[DT], av1[DT];
  {
    const uint32_t P0 = rows_lane_off(0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) ak[ks] = sbase + (P0 ^ (32u * ks));  // + 8192: rows 32..63 (same swizzle)
    uint32_t y0, y1;
    tr_lane_offs(y0, y1);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      av0[dt] = sbase + (y0 ^ (64u * dt));
      av1[dt] = sbase + (y1 ^ (64u * dt));
    }
  }

  f32x16 o[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) o[i] = f32x16{};
  float m = -INFINITY, l = 0.f;

  // prologue: K_0, V_0, K_1 in flight; S_0 once K_0 has landed
  stage(smem + 0, p.k, p.sk, dk, kt_begin);
  stage(smem + 2 * TL, p.v, p.sv, dv, kt_begin);
  if (kt_begin + 1 < kt_end) {
    stage(smem + TL, p.k, p.sk, dk, kt_begin + 1);
    // this wave's PW K_0 DMAs (issued first) have landed; V_0 and K_1 (2 PW) may still be in flight
    if constexpr (NW == 8) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  } else {
    if constexpr (NW == 8) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  __syncthreads();
  f32x16 sc[2];
  {
    bf16x8 kr[2][KS];
    static_for<KS>([&](auto KSC) {
      constexpr int ks = decltype(KSC)::value;
      kr[0][ks] = lds_b128<0>(ak[ks]);
      kr[1][ks] = lds_b128<8192>(ak[ks]);
    });
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      lds_wait_tie<0>(kr[t][0], kr[t][1], kr[t][2], kr[t][3]);
      lds_wait_tie<0>(kr[t][4], kr[t][5], kr[t][6], kr[t][7]);
    }
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      sc[t] = f32x16{};
#pragma unroll
      for (int ks = 0; ks < KS; ++ks) sc[t] = mfma(kr[t][ks], qf[ks], sc[t]);
    }
  }

  const int skip_from = (SKIPW && p.causal && p.window <= 0) ? wq_hi / BN + 1 : 0x7fffffff;
  auto tile = [&](auto BUFC, int kt) {
    constexpr int buf = decltype(BUFC)::value;
    constexpr int KN = (buf ^ 1) * TL;          // K_{kt+1}
    constexpr int VT = 2 * TL + buf * TL;       // V_kt
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // V_kt and K_{kt+1} of this wave have landed
    __syncthreads();                                   // ... of every wave; V_{kt-1} and K_kt are free
    if (kt + 1 < kt_end) stage(smem + 2 * TL + (buf ^ 1) * TL, p.v, p.sv, dv, kt + 1);
    if (kt + 2 < kt_end) stage(smem + buf * TL, p.k, p.sk, dk, kt + 2);
    if (SKIPW && kt >= skip_from) return;  // wave-uniform

    const int k0 = kt * BN;
    const bool need_mask = (k0 + BN > len) || (p.causal && k0 + BN - 1 > wq_lo) ||
                           (p.window > 0 && k0 <= wq_hi - p.window) || (wq_hi >= len);
    if (need_mask) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (outside(k0 + 32 * t + acc_row(r, h), klo, khi)) sc[t][r] = -INFINITY;
    }
    float tm0 = -INFINITY, tm1 = -INFINITY;  // two independent max chains
#pragma unroll
    for (int r = 0; r < 16; r += 2) {
      tm0 = max3_raw(tm0, sc[0][r], sc[0][r + 1]);
      tm1 = max3_raw(tm1, sc[1][r], sc[1][r + 1]);
    }
    float tmax = fmaxf(tm0, tm1);
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * c;
    const bool move = !__all(tmax <= m + kDeferThr);  // deferred running max (guide T13)
    const float mnew = move ? fmaxf(m, tmax) : m;
    const float alpha = move ? ((m == -INFINITY) ? 0.f : fast_exp2(m - mnew)) : 1.f;
    m = mnew;
    const float muse = (m == -INFINITY) ? 0.f : m;
    if (move) {  // before the interleaved blocks: a branch after them would let the compiler sink the exponentials
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] *= alpha;
    }

    // ---- block A: S_{kt+1} = K_{kt+1}.Q^T (4 chunks of 4 k-steps, double-buffered) beside exp(S_kt[keys 0..31])
    f32x16 sn[2];
    bf16x8 kr[2][4];
    float rs0 = 0.f, rs1 = 0.f;
    static_for<4>([&](auto IC) {
      constexpr int i = decltype(IC)::value;
      kr[0][i] = lds_b128<KN>(ak[i]);
    });
    static_for<4>([&](auto JC) {
      constexpr int j = decltype(JC)::value;
      constexpr int t = j >> 1;
      if constexpr (j + 1 < 4) {
        static_for<4>([&](auto IC) {
          constexpr int i = decltype(IC)::value;
          kr[(j + 1) & 1][i] = lds_b128<KN + 8192 * ((j + 1) >> 1)>(ak[4 * ((j + 1) & 1) + i]);
        });
        lds_wait_tie<4>(kr[j & 1][0], kr[j & 1][1], kr[j & 1][2], kr[j & 1][3]);
      } else {
        lds_wait_tie<0>(kr[j & 1][0], kr[j & 1][1], kr[j & 1][2], kr[j & 1][3]);
      }
      if constexpr ((j & 1) == 0) sn[t] = f32x16{};
#pragma unroll
      for (int i = 0; i < 4; ++i) sn[t] = mfma(kr[j & 1][i], qf[4 * (j & 1) + i], sn[t]);
#pragma unroll
      for (int r = 4 * j; r < 4 * j + 4; ++r) {
        const float e = fast_exp2(__builtin_fmaf(sc[0][r], c, -muse));
        sc[0][r] = e;
        (r & 1 ? rs1 : rs0) += e;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
        __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // then fma + exp + add
      }
    });
    bf16x8 pb[4];
    pb[0] = acc_to_b<0>(sc[0]);
    pb[1] = acc_to_b<1>(sc[0]);

    // ---- block B: O += V_kt^T.P_kt, key sub-block st outer, with exp(S_kt[keys 32..63]) beside the first half ----
    bf16x8 vf[2][DT];
    static_for<DT>([&](auto DC) {
      constexpr int dt = decltype(DC)::value;
      vf[0][dt] = lds_tr8<VT>(av0[dt], av1[dt]);
    });
    static_for<4>([&](auto SC) {
      constexpr int st = decltype(SC)::value;
      if constexpr (st + 1 < 4) {
        static_for<DT>([&](auto DC) {
          constexpr int dt = decltype(DC)::value;
          vf[(st + 1) & 1][dt] = lds_tr8<VT + 4096 * (st + 1)>(av0[dt], av1[dt]);
        });
        lds_wait_tie<8>(vf[st & 1][0], vf[st & 1][1], vf[st & 1][2], vf[st & 1][3]);
      } else {
        lds_wait_tie<0>(vf[st & 1][0], vf[st & 1][1], vf[st & 1][2], vf[st & 1][3]);
      }
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) o[dt] = mfma(vf[st & 1][dt], pb[st], o[dt]);
      if constexpr (st < 2) {
#pragma unroll
        for (int r = 8 * st; r < 8 * st + 8; ++r) {
          const float e = fast_exp2(__builtin_fmaf(sc[1][r], c, -muse));
          sc[1][r] = e;
          (r & 1 ? rs1 : rs0) += e;
        }
        if constexpr (st == 1) {
          pb[2] = acc_to_b<0>(sc[1]);
          pb[3] = acc_to_b<1>(sc[1]);
        }
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);
        }
      }
    });
    float rs = rs0 + rs1;
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
    sc[0] = sn[0];
    sc[1] = sn[1];
  };
  int kt = kt_begin;
  for (; kt + 1 < kt_end; kt += 2) {
    tile(std::integral_constant<int, 0>{}, kt);
    tile(std::integral_constant<int, 1>{}, kt + 1);
  }
  if (kt < kt_end) tile(std::integral_constant<int, 0>{}, kt);

  if (myq < len) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16* op = p.o + (int64_t)(start + myq) * p.so + (int64_t)hq * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) store_row_block<D>(op, o[dt], dt, h, inv);
    if (h == 0 && p.lse) {
      const float lse = (l > 0.f) ? (m + __log2f(l)) / kLog2e : -INFINITY;
      p.lse[(int64_t)hq * p.total_tokens + start + myq] = lse;
    }
  }
}

// =====================================================================================
// backward pre-pass: delta[hq][t] = sum_d dO * O   (16 lanes per row, 4 rows per wave)
// =====================================================================================
template <int D>
__global__ __launch_bounds__(256) void attn_bwd_delta_kernel(AttnParams p) {
  const int64_t rows = (int64_t)p.total_tokens * p.hq;
  const int64_t row = (int64_t)blockIdx.x * 16 + (threadIdx.x >> 4);
  const int sub = threadIdx.x & 15;
  float acc = 0.f;
  int64_t t = 0;
  int hq = 0;
  if (row < rows) {
    t = row / p.hq;
    hq = (int)(row - t * p.hq);
#pragma unroll
    for (int c = sub; c < D / 8; c += 16) {
      float a[8], bb[8];
      Vec8<bf16>::load(p.o + t * p.so + (int64_t)hq * D + c * 8, a);
      Vec8<bf16>::load(p.dout + t * p.sdo + (int64_t)hq * D + c * 8, bb);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc += a[j] * bb[j];
    }
  }
#pragma unroll
  for (int off = 8; off >= 1; off >>= 1) acc += __shfl_xor(acc, off, 16);
  if (row < rows && sub == 0) {
    p.delta[(int64_t)hq * p.total_tokens + t] = acc;
    // the dK/dV loop's exponent is S * c - lse * log2(e): pre-scaled once per row here instead of once per
    // (row, key-block, GQA head) in the loop -- 16 fewer VALU per 32 MFMAs there
    if (p.lse2) p.lse2[(int64_t)hq * p.total_tokens + t] = p.lse[(int64_t)hq * p.total_tokens + t] * kLog2e;
  }
}

// =====================================================================================
// backward dK, dV
// =====================================================================================
// C0 / CN: this launch produces the 32-column blocks [C0, C0 + CN) of dK and dV. Head dims > 128 run two
// launches over the two column halves (S and dP are recomputed per half) so the accumulators fit the register
// file without scratch spills.
template <int D, int NW, int C0 = 0, int CN = Dim<D>::DT>
__global__ __launch_bounds__(64 * NW) void attn_bwd_dkdv_kernel(AttnParams p) {
  constexpr int BK = 32 * NW;
  constexpr int KS = Dim<D>::KS, TL = Dim<D>::TILE;
  // LDS: Q[2], dO[2] (TL bytes each), lse[2][64], delta[2][64]
  __shared__ __attribute__((aligned(16))) char smem[4 * TL + 4 * 256];
  const int b = blockIdx.z, hk = blockIdx.y;
  int start, len;
  seq_bounds(p, b, start, len);
  const int nkb = (len + BK - 1) / BK;
  const int kb = blockIdx.x;
  if (kb >= nkb || len == 0) return;
  const int G = p.hq / p.hkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int kw0 = kb * BK + 32 * w;      // this wave's first key
  const int myk = kw0 + (lane & 31);
  int qlo, qhi;
  query_span(p, myk, len, qlo, qhi);
  const float c = p.scale * kLog2e;

  // K and V fragments (B operands): K[myk][16ks + 8h ..]
  bf16x8 kf[KS], vf[KS];
  {
    const int kr = myk < len ? myk : len - 1;
    const bf16* kp = p.k + (int64_t)(start + kr) * p.sk + (int64_t)hk * D + 8 * h;
    const bf16* vp = p.v + (int64_t)(start + kr) * p.sv + (int64_t)hk * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      kf[ks] = *reinterpret_cast<const bf16x8*>(kp + 16 * ks);
      vf[ks] = *reinterpret_cast<const bf16x8*>(vp + 16 * ks);
    }
  }
  f32x16 dk[CN], dv[CN];
#pragma unroll
  for (int i = 0; i < CN; ++i) dk[i] = dv[i] = f32x16{};

  // query-tile range (same for every q-head of the group)
  int qt_begin = 0;
  if (p.causal) qt_begin = (kb * BK) / BN;
  int qt_end = (len + BN - 1) / BN;
  if (p.window > 0) {
    const int lastq = kb * BK + BK - 1 + p.window - 1;
    const int e = lastq / BN + 1;
    qt_end = e < qt_end ? e : qt_end;
  }
  const int nqt = qt_end - qt_begin;
  const int total = nqt * G;
  if (total <= 0) {
    // still write zeros below
  }

  auto stage = [&](int it, int buf) {
    const int g = it / nqt, qt = qt_begin + it % nqt;
    const int hq = hk * G + g;
    char* Qt = smem + buf * TL;
    char* Ot = smem + 2 * TL + buf * TL;
    float* Lt = reinterpret_cast<float*>(smem + 4 * TL + buf * 256);
    float* Dt = reinterpret_cast<float*>(smem + 4 * TL + 512 + buf * 256);
    stage_tile_d<NW, D>(Qt, [=](int row) {
      int r = qt * BN + row;
      r = r < len ? r : len - 1;
      return p.q + (int64_t)(start + r) * p.sq + (int64_t)hq * D;
    });
    stage_tile_d<NW, D>(Ot, [=](int row) {
      int r = qt * BN + row;
      r = r < len ? r : len - 1;
      return p.dout + (int64_t)(start + r) * p.sdo + (int64_t)hq * D;
    });
    if (w < 2) {
      int r = qt * BN + lane;
      r = r < len ? r : len - 1;
      const float* src = (w == 0 ? p.lse : p.delta) + (int64_t)hq * p.total_tokens + start + r;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(w == 0 ? Lt : Dt), 4, 0, 0);
    }
  };

  if (total > 0) {
    stage(0, 0);
    __syncthreads();
  }
  for (int it = 0; it < total; ++it) {
    const int buf = it & 1;
    if (it + 1 < total) stage(it + 1, buf ^ 1);
    const int qt = qt_begin + it % nqt;
    const char* Qt = smem + buf * TL;
    const char* Ot = smem + 2 * TL + buf * TL;
    const float* Lt = reinterpret_cast<const float*>(smem + 4 * TL + buf * 256);
    const float* Dt = reinterpret_cast<const float*>(smem + 4 * TL + 512 + buf * 256);
    const int qbase = qt * BN;
    // wave-uniform skip: all queries of the tile before this wave's keys (causal)
    bool skip = (kw0 >= len);
    if (p.causal && qbase + BN - 1 < kw0) skip = true;
    if (p.window > 0 && qbase > kw0 + 31 + p.window - 1) skip = true;
    if (!skip) {
#pragma unroll
      for (int sub = 0; sub < 2; ++sub) {
        // S = Q.K^T (key on lane): rows = queries 32*sub + acc_row
        f32x16 sacc = f32x16{}, dpacc = f32x16{};
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) sacc = mfma(rows_d(Qt, 32 * sub, ks), kf[ks], sacc);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) dpacc = mfma(rows_d(Ot, 32 * sub, ks), vf[ks], dpacc);
        // P and dS
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int qr = 32 * sub + acc_row(r, h);
          const int qi = qbase + qr;
          float pr = fast_exp2(sacc[r] * c - Lt[qr] * kLog2e);
          if (outside(qi, qlo, qhi)) pr = 0.f;
          sacc[r] = pr;
          dpacc[r] = pr * (dpacc[r] - Dt[qr]);
        }
        const bf16x8 p0 = acc_to_b<0>(sacc), p1 = acc_to_b<1>(sacc);
        const bf16x8 s0 = acc_to_b<0>(dpacc), s1 = acc_to_b<1>(dpacc);
#pragma unroll
        for (int i = 0; i < CN; ++i) {
          const int dt = C0 + i;
          dv[i] = mfma(tr_d(Ot, 2 * sub, dt), p0, dv[i]);
          dv[i] = mfma(tr_d(Ot, 2 * sub + 1, dt), p1, dv[i]);
          dk[i] = mfma(tr_d(Qt, 2 * sub, dt), s0, dk[i]);
          dk[i] = mfma(tr_d(Qt, 2 * sub + 1, dt), s1, dk[i]);
        }
      }
    }
    __syncthreads();
  }
  if (myk < len) {
    bf16* kp = p.dk + (int64_t)(start + myk) * p.sdk + (int64_t)hk * D;
    bf16* vp = p.dv + (int64_t)(start + myk) * p.sdv + (int64_t)hk * D;
#pragma unroll
    for (int i = 0; i < CN; ++i) {
      store_row_block<D>(kp, dk[i], C0 + i, h, p.scale);
      store_row_block<D>(vp, dv[i], C0 + i, h, 1.f);
    }
  }
}

// PIPE >= 2 (head_dim 128, 8 waves): a FULL 64-row tile's LDS-DMA from a wave-uniform tile base plus per-lane 32-bit
// byte offsets computed once per kernel (row 4n + lane/16 of piece n = 2w + i, swizzled 16-B chunk) -- the generic
// stage_tile_d recomputes a clamped 64-bit row address per lane and piece on every tile (~2 VALU per MFMA of the
// backward loops). Partial tiles (the sequence end) keep the clamped path.
__device__ __forceinline__ void dma_offs8(int64_t stride, int32_t (&off)[2]) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int row = 4 * (2 * w + i) + (lane >> 4);
    const int ch = (lane & 15) ^ swz(row);
    off[i] = (int32_t)(((int64_t)row * stride + 8 * ch) * 2);
  }
}
__device__ __forceinline__ void stage_full8(char* tile, const bf16* tile_base, const int32_t (&off)[2]) {
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 2; ++i)
    __builtin_amdgcn_global_load_lds((gbl_void*)((const char*)tile_base + off[i]), (lds_void*)(tile + (2 * w + i) * 1024),
                                     16, 0, 0);
}

// =====================================================================================
// backward dK/dV, 8 waves, K/V resident in LDS (2 waves per SIMD)
// =====================================================================================
// Workgroup = 128 keys of one (batch, kv-head). Wave w owns key group kg = w & 3 (32 keys, key on
// the lane) and query half qh = w >> 2 of every 64-row Q/dO tile, so the 8 waves split each tile's
// work instead of each holding private K/V fragments: K and V live in LDS (64 KiB) and are read as
// the B operand exactly like Q rows are read as the A operand. Per wave: dK/dV accumulators
// (128 regs) + one 32x32 S/dP pair, which fits 256 registers -> 2 waves per SIMD, so one wave's
// softmax/VALU section overlaps the other wave's MFMAs. The two query halves' partial dK/dV are
// summed through LDS once at the end.
// PIPE: LDS operand reads issued two MFMAs ahead of their use as inline asm with counted lgkmcnt waits (a ring of
// three fragments), instead of the compiler's load -> lgkmcnt(0) -> MFMA per product, which exposes the LDS latency
// of every read (the MFMA pipe sat idle ~2/3 of the time: PMC 37 % MFMA busy).
template <int D, int PRIO, bool EVO = false, int PIPE = 0>
__global__ __launch_bounds__(512) void attn_bwd_dkdv_split_kernel(AttnParams p) {
  constexpr int BK = 128;
  constexpr int KS = Dim<D>::KS, DT = Dim<D>::DT;
  static_assert(D <= 128, "split dK/dV kernel keeps 8 tiles in LDS: head_dim <= 128");
  // LDS: K (2 x 16K), V (2 x 16K), Q[2] (16K each), dO[2] (16K each), lse[2][64], delta[2][64]
  __shared__ __attribute__((aligned(1024))) char smem[8 * 16384 + 4 * 256];  // 1 KiB: rows_x / tr_x bases
  char* const Kt = smem;
  char* const Vt = smem + 2 * 16384;
  char* const Qbase = smem + 4 * 16384;
  char* const Obase = smem + 6 * 16384;
  float* const LDbase = reinterpret_cast<float*>(smem + 8 * 16384);
  int kb, hk, b;
  lpt_ids(kb, hk, b);
  int start, len;
  seq_bounds(p, b, start, len);
  const int nkb = (len + BK - 1) / BK;
  if (kb >= nkb || len == 0) return;
  const int G = p.hq / p.hkv;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int kg = w & 3, qh = w >> 2;
  const int kw0 = kb * BK + 32 * kg;  // this wave's first key
  const int myk = kw0 + (lane & 31);
  int qlo, qhi;
  query_span(p, myk, len, qlo, qhi);
  const float c = p.scale * kLog2e;
  const char* Kw = Kt + (kg >> 1) * 16384;
  const char* Vw = Vt + (kg >> 1) * 16384;
  const int krow0 = 32 * (kg & 1);
  // PIPE: one per-lane register per operand role (closed-form XOR-layout addresses, attn_common.h)
  const uint32_t pq = rows_lane_off(32 * qh), pk = rows_lane_off(krow0);
  uint32_t ty0, ty1;
  tr_lane_offs(ty0, ty1);

  // K / V tiles of the block (rows clamped to the sequence)
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    stage_tile_d<8, D>(Kt + t * 16384, [=](int row) {
      int r = kb * BK + 64 * t + row;
      r = r < len ? r : len - 1;
      return p.k + (int64_t)(start + r) * p.sk + (int64_t)hk * D;
    });
    stage_tile_d<8, D>(Vt + t * 16384, [=](int row) {
      int r = kb * BK + 64 * t + row;
      r = r < len ? r : len - 1;
      return p.v + (int64_t)(start + r) * p.sv + (int64_t)hk * D;
    });
  }

  f32x16 dk[DT], dv[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) dk[i] = dv[i] = f32x16{};

  int qt_begin = 0;
  if (p.causal) qt_begin = (kb * BK) / BN;
  int qt_end = (len + BN - 1) / BN;
  if (p.window > 0) {
    const int lastq = kb * BK + BK - 1 + p.window - 1;
    const int e = lastq / BN + 1;
    qt_end = e < qt_end ? e : qt_end;
  }
  const int nqt = qt_end - qt_begin;
  const int total = nqt * G;

  int32_t oq[2] = {0, 0}, odo[2] = {0, 0};
  if constexpr (PIPE >= 2 && D == 128) {
    dma_offs8(p.sq, oq);
    dma_offs8(p.sdo, odo);
  }
  auto stage = [&](int it, int buf) {
    const int g = it / nqt, qt = qt_begin + it % nqt;
    const int hq = hk * G + g;
    if constexpr (PIPE >= 2 && D == 128) {
      if (qt * BN + BN <= len && p.sq < (1 << 24) && p.sdo < (1 << 24)) {  // 32-bit lane offsets
        const int64_t r0 = start + qt * BN;
        stage_full8(Qbase + buf * 16384, p.q + r0 * p.sq + (int64_t)hq * D, oq);
        stage_full8(Obase + buf * 16384, p.dout + r0 * p.sdo + (int64_t)hq * D, odo);
        if (w < 2) {  // PIPE 2 launches guarantee p.lse2 (the pre-scaled lse)
          const float* src = (w == 0 ? p.lse2 : p.delta) + (int64_t)hq * p.total_tokens + r0 + lane;
          __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(LDbase + buf * 64 + w * 128), 4, 0, 0);
        }
        return;
      }
    }
    stage_tile_d<8, D>(Qbase + buf * 16384, [=](int row) {
      int r = qt * BN + row;
      r = r < len ? r : len - 1;
      return p.q + (int64_t)(start + r) * p.sq + (int64_t)hq * D;
    });
    stage_tile_d<8, D>(Obase + buf * 16384, [=](int row) {
      int r = qt * BN + row;
      r = r < len ? r : len - 1;
      return p.dout + (int64_t)(start + r) * p.sdo + (int64_t)hq * D;
    });
    if (w < 2) {
      int r = qt * BN + lane;
      r = r < len ? r : len - 1;
      const float* src = (w == 0 ? (PIPE >= 2 ? p.lse2 : p.lse) : p.delta) + (int64_t)hq * p.total_tokens + start + r;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(LDbase + buf * 64 + w * 128), 4, 0, 0);
    }
  };

  if (total > 0) stage(0, 0);
  __syncthreads();
  if constexpr (PRIO != 0) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  }
  for (int it = 0; it < total; ++it) {
    const int buf = it & 1;
    if (it + 1 < total) stage(it + 1, buf ^ 1);
    const int qt = qt_begin + it % nqt;
    const char* Qt = Qbase + buf * 16384;
    const char* Ot = Obase + buf * 16384;
    const float* Lt = LDbase + buf * 64;
    const float* Dt = LDbase + 128 + buf * 64;
    const int q0 = qt * BN + 32 * qh;  // this wave's first query
    bool skip = (kw0 >= len) || (q0 >= len);
    if (p.causal && q0 + 31 < kw0) skip = true;
    if (p.window > 0 && q0 > kw0 + 31 + p.window - 1) skip = true;
    if (!skip) {
      const bool need_mask = (p.causal && q0 < kw0 + 31) || p.window > 0 || q0 + 32 > len || kw0 + 32 > len;
      f32x16 sacc = f32x16{}, dpacc = f32x16{};
      if constexpr (PIPE != 0 && D == 128) {  // (PIPE 2: same loop, fast staging above)
        bf16x8 fa[3], fb[3];
        // O tile = Q tile + 2 slots, V = K + 2 slots: immediates on one base register each
        const uint32_t bq = (uint32_t)(uintptr_t)Qt + pq, bk = (uint32_t)(uintptr_t)Kw + pk;
        auto ld = [&](int j) {
          const int ks = j % KS;
          if (j < KS) {
            fa[j % 3] = rows_x<0>(bq, ks);
            fb[j % 3] = rows_x<0>(bk, ks);
          } else {
            fa[j % 3] = rows_x<2 * 16384>(bq, ks);
            fb[j % 3] = rows_x<2 * 16384>(bk, ks);
          }
        };
        ld(0);
        ld(1);
#pragma unroll
        for (int j = 0; j < 2 * KS; ++j) {
          if (j + 2 < 2 * KS) {
            ld(j + 2);
            lds_wait_tie<4>(fa[j % 3], fb[j % 3]);
          } else if (j + 1 < 2 * KS) {
            lds_wait_tie<2>(fa[j % 3], fb[j % 3]);
          } else {
            lds_wait_tie<0>(fa[j % 3], fb[j % 3]);
          }
          if (j < KS)
            sacc = mfma(fa[j % 3], fb[j % 3], sacc);
          else
            dpacc = mfma(fa[j % 3], fb[j % 3], dpacc);
        }
      } else {
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) sacc = mfma(read_rows(Qt, 32 * qh, ks), read_rows(Kw, krow0, ks), sacc);
#pragma unroll
        for (int ks = 0; ks < KS; ++ks) dpacc = mfma(read_rows(Ot, 32 * qh, ks), read_rows(Vw, krow0, ks), dpacc);
      }
#pragma unroll
      for (int r4 = 0; r4 < 4; ++r4) {
        const int qr0 = 32 * qh + 8 * r4 + 4 * h;  // rows acc_row(4*r4 + j, h) = qr0 + j
        const f32x4 l4 = *reinterpret_cast<const f32x4*>(Lt + qr0);
        const f32x4 d4 = *reinterpret_cast<const f32x4*>(Dt + qr0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int r = 4 * r4 + j;
          float x = PIPE >= 2 ? sacc[r] * c - l4[j] : sacc[r] * c - l4[j] * kLog2e;  // PIPE 2: lse2 staged
          if constexpr (EVO) x += evo_bias(p, b, hk, qt * BN + qr0 + j, myk) * kLog2e;
          float pr = fast_exp2(x);
          if constexpr (EVO) {
            if (masked(p, qt * BN + qr0 + j, myk, len)) pr = 0.f;
          }
          sacc[r] = pr;
          dpacc[r] = pr * (dpacc[r] - d4[j]);
        }
      }
      if (!EVO && need_mask) {  // wave-uniform branch: interior tiles run no mask VALU at all
#pragma unroll
        for (int r = 0; r < 16; ++r)
          if (outside(qt * BN + 32 * qh + acc_row(r, h), qlo, qhi)) sacc[r] = dpacc[r] = 0.f;
      }
      const bf16x8 p0 = acc_to_b<0>(sacc), p1 = acc_to_b<1>(sacc);
      const bf16x8 s0 = acc_to_b<0>(dpacc), s1 = acc_to_b<1>(dpacc);
      if constexpr (PIPE != 0 && D == 128) {
        // j = 4 dt + r: r 0/1 -> dV with dO^T halves, r 2/3 -> dK with Q^T halves
        bf16x8 ft[3];
        // k-step s = 2 qh + (j & 1): the qh part in the base, the (j & 1) part and the O slot in the immediate
        const uint32_t b0 = (uint32_t)(uintptr_t)Qt + 8192u * qh + ty0, b1 = (uint32_t)(uintptr_t)Qt + 8192u * qh + ty1;
        auto ldt = [&](int j) {
          const int dt = j >> 2;
          switch (j & 3) {
            case 0: ft[j % 3] = tr_x<2 * 16384>(b0, b1, dt); break;         // dO^T, k-step 2 qh
            case 1: ft[j % 3] = tr_x<2 * 16384 + 4096>(b0, b1, dt); break;  // dO^T, k-step 2 qh + 1
            case 2: ft[j % 3] = tr_x<0>(b0, b1, dt); break;                 // Q^T
            default: ft[j % 3] = tr_x<4096>(b0, b1, dt); break;
          }
        };
        ldt(0);
        ldt(1);
#pragma unroll
        for (int j = 0; j < 4 * DT; ++j) {
          if (j + 2 < 4 * DT) {
            ldt(j + 2);
            lds_wait_tie<4>(ft[j % 3]);
          } else if (j + 1 < 4 * DT) {
            lds_wait_tie<2>(ft[j % 3]);
          } else {
            lds_wait_tie<0>(ft[j % 3]);
          }
          const int dt = j >> 2;
          switch (j & 3) {
            case 0: dv[dt] = mfma(ft[j % 3], p0, dv[dt]); break;
            case 1: dv[dt] = mfma(ft[j % 3], p1, dv[dt]); break;
            case 2: dk[dt] = mfma(ft[j % 3], s0, dk[dt]); break;
            default: dk[dt] = mfma(ft[j % 3], s1, dk[dt]); break;
          }
        }
      } else {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          dv[dt] = mfma(read_tr(Ot, 2 * qh, dt), p0, dv[dt]);
          dv[dt] = mfma(read_tr(Ot, 2 * qh + 1, dt), p1, dv[dt]);
          dk[dt] = mfma(read_tr(Qt, 2 * qh, dt), s0, dk[dt]);
          dk[dt] = mfma(read_tr(Qt, 2 * qh + 1, dt), s1, dk[dt]);
        }
      }
    }
    __syncthreads();
  }
  // sum the two query halves: qh=1 waves park their partials in LDS (32 KiB per wave)
  float* red = reinterpret_cast<float*>(smem) + kg * 8192;
  if (qh == 1) {
#pragma unroll
    for (int dt = 0; dt < DT; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        red[(dt * 16 + r) * 64 + lane] = dk[dt][r];
        red[(64 + dt * 16 + r) * 64 + lane] = dv[dt][r];
      }
  }
  __syncthreads();
  if (qh == 0 && myk < len) {
    bf16* kp = p.dk + (int64_t)(start + myk) * p.sdk + (int64_t)hk * D;
    bf16* vp = p.dv + (int64_t)(start + myk) * p.sdv + (int64_t)hk * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      f32x16 a, b;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        a[r] = dk[dt][r] + red[(dt * 16 + r) * 64 + lane];
        b[r] = dv[dt][r] + red[(64 + dt * 16 + r) * 64 + lane];
      }
      store_row_block<D>(kp, a, dt, h, p.scale);
      store_row_block<D>(vp, b, dt, h, 1.f);
    }
  }
}

// =====================================================================================
// backward dQ
// =====================================================================================
// PIPE: as in the dK/dV kernel -- LDS operand reads two MFMAs ahead as inline asm with counted waits, so neither
// the per-read LDS latency nor the compiler's vmcnt(0) in front of the transposed-read builtin (which waits for
// the NEXT tile's LDS-DMA in the middle of every iteration) stalls the MFMA pipe.
template <int D, int NW, int PRIO, bool EVO = false, int PIPE = 0>
__global__ __launch_bounds__(64 * NW) void attn_bwd_dq_kernel(AttnParams p) {
  constexpr int BM = 32 * NW;
  constexpr int KS = Dim<D>::KS, DT = Dim<D>::DT, TL = Dim<D>::TILE;
  __shared__ __attribute__((aligned(1024))) char smem[4 * TL];  // K[2], V[2]; 1 KiB: rows_x / tr_x bases
  int blk, hq, b;
  lpt_ids(blk, hq, b);
  int start, len;
  seq_bounds(p, b, start, len);
  const int nqb = (len + BM - 1) / BM;
  const int qb = p.causal ? (gridDim.x - 1 - blk) : blk;
  if (qb >= nqb || len == 0) return;
  const int hk = hq / (p.hq / p.hkv);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6, h = lane >> 5;
  const int q0 = qb * BM;
  const int myq = q0 + 32 * w + (lane & 31);
  const float c = p.scale * kLog2e;
  int klo, khi;
  key_span(p, myq, len, klo, khi);
  const int qr = myq < len ? myq : len - 1;

  bf16x8 qf[KS], df[KS];
  {
    const bf16* qp = p.q + (int64_t)(start + qr) * p.sq + (int64_t)hq * D + 8 * h;
    const bf16* dp = p.dout + (int64_t)(start + qr) * p.sdo + (int64_t)hq * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      qf[ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
      df[ks] = *reinterpret_cast<const bf16x8*>(dp + 16 * ks);
    }
  }
  const float lse2 = p.lse[(int64_t)hq * p.total_tokens + start + qr] * kLog2e;
  const float dlt = p.delta[(int64_t)hq * p.total_tokens + start + qr];

  int kt_end = (len + BN - 1) / BN;
  if (p.causal) {
    const int last = q0 + BM - 1 < len - 1 ? q0 + BM - 1 : len - 1;
    kt_end = last / BN + 1;
  }
  int kt_begin = 0;
  if (p.window > 0) {
    const int first = q0 - p.window + 1;
    kt_begin = first > 0 ? first / BN : 0;
  }
  auto kptr = [&](int kt) {
    return [=](int row) {
      int r = kt * BN + row;
      r = r < len ? r : len - 1;
      return p.k + (int64_t)(start + r) * p.sk + (int64_t)hk * D;
    };
  };
  auto vptr = [&](int kt) {
    return [=](int row) {
      int r = kt * BN + row;
      r = r < len ? r : len - 1;
      return p.v + (int64_t)(start + r) * p.sv + (int64_t)hk * D;
    };
  };
  f32x16 dq[DT];
#pragma unroll
  for (int i = 0; i < DT; ++i) dq[i] = f32x16{};
  const int wq_lo = q0 + 32 * w, wq_hi = q0 + 32 * w + 31;
  const uint32_t pr0 = rows_lane_off(0), pr1 = rows_lane_off(32);  // PIPE: closed-form LDS addresses
  uint32_t ty0, ty1;
  tr_lane_offs(ty0, ty1);

  int32_t okk[2] = {0, 0}, ovv[2] = {0, 0};
  if constexpr (PIPE >= 2 && D == 128 && NW == 8) {
    dma_offs8(p.sk, okk);
    dma_offs8(p.sv, ovv);
  }
  stage_tile_d<NW, D>(smem + 0, kptr(kt_begin));
  stage_tile_d<NW, D>(smem + 2 * TL, vptr(kt_begin));
  __syncthreads();
  if constexpr (PRIO != 0 && NW == 8) {
    if (__builtin_amdgcn_readfirstlane(threadIdx.x) >= 256) __builtin_amdgcn_s_setprio(1);
  }
  for (int kt = kt_begin; kt < kt_end; ++kt) {
    const int buf = (kt - kt_begin) & 1;
    const char* Kt = smem + buf * TL;
    const char* Vt = smem + 2 * TL + buf * TL;
    if (kt + 1 < kt_end) {
      if (PIPE >= 2 && D == 128 && NW == 8 && (kt + 1) * BN + BN <= len && p.sk < (1 << 24) && p.sv < (1 << 24)) {
        const int64_t r0 = start + (kt + 1) * BN;
        stage_full8(smem + (buf ^ 1) * TL, p.k + r0 * p.sk + (int64_t)hk * D, okk);
        stage_full8(smem + 2 * TL + (buf ^ 1) * TL, p.v + r0 * p.sv + (int64_t)hk * D, ovv);
      } else {
        stage_tile_d<NW, D>(smem + (buf ^ 1) * TL, kptr(kt + 1));
        stage_tile_d<NW, D>(smem + 2 * TL + (buf ^ 1) * TL, vptr(kt + 1));
      }
    }
    const int k0 = kt * BN;
    bool skip = (k0 >= len) || (wq_lo >= len);
    if (p.causal && k0 > wq_hi) skip = true;
    if (p.window > 0 && k0 + BN - 1 <= wq_lo - p.window) skip = true;
    if (!skip) {
      f32x16 s[2], dp[2];
      if constexpr (PIPE != 0 && D == 128 && !EVO) {
        // j = 16 t + 8 which + ks: which 0 -> S (K rows x Q), 1 -> dP (V rows x dO)
        s[0] = s[1] = dp[0] = dp[1] = f32x16{};
        bf16x8 fa[3];
        const uint32_t bk = (uint32_t)(uintptr_t)Kt + pr0;  // V = K + 2 slots, rows 32.. = +8192: immediates
        auto ld = [&](int j) {
          const int t = j >> 4, which = (j >> 3) & 1, ks = j & 7;
          if (which == 0)
            fa[j % 3] = t ? rows_x<8192>(bk, ks) : rows_x<0>(bk, ks);
          else
            fa[j % 3] = t ? rows_x<2 * TL + 8192>(bk, ks) : rows_x<2 * TL>(bk, ks);
        };
        ld(0);
        ld(1);
#pragma unroll
        for (int j = 0; j < 32; ++j) {
          if (j + 2 < 32) {
            ld(j + 2);
            lds_wait_tie<2>(fa[j % 3]);
          } else if (j + 1 < 32) {
            lds_wait_tie<1>(fa[j % 3]);
          } else {
            lds_wait_tie<0>(fa[j % 3]);
          }
          const int t = j >> 4, which = (j >> 3) & 1, ks = j & 7;
          if (which)
            dp[t] = mfma(fa[j % 3], df[ks], dp[t]);
          else
            s[t] = mfma(fa[j % 3], qf[ks], s[t]);
        }
      } else {
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          s[t] = f32x16{};
          dp[t] = f32x16{};
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) s[t] = mfma(rows_d(Kt, 32 * t, ks), qf[ks], s[t]);
#pragma unroll
          for (int ks = 0; ks < KS; ++ks) dp[t] = mfma(rows_d(Vt, 32 * t, ks), df[ks], dp[t]);
        }
      }
      // only tiles that straddle the causal diagonal / window edge / sequence end need the per-element mask
      const bool need_mask = (k0 + BN > len) || (p.causal && k0 + BN - 1 > wq_lo) ||
                             (p.window > 0 && k0 <= wq_hi - p.window) || (wq_hi >= len);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int key = k0 + 32 * t + acc_row(r, h);
          float x = s[t][r] * c - lse2;
          if constexpr (EVO) x += evo_bias(p, b, hq, myq, key) * kLog2e;
          float pr = fast_exp2(x);
          if constexpr (EVO) {
            const bool off = masked(p, myq, key, len);
            if (off) pr = 0.f;
            s[t][r] = pr * (dp[t][r] - dlt);  // dS^T
            // pair-bias gradient, summed over the N rows of the MSA (float atomics into [B][H][L][L])
            if (p.db2 && !off)
              atomicAdd(p.db2 + ((int64_t)((b / p.evo_n) * p.hq + hq) * len + myq) * len + key, s[t][r]);
          } else {
            s[t][r] = pr * (dp[t][r] - dlt);  // dS^T
          }
        }
      if (!EVO && need_mask) {  // wave-uniform branch: interior tiles run no mask VALU at all
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r)
            if (outside(k0 + 32 * t + acc_row(r, h), klo, khi)) s[t][r] = 0.f;
      }
      if constexpr (EVO) {
        if (p.db1) {  // mask-bias gradient: sum over this wave's 32 queries, then over heads by atomics
#pragma unroll
          for (int t = 0; t < 2; ++t)
#pragma unroll
            for (int r = 0; r < 16; ++r) {
              float v = s[t][r];
#pragma unroll
              for (int off = 1; off < 32; off <<= 1) v += __shfl_xor(v, off, 64);
              const int key = k0 + 32 * t + acc_row(r, h);
              if ((lane & 31) == 0 && key < len) atomicAdd(p.db1 + (int64_t)b * len + key, v);
            }
        }
      }
      const bf16x8 sb[4] = {acc_to_b<0>(s[0]), acc_to_b<1>(s[0]), acc_to_b<0>(s[1]), acc_to_b<1>(s[1])};
      if constexpr (PIPE != 0 && D == 128 && !EVO) {
        bf16x8 ft[3];
        const uint32_t b0 = (uint32_t)(uintptr_t)Kt + ty0, b1 = (uint32_t)(uintptr_t)Kt + ty1;
        auto ldt = [&](int j) {
          const int dt = j >> 2;
          switch (j & 3) {  // k-step s = j & 3 in the immediate
            case 0: ft[j % 3] = tr_x<0>(b0, b1, dt); break;
            case 1: ft[j % 3] = tr_x<4096>(b0, b1, dt); break;
            case 2: ft[j % 3] = tr_x<8192>(b0, b1, dt); break;
            default: ft[j % 3] = tr_x<12288>(b0, b1, dt); break;
          }
        };
        ldt(0);
        ldt(1);
#pragma unroll
        for (int j = 0; j < 4 * DT; ++j) {
          if (j + 2 < 4 * DT) {
            ldt(j + 2);
            lds_wait_tie<4>(ft[j % 3]);
          } else if (j + 1 < 4 * DT) {
            lds_wait_tie<2>(ft[j % 3]);
          } else {
            lds_wait_tie<0>(ft[j % 3]);
          }
          dq[j >> 2] = mfma(ft[j % 3], sb[j & 3], dq[j >> 2]);
        }
      } else {
#pragma unroll
        for (int dt = 0; dt < DT; ++dt)
#pragma unroll
          for (int st = 0; st < 4; ++st) dq[dt] = mfma(tr_d(Kt, st, dt), sb[st], dq[dt]);
      }
    }
    __syncthreads();
  }
  if (myq < len) {
    bf16* qp = p.dq + (int64_t)(start + myq) * p.sdq + (int64_t)hq * D;
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) store_row_block<D>(qp, dq[dt], dt, h, p.scale);
  }
}

AttnParams make_params(const void* q, const void* k, const void* v, void* o, float* lse, const void* dout, void* dq,
                       void* dk, void* dv, float* delta, const int64_t* strides, const int* cu_seqlens,
                       const int* seq_lens, int batch, int seq_len, int total_tokens, int hq, int hkv, float scale,
                       int causal, int window) {
  AttnParams p;
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
  p.lse2 = nullptr;
  p.sq = strides[0];
  p.sk = strides[1];
  p.sv = strides[2];
  p.so = strides[3];
  p.sdo = strides[4];
  p.sdq = strides[5];
  p.sdk = strides[6];
  p.sdv = strides[7];
  p.cu_seqlens = cu_seqlens;
  p.seq_lens = seq_lens;
  p.seq_len = seq_len;
  p.total_tokens = total_tokens;
  p.batch = batch;
  p.hq = hq;
  p.hkv = hkv;
  p.scale = scale;
  p.causal = causal;
  p.window = window;
  p.b1 = p.b2 = nullptr;
  p.bias_f32 = 0;
  p.db1 = p.db2 = nullptr;
  p.evo_n = 1;
  return p;
}

}  // namespace

int g_fwd_nw = 8, g_dkdv_nw = 8, g_dq_nw = 8, g_fwd_var = 20, g_bwd_prio = 1, g_bwd_pipe = 0, g_dq_var = 0;

// forward variants (hds_attn_fwd_variant). Shipped library: 20 = one wave per SIMD, 64 rows per wave, hand-scheduled
// MFMA blocks (flash_attn_w64.hip, the default); 5 = 8 waves, software-pipelined softmax (attn_fwd_sp_kernel, the
// fallback); 2 = 8 waves, deferred max (attn_fwd_kernel; the head dims other than 128 always run it).
// The A/B build (ops/build.py build_kernels_diag: -DHDS_FA_DIAG=1, its own .so) adds the experiment variants:
// 0/1/3 = attn_fwd_kernel priority / deferred-max bits, 4 = staggered wave groups, 6-8 = variant-5 ablations,
// 9-11/18 = earlier one-wave-per-SIMD schedules, 12/19/21 = cycle stamps, 13-17 = timing-only diagnostics (WRONG
// results). The shipped library rejects every one of them, so no setting can select a wrong-result kernel.
HDS_EXPORT int hds_attn_fwd_variant(int var) {
#if HDS_FA_DIAG
  if (var < 0 || var > 21) return hipErrorInvalidValue;
#else
  if (var != 2 && var != 5 && var != 20) return hipErrorInvalidValue;
#endif
  g_fwd_var = var;
  return 0;
}

// 1 when this library carries the A/B experiment / diagnostic variants (never the shipped one)
HDS_EXPORT int hds_attn_diag_build() { return HDS_FA_DIAG ? 1 : 0; }

// backward: dK/dV kernel with LDS reads pipelined two MFMAs ahead (0 / 1; head_dim 128)
HDS_EXPORT int hds_attn_bwd_pipe(int on) {
  g_bwd_pipe = on < 0 ? 0 : (on > 2 ? 2 : on);  // 2: + uniform-base LDS-DMA staging of full tiles
  return 0;
}

// backward dQ kernel: 0 = 8 waves x 32 query rows (attn_bwd_dq_kernel), 1 = one wave per SIMD x 64 rows
// (attn_bwd_dq_w64_kernel, head_dim 128)
HDS_EXPORT int hds_attn_bwd_dq_variant(int var) {
  if (var < 0 || var > 1) return hipErrorInvalidValue;
  g_dq_var = var;
  return 0;
}

// backward: static s_setprio(1) for waves 4-7 of the 8-wave dK/dV and dQ kernels (0 / 1)
HDS_EXPORT int hds_attn_bwd_prio(int on) {
  g_bwd_prio = on ? 1 : 0;
  return 0;
}

// runtime selection of the waves-per-workgroup variants (4 or 8)
HDS_EXPORT int hds_attn_config(int fwd_nw, int dkdv_nw, int dq_nw) {
  if (fwd_nw == 4 || fwd_nw == 8) g_fwd_nw = fwd_nw;
  if (dkdv_nw == 4 || dkdv_nw == 8) g_dkdv_nw = dkdv_nw;
  if (dq_nw == 4 || dq_nw == 8) g_dq_nw = dq_nw;
  return 0;
}

namespace {

template <int D>
int launch_fwd(const AttnParams& p, int batch, int max_len, int hq, hipStream_t st) {
  if constexpr (D <= 128) {
    if (g_fwd_nw == 8) {
      const dim3 grid((max_len + 255) / 256, hq, batch);
      if constexpr (D == 128) {  // the A/B variants exist for the training head dim only
        switch (g_fwd_var) {
          case 5: hipLaunchKernelGGL((attn_fwd_sp_kernel<D>), grid, dim3(512), 0, st, p); break;
          case 20: return hds_attn_fwd_w64_launch(&p, sizeof(p), batch, max_len, hq, 11, st);
#if HDS_FA_DIAG
          case 4: hipLaunchKernelGGL((attn_fwd_stg_kernel<D>), grid, dim3(512), 0, st, p); break;
          case 6: hipLaunchKernelGGL((attn_fwd_sp_kernel<D, false>), grid, dim3(512), 0, st, p); break;
          case 7: hipLaunchKernelGGL((attn_fwd_sp_kernel<D, true, true>), grid, dim3(512), 0, st, p); break;
          case 8:
            hipLaunchKernelGGL((attn_fwd_sp_kernel<D, true, false, 4>), dim3((max_len + 127) / 128, hq, batch),
                               dim3(256), 0, st, p);
            break;
          case 9: return hds_attn_fwd_w64_launch(&p, sizeof(p), batch, max_len, hq, 0, st);
          case 10: return hds_attn_fwd_w64_launch(&p, sizeof(p), batch, max_len, hq, 1, st);
          case 11: return hds_attn_fwd_w64_launch(&p, sizeof(p), batch, max_len, hq, 2, st);
          case 12: return hds_attn_fwd_w64_launch(&p, sizeof(p), batch, max_len, hq, 3, st);
          case 13: return hds_attn_fwd_w64_launch(&p, sizeof(p), batch, max_len, hq, 4, st);
          case 14: return hds_attn_fwd_w64_launch(&p, sizeof(p), batch, max_len, hq, 5, st);
          case 15: return hds_attn_fwd_w64_launch(&p, sizeof(p), batch, max_len, hq, 6, st);
          case 16: return hds_attn_fwd_w64_launch(&p, sizeof(p), batch, max_len, hq, 7, st);
          case 17: return hds_attn_fwd_w64_launch(&p, sizeof(p), batch, max_len, hq, 8, st);
          case 18: return hds_attn_fwd_w64_launch(&p, sizeof(p), batch, max_len, hq, 9, st);
          case 19: return hds_attn_fwd_w64_launch(&p, sizeof(p), batch, max_len, hq, 10, st);
          case 21: return hds_attn_fwd_w64_launch(&p, sizeof(p), batch, max_len, hq, 12, st);
          case 0: hipLaunchKernelGGL((attn_fwd_kernel<D, 8, 0>), grid, dim3(512), 0, st, p); break;
          case 1: hipLaunchKernelGGL((attn_fwd_kernel<D, 8, 1>), grid, dim3(512), 0, st, p); break;
          case 3: hipLaunchKernelGGL((attn_fwd_kernel<D, 8, 3>), grid, dim3(512), 0, st, p); break;
#endif
          default: hipLaunchKernelGGL((attn_fwd_kernel<D, 8, 2>), grid, dim3(512), 0, st, p); break;
        }
      } else {
        hipLaunchKernelGGL((attn_fwd_kernel<D, 8, 2>), grid, dim3(512), 0, st, p);
      }
      return hipGetLastError();
    }
  }
  // head_dim > 128 keeps 1 wave per SIMD (accumulators need the full register file)
  hipLaunchKernelGGL((attn_fwd_kernel<D, 4, 2>), dim3((max_len + 127) / 128, hq, batch), dim3(256), 0, st, p);
  return hipGetLastError();
}

template <int D>
int launch_bwd(const AttnParams& p, int batch, int max_len, int total_tokens, int hq, int hkv, hipStream_t st) {
  const int64_t rows = (int64_t)total_tokens * hq;
  hipLaunchKernelGGL(attn_bwd_delta_kernel<D>, dim3((rows + 15) / 16), dim3(256), 0, st, p);
  bool done = false;
  if constexpr (D <= 128) {
    if (g_dkdv_nw == 8) {
      const dim3 grid((max_len + 127) / 128, hkv, batch);
      if (g_bwd_pipe == 2 && D == 128 && p.lse2)
        hipLaunchKernelGGL((attn_bwd_dkdv_split_kernel<D, 1, false, 2>), grid, dim3(512), 0, st, p);
      else if (g_bwd_pipe && D == 128)
        hipLaunchKernelGGL((attn_bwd_dkdv_split_kernel<D, 1, false, 1>), grid, dim3(512), 0, st, p);
      else if (g_bwd_prio)
        hipLaunchKernelGGL((attn_bwd_dkdv_split_kernel<D, 1>), grid, dim3(512), 0, st, p);
      else
        hipLaunchKernelGGL((attn_bwd_dkdv_split_kernel<D, 0>), grid, dim3(512), 0, st, p);
      done = true;
    }
  }
  if (!done) {
    const dim3 grid((max_len + 127) / 128, hkv, batch);
    constexpr int DT = Dim<D>::DT;
    if constexpr (D <= 128) {
      hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, 4>), grid, dim3(256), 0, st, p);
    } else if constexpr (D < 256) {
      hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, 4, 0, DT / 2>), grid, dim3(256), 0, st, p);
      hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, 4, DT / 2, DT - DT / 2>), grid, dim3(256), 0, st, p);
    } else {  // 256: column quarters (K/V fragments alone take 128 registers)
      hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, 4, 0, 2>), grid, dim3(256), 0, st, p);
      hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, 4, 2, 2>), grid, dim3(256), 0, st, p);
      hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, 4, 4, 2>), grid, dim3(256), 0, st, p);
      hipLaunchKernelGGL((attn_bwd_dkdv_kernel<D, 4, 6, 2>), grid, dim3(256), 0, st, p);
    }
  }
  done = false;
  if constexpr (D == 128) {
    if (g_dq_var == 1) {
      const int rc = hds_attn_bwd_dq_w64_launch(&p, sizeof(p), batch, max_len, hq, st);
      if (rc != 0) return rc;
      done = true;
    }
  }
  if constexpr (D <= 128) {
    if (!done && g_dq_nw == 8) {
      const dim3 grid((max_len + 255) / 256, hq, batch);
      if (g_bwd_pipe == 2 && D == 128)
        hipLaunchKernelGGL((attn_bwd_dq_kernel<D, 8, 1, false, 2>), grid, dim3(512), 0, st, p);
      else if (g_bwd_pipe && D == 128)
        hipLaunchKernelGGL((attn_bwd_dq_kernel<D, 8, 1, false, 1>), grid, dim3(512), 0, st, p);
      else if (g_bwd_prio)
        hipLaunchKernelGGL((attn_bwd_dq_kernel<D, 8, 1>), grid, dim3(512), 0, st, p);
      else
        hipLaunchKernelGGL((attn_bwd_dq_kernel<D, 8, 0>), grid, dim3(512), 0, st, p);
      done = true;
    }
  }
  if (!done)
    hipLaunchKernelGGL((attn_bwd_dq_kernel<D, 4, 0>), dim3((max_len + 127) / 128, hq, batch), dim3(256), 0, st, p);
  return hipGetLastError();
}

#define HDS_ATTN_DIMS(X) X(32) X(48) X(64) X(80) X(96) X(112) X(128) X(160) X(192) X(256)

}  // namespace

// head dims with a compiled kernel (for python-side dispatch)
HDS_EXPORT int hds_attn_head_dim_supported(int head_dim) {
#define HDS_CASE(d) \
  if (head_dim == d) return 1;
  HDS_ATTN_DIMS(HDS_CASE)
#undef HDS_CASE
  return 0;
}

// strides: int64[8] token strides (elements) for q, k, v, o, dout, dq, dk, dv
// max_len: max sequence length in the batch (grid sizing)
// seq_lens: optional [B] valid lengths of a right-padded [B, seq_len] batch (key-padding masks); rows past a
// sequence's length are neither read as keys nor written as outputs
HDS_EXPORT int hds_attn_fwd(const void* q, const void* k, const void* v, void* o, float* lse, const int64_t* strides,
                            const int* cu_seqlens, const int* seq_lens, int batch, int seq_len, int max_len,
                            int total_tokens, int hq, int hkv, int head_dim, float scale, int causal, int window,
                            hipStream_t st) {
  if (hq % hkv) return hipErrorInvalidValue;
  AttnParams p = make_params(q, k, v, o, lse, nullptr, nullptr, nullptr, nullptr, nullptr, strides, cu_seqlens,
                             seq_lens, batch, seq_len, total_tokens, hq, hkv, scale, causal, window);
#define HDS_CASE(d) \
  if (head_dim == d) return launch_fwd<d>(p, batch, max_len, hq, st);
  HDS_ATTN_DIMS(HDS_CASE)
#undef HDS_CASE
  return hipErrorInvalidValue;
}

HDS_EXPORT int hds_attn_bwd(const void* q, const void* k, const void* v, const void* o, const float* lse,
                            const void* dout, void* dq, void* dk, void* dv, float* delta, const int64_t* strides,
                            const int* cu_seqlens, const int* seq_lens, int batch, int seq_len, int max_len,
                            int total_tokens, int hq, int hkv, int head_dim, float scale, int causal, int window,
                            hipStream_t st) {
  if (hq % hkv) return hipErrorInvalidValue;
  AttnParams p = make_params(q, k, v, (void*)o, (float*)lse, dout, dq, dk, dv, delta, strides, cu_seqlens, seq_lens,
                             batch, seq_len, total_tokens, hq, hkv, scale, causal, window);
  p.lse2 = delta + (int64_t)hq * total_tokens;  // delta scratch is [2][Hq][T]: rowsum(dO * O), then lse * log2(e)
#define HDS_CASE(d) \
  if (head_dim == d) return launch_bwd<d>(p, batch, max_len, total_tokens, hq, hkv, st);
  HDS_ATTN_DIMS(HDS_CASE)
#undef HDS_CASE
  return hipErrorInvalidValue;
}

// Evoformer attention backward (DS4Sci_EvoformerAttention): q/k/v/o/dout/dq/dk/dv [B, N, L, H, D] contiguous,
// lse / delta in this file's [H][B*N*L] layout, biases b1 [B, N, 1, 1, L] and b2 [B, 1, H, L, L] (bf16 or fp32,
// either may be null), fp32 gradient accumulators db1 [B*N, L] / db2 [B, H, L, L] (zeroed by the caller; null
// when not wanted). Runs the FlashAttention backward kernels with the biases folded into P.
HDS_EXPORT int hds_evoformer_bwd(const void* q, const void* k, const void* v, const void* o, const float* lse,
                                 const void* dout, void* dq, void* dk, void* dv, float* delta, const void* b1,
                                 const void* b2, int bias_f32, float* db1, float* db2, int B, int N, int L, int H,
                                 int D, float scale, hipStream_t st) {
  if (!(D == 32 || D == 64 || D == 128) || B <= 0 || N <= 0 || L <= 0 || H <= 0) return hipErrorInvalidValue;
  int64_t strides[8];
  for (int i = 0; i < 8; ++i) strides[i] = (int64_t)H * D;
  const int batch = B * N, total = B * N * L;
  AttnParams p = make_params(q, k, v, (void*)o, (float*)lse, dout, dq, dk, dv, delta, strides, nullptr, nullptr,
                             batch, L, total, H, H, scale, 0, 0);
  p.b1 = b1;
  p.b2 = b2;
  p.bias_f32 = bias_f32;
  p.db1 = db1;
  p.db2 = db2;
  p.evo_n = N;
  const int64_t rows = (int64_t)total * H;
  switch (D) {
#define HDS_EVO(d)                                                                                              \
  case d:                                                                                                       \
    hipLaunchKernelGGL(attn_bwd_delta_kernel<d>, dim3((rows + 15) / 16), dim3(256), 0, st, p);                 \
    hipLaunchKernelGGL((attn_bwd_dkdv_split_kernel<d, 1, true>), dim3((L + 127) / 128, H, batch), dim3(512), 0, \
                       st, p);                                                                                  \
    hipLaunchKernelGGL((attn_bwd_dq_kernel<d, 8, 1, true>), dim3((L + 255) / 256, H, batch), dim3(512), 0, st, \
                       p);                                                                                      \
    break;
    HDS_EVO(32)
    HDS_EVO(64)
    HDS_EVO(128)
#undef HDS_EVO
  }
  return hipGetLastError();
}
