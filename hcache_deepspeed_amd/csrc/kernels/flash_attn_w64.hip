// FlashAttention forward, one wave per SIMD, 64 query rows per wave: variants 9-21 of hds_attn_fwd_variant, 20 the
// library default. Its own translation unit so that it builds with its own code-generation options (ops/build.py
// FILE_FLAGS: -amdgpu-mfma-vgpr-form, no SLP vectorisation).
#include "flash_attn_shared.h"

namespace {

// =====================================================================================
// forward, one wave per SIMD, 64 query rows per wave, hand-owned accumulator file
// =====================================================================================
// The guide's one-wave-per-SIMD structure (cdna_hip_programming.md "4-wave, one-wave-per-SIMD"): 4 waves x 64 query
// rows = 256 rows per workgroup, so every K/V fragment read from LDS feeds TWICE the MFMAs of the 8-wave kernel and
// each SIMD runs one instruction stream. Per tile and wave: 32 S MFMAs (2 key halves x 2 query halves x 8 k-steps) +
// 32 P.V MFMAs = 64 v_mfma_f32_32x32x16_bf16 (the 2,048-cycle floor of a tile).
// Register plan (512 per lane): O^T (4 column blocks x 2 query halves x 16) = 128 in the ACCUMULATOR file through
// inline-asm MFMAs ("+a"); variant 11 also keeps Q (64) there as the S MFMAs' "a" operand; S, P and the K/V fragments
// are arch VGPRs. hipcc neither models nor pads an asm MFMA's hazards (guide §5.7 item 2), so: block A ends with the
// wait states an XDL result needs before a VALU reads it, the first P.V MFMA after the bf16 P is written opens with
// s_nop 1, and the O read-back (rescale, epilogue) is preceded by a full drain.
//   variant 9  (MODE 0): S_{kt+1} beside the whole softmax of tile kt, P.V alone (hipcc-scheduled builtins for S)
//   variant 10 (MODE 1): the softmax split over both MFMA blocks (below), builtin S MFMAs
//   variant 11 (MODE 2): 10 with block A hand-scheduled: asm S MFMAs on Q in AGPRs, each followed by its VALU slot
//   variants 12-17: 11 + s_memtime stamps per segment (12), timing-only diagnostics (13-17)
//   variant 18 (MODE 9): 11 with the LDS-DMA pieces spread over all of block A; 20 (MODE 11, the default): 18 with the
//   first P.V group's V fragments read in block A's last slots; 19 / 21: their stamps
__device__ __forceinline__ void mfma_pv(f32x16& o, const bf16x8& v, const bf16x8& pb) {  // O^T(a) += V^T . P^T
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(o) : "v"(v), "v"(pb));
}
__device__ __forceinline__ void mfma_pv_fresh(f32x16& o, const bf16x8& v, const bf16x8& pb) {  // P just written
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(o) : "v"(v), "v"(pb));
}
// S MFMAs of the hand-scheduled block A (variant 11): Q from the accumulator file ("a"), K and S in VGPRs. hipcc does
// not pad asm MFMA hazards: the block ends with 13 wait states before any VALU reads S (s_tile_m).
__device__ __forceinline__ void mfma_s_first(f32x16& s, const bf16x8& k, const bf16x8& q) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(s) : "v"(k), "a"(q));
}
__device__ __forceinline__ void mfma_s(f32x16& s, const bf16x8& k, const bf16x8& q) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(s) : "v"(k), "a"(q));
}
// max / sum with the other 32-lane half (lane ^ 32) through v_permlane32_swap: a VALU op, where __shfl_xor may become a
// ds_bpermute round trip through the LDS pipe (~100+ cycles, exposed at one wave per SIMD)
__device__ __forceinline__ float xor32_max(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_max_raw(float x) {  // no NaN canonicalisation (the operands are finite)
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return max3_raw(__uint_as_float(r[0]), __uint_as_float(r[1]), __uint_as_float(r[1]));
}
__device__ __forceinline__ float xor32_sum(float x) {
  const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
// cycle stamp (cdna_hip_programming.md "In-kernel stamps"): s_memtime with its own lgkmcnt(0), fenced on both sides.
// Placed only where no LDS read is in flight (block boundaries).
__device__ __forceinline__ uint64_t memtime_stamp() {
  uint64_t t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t) : : "memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#if HDS_FA_DIAG
__device__ unsigned long long g_w64_stamps[4][8];  // per wave index: segment cycles, tiles, waves (summed)
#endif
constexpr float kMaskPen = 1048576.f;  // 2^20, times the -1 of a masked score (see mask_tile)
__device__ __forceinline__ void xdl_drain() { asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 3" ::: "memory"); }

template <int D, int MODE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void attn_fwd_w64_kernel(AttnParams p) {
  constexpr int NW = 4, BM = 64 * NW, PW = 16 / NW;
  constexpr int KS = Dim<D>::KS, DT = Dim<D>::DT, TL = Dim<D>::TILE;
  static_assert(D == 128, "one-wave-per-SIMD forward: head_dim 128");
  constexpr bool REB = MODE >= 1;     // softmax VALU split over both MFMA blocks (variant 10)
  constexpr bool MANUAL_A = MODE >= 2;  // block A as asm MFMAs reading Q from the accumulator file (variant 11)
  // variant 18 (MODE 9) = 11 with the 8 LDS-DMA pieces spread over all of block A (one per 4 slots); 20 (MODE 11) = 18
  // with the first P.V group's V fragments read in block A's last 8 slots (after its last K wait); 19 / 21 = their stamps
  constexpr bool SPREAD = MODE >= 9, VPRE = MODE >= 11;
  constexpr bool STAMPS = (MODE >= 3 && MODE <= 8) || MODE == 10 || MODE == 12;  // 12 = 11 + per-segment stamps
  // timing-only diagnostics (wrong results, never a default): 13 = 12 with v_mul in place of v_exp_f32 in block A,
  // 14 = 12 with the LDS-DMA pieces issued in block B instead of block A
  constexpr bool DIAG_NOEXP = MODE == 4, DIAG_NOVALU_A = MODE == 6, DIAG_NOAGPR = MODE == 7;
  constexpr bool DIAG_SACC = MODE == 8;  // 17: S MFMAs accumulate into the accumulator file (garbage O: timing only)
  constexpr bool DIAG_DMA_B = MODE == 5 || MODE == 6;  // 15: block A without its VALU slots; 16: S MFMAs on VGPRs only
  uint64_t st_acc[6] = {0, 0, 0, 0, 0, 0}, st_prev = 0;
  auto stamp = [&](auto SEG) {
    if constexpr (STAMPS) {
      constexpr int sg = decltype(SEG)::value;
      const uint64_t t = memtime_stamp();
      if constexpr (sg >= 0) st_acc[sg] += t - st_prev;
      st_prev = t;
    }
  };
  __shared__ __attribute__((aligned(1024))) char smem[4 * TL];  // K[2], V[2]
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
  const int wq_lo = q0 + 64 * w, wq_hi = wq_lo + 63;
  const float c = p.scale * kLog2e;
  int myq[2], klo[2], khi[2];
#pragma unroll
  for (int qh = 0; qh < 2; ++qh) {
    myq[qh] = wq_lo + 32 * qh + (lane & 31);
    key_span(p, myq[qh], len, klo[qh], khi[qh]);
  }
  bf16x8 qf[2][KS];  // accumulator file (asm "a" operands)
#pragma unroll
  for (int qh = 0; qh < 2; ++qh) {
    const int qr = myq[qh] < len ? myq[qh] : len - 1;
    const bf16* qp = p.q + (int64_t)(start + qr) * p.sq + (int64_t)hq * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) qf[qh][ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
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
  int32_t dk[PW], dv[PW];
#pragma unroll
  for (int i = 0; i < PW; ++i) {
    const int row = 4 * (w * PW + i) + (lane >> 4);
    const int ch = (lane & 15) ^ swz(row);
    dk[i] = (int32_t)(((int64_t)row * p.sk + 8 * ch) * 2);
    dv[i] = (int32_t)(((int64_t)row * p.sv + 8 * ch) * 2);
  }
  // LDS-DMA of tile kt: wave-uniform tile base + this lane's byte offset; the last, partial tile clamps its rows to
  // the sequence end (the same instruction stream, offsets recomputed)
  auto stage = [&](char* dst, const bf16* base, int64_t stride, const int32_t* off, int kt) {
    const char* tb = (const char*)(base + (int64_t)(start + kt * BN) * stride + (int64_t)hk * D);
    const bool full = kt * BN + BN <= len;
#pragma unroll
    for (int i = 0; i < PW; ++i) {
      int32_t o = off[i];
      if (!full) {
        const int row = 4 * (w * PW + i) + (lane >> 4);
        const int r = min(kt * BN + row, len - 1) - kt * BN;
        o = (int32_t)(((int64_t)r * stride + 8 * ((lane & 15) ^ swz(row))) * 2);
      }
      __builtin_amdgcn_global_load_lds((gbl_void*)(tb + o), (lds_void*)(dst + (w * PW + i) * 1024), 16, 0, 0);
    }
  };
  const uint32_t sbase = (uint32_t)(uintptr_t)smem;
  uint32_t ak[KS], av0[DT], av1[DT];
  {
    const uint32_t P0 = rows_lane_off(0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) ak[ks] = sbase + (P0 ^ (32u * ks));
    uint32_t y0, y1;
    tr_lane_offs(y0, y1);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      av0[dt] = sbase + (y0 ^ (64u * dt));
      av1[dt] = sbase + (y1 ^ (64u * dt));
    }
  }
  f32x16 o[DT][2];  // accumulator file (asm "+a")
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) o[dt][0] = o[dt][1] = f32x16{};
  float m[2] = {-INFINITY, -INFINITY}, l[2] = {0.f, 0.f};

  // S of one 64-key tile for both query halves, sn[t][qh] (t = key half), K fragments streamed 4 at a time; beside
  // its 32 MFMAs, FX(chunk) runs the softmax VALU of the PREVIOUS tile in 4 chunks (the MFMAs are the builtin in its
  // VGPR form -- this TU is built with -amdgpu-mfma-vgpr-form -- so sched_group_barrier can interleave them).
  auto s_tile = [&](auto KOFF, f32x16 (&sn)[2][2], auto&& FX) {
    constexpr bool TRANS_SPLIT = REB;
    constexpr int KO = decltype(KOFF)::value;
    static_for<2>([&](auto TC) {
      constexpr int t = decltype(TC)::value;
      bf16x8 kr[2][4];
      static_for<4>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        kr[0][i] = lds_b128<KO + 8192 * t>(ak[i]);
      });
      static_for<2>([&](auto JC) {
        constexpr int j = decltype(JC)::value;
        if constexpr (j == 0) {
          static_for<4>([&](auto IC) {
            constexpr int i = decltype(IC)::value;
            kr[1][i] = lds_b128<KO + 8192 * t>(ak[4 + i]);
          });
          lds_wait_tie<4>(kr[0][0], kr[0][1], kr[0][2], kr[0][3]);
        } else {
          lds_wait_tie<0>(kr[1][0], kr[1][1], kr[1][2], kr[1][3]);
        }
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          if constexpr (j == 0) sn[t][qh] = f32x16{};
#pragma unroll
          for (int i = 0; i < 4; ++i) sn[t][qh] = mfma(kr[j][i], qf[qh][4 * j + i], sn[t][qh]);
        }
        FX(std::integral_constant<int, 2 * t + j>{});
        if constexpr (TRANS_SPLIT) {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
            __builtin_amdgcn_sched_group_barrier(0x400, 2, 0);  // 2 exp2 (8 issue cycles each)
            __builtin_amdgcn_sched_group_barrier(0x002, 3, 0);  // 2 row-sum adds + 1 cvt
          }
        } else {
#pragma unroll
          for (int i = 0; i < 8; ++i) {
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // 1 MFMA
            __builtin_amdgcn_sched_group_barrier(0x002, 6, 0);  // then ~6 VALU (fma, exp, add pairs / cvt)
          }
        }
      });
    });
  };
  auto no_fx = [](auto) {};
  // variant 11's block A: the same 32 S MFMAs as inline asm, K fragments through a 3-deep ring of 4-fragment groups
  // g = 2 t + j (two groups in flight), each MFMA followed by its VALU slot SLOT(m), m = 8 g + 4 qh + i, fenced by
  // sched_barrier so the source order is the issue order
  auto s_tile_m = [&](auto KOFF, f32x16 (&sn)[2][2], auto&& SLOT) {
    constexpr int KO = decltype(KOFF)::value;
    bf16x8 kr[3][4];
    auto issue = [&](auto GC) {
      constexpr int g = decltype(GC)::value, t = g >> 1, j = g & 1, b = g % 3;
      static_for<4>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        kr[b][i] = lds_b128<KO + 8192 * t>(ak[4 * j + i]);
      });
    };
    issue(std::integral_constant<int, 0>{});
    issue(std::integral_constant<int, 1>{});
    static_for<4>([&](auto GC) {
      constexpr int g = decltype(GC)::value, t = g >> 1, j = g & 1, b = g % 3;
      if constexpr (g == 0) {
        issue(std::integral_constant<int, 2>{});
        lds_wait_tie<8>(kr[b][0], kr[b][1], kr[b][2], kr[b][3]);
      } else if constexpr (g == 1) {
        lds_wait_tie<4>(kr[b][0], kr[b][1], kr[b][2], kr[b][3]);  // (group 3 not issued yet: 4 = group 2)
      } else if constexpr (g == 2) {
        issue(std::integral_constant<int, 3>{});  // into group 0's buffer: its MFMAs have issued
        lds_wait_tie<4>(kr[b][0], kr[b][1], kr[b][2], kr[b][3]);
      } else {
        lds_wait_tie<0>(kr[b][0], kr[b][1], kr[b][2], kr[b][3]);
      }
      static_for<8>([&](auto IC) {
        // the two query halves alternate (qh 0, 1 on K fragment i, then i + 1): consecutive MFMAs accumulate into
        // different S tiles; each chain keeps its k order
        constexpr int ii = decltype(IC)::value, qh = ii & 1, i = ii >> 1, m = 8 * g + ii;
        if constexpr (j == 0 && i == 0)
          if constexpr (DIAG_SACC)
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=a"(o[2 * t + qh][0]) : "v"(kr[b][i]), "a"(qf[qh][4 * j + i]));
          else if constexpr (DIAG_NOAGPR)
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(sn[t][qh]) : "v"(kr[b][i]), "v"(kr[b][i]));
          else
            mfma_s_first(sn[t][qh], kr[b][i], qf[qh][4 * j + i]);
        else
          if constexpr (DIAG_SACC)
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(o[2 * t + qh][0]) : "v"(kr[b][i]), "a"(qf[qh][4 * j + i]));
          else if constexpr (DIAG_NOAGPR)
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(sn[t][qh]) : "v"(kr[b][i]), "v"(kr[b][i]));
          else
            mfma_s(sn[t][qh], kr[b][i], qf[qh][4 * j + i]);
        SLOT(std::integral_constant<int, m>{});
        __builtin_amdgcn_sched_barrier(0);
      });
    });
    SLOT(std::integral_constant<int, 32>{});  // drain of a one-slot software pipeline
    asm volatile("s_nop 7\n\ts_nop 4" ::: "memory");  // XDL result -> VALU read of S
  };

  // arithmetic mask of tile kt on the scores sn: key = base + (r & 3) + 8 (r >> 2) with base = k0 + 32 t + 4 h; the
  // sign of (key - lo) | (hi - key) says "outside [lo, hi]", and a masked score drops by kMaskPen. No per-element
  // compare: 64 v_cmp masks of the two query halves live at once would spill the SGPR file. The penalty is ONE
  // moderate constant, not -inf or a multiple of 1e30: a row whose keys in the first tile are all masked takes its
  // running max from masked scores, and fma(s, c, -max) must not round above 0 by more than exp2 can take (a 1e30
  // scale rounds by ~1e22 there: exp2 -> inf, and inf x alpha = 0 -> NaN); 2^20 keeps the rounding < 0.01 and still
  // sends every masked exp2 to 0 once a real key arrives (alpha = exp2(-2^20 c) = 0 rescales the masked start away)
  auto mask_tile = [&](f32x16 (&sn)[2][2], int kt) {
    const int k0 = kt * BN;
    const bool need_mask = (k0 + BN > len) || (p.causal && k0 + BN - 1 > wq_lo) ||
                           (p.window > 0 && k0 <= wq_hi - p.window) || (wq_hi >= len);
    if (need_mask) {
#pragma unroll
      for (int qh = 0; qh < 2; ++qh)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int base = k0 + 32 * t + 4 * h;
          const int A = base - klo[qh], B = khi[qh] - base;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ar = (r & 3) + 8 * (r >> 2);
            const int pen = ((A + ar) | (B - ar)) >> 31;  // -1 outside [lo, hi], 0 inside
            sn[t][qh][r] = __builtin_fmaf((float)pen, kMaskPen, sn[t][qh][r]);
          }
        }
    }
  };

  if constexpr (REB) {
    constexpr bool kAddsInB = false;  // row sums of key half 1 in block B (more balanced, 32 more live VGPRs there)
    // ---- rebalanced pipeline: the softmax VALU of a tile is split over BOTH MFMA blocks so that no MFMA gap carries
    // more than ~24 cycles of vector issue (MI355X_MICROARCH.md, one wave per SIMD: 32-cycle gap, 8 held by the MFMA)
    //   block A (32 S_{kt+1} MFMAs): exp2 of x_kt (64 x 8 cyc), bf16 P_kt (16 cvt), K reads, half of the row sums
    //   block B (32 P_kt.V_kt MFMAs): the other row sums, the max of S_{kt+1} (32 max3), the running-max update and
    //            x_{kt+1} = S_{kt+1} c - m (64 fma), V reads
    // x_kt enters the tile already scaled and shifted: exp2 is the only op between it and P.
    f32x16 x[2][2], sn[2][2];
    float tm[2][2], alpha[2] = {1.f, 1.f}, muse[2] = {0.f, 0.f}, rs[2][2];
    bool move_any = false;
    // block-B VALU, slot s = 0..31 (one per P.V MFMA): 0..15 the max of sn, 15 the max update, 16..31 sn c - m (in
    // place: x_kt dies with the row sums of slots 0..15, and the next tile's x is this sn)
    auto bvx = [&](auto SC) {
      constexpr int sl = decltype(SC)::value;
      if constexpr (sl < 16) {
        constexpr int qh = sl >> 3, t = (sl >> 2) & 1, r = (sl & 3) * 4;
        if constexpr (r == 0) {
          tm[qh][t] = max3_raw(sn[t][qh][0], sn[t][qh][1], sn[t][qh][2]);
          tm[qh][t] = max3_raw(tm[qh][t], sn[t][qh][3], sn[t][qh][3]);
        } else {
          tm[qh][t] = max3_raw(tm[qh][t], sn[t][qh][r], sn[t][qh][r + 1]);
          tm[qh][t] = max3_raw(tm[qh][t], sn[t][qh][r + 2], sn[t][qh][r + 3]);
        }
        if constexpr (sl == 15) {
          move_any = false;
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            // branch-free (this runs between two P.V MFMAs): scores are finite after the mask (no -inf), so the
            // new max is finite, exp2(m - mnew) is 0 for the first tile's m = -inf and exactly 1 when m did not move
            const float tmax = xor32_max_raw(max3_raw(tm[q][0], tm[q][1], tm[q][1])) * c;
            const bool move = !__all(tmax <= m[q] + kDeferThr);
            const float mnew = move ? max3_raw(m[q], tmax, tmax) : m[q];
            alpha[q] = fast_exp2(m[q] - mnew);
            m[q] = mnew;
            muse[q] = mnew;
            move_any |= move;
          }
        }
      } else {
        constexpr int u = sl - 16, qh = u >> 3, t = (u >> 2) & 1, r = (u & 3) * 4;
        float y0 = __builtin_fmaf(sn[t][qh][r], c, -muse[qh]), y1 = __builtin_fmaf(sn[t][qh][r + 1], c, -muse[qh]);
        float y2 = __builtin_fmaf(sn[t][qh][r + 2], c, -muse[qh]), y3 = __builtin_fmaf(sn[t][qh][r + 3], c, -muse[qh]);
        asm volatile("" : "+v"(y0), "+v"(y1), "+v"(y2), "+v"(y3));  // stay in this slot (pure: would sink otherwise)
        sn[t][qh][r] = y0;  // in place
        sn[t][qh][r + 1] = y1;
        sn[t][qh][r + 2] = y2;
        sn[t][qh][r + 3] = y3;
      }
    };
    // row sums of the exponentials of key half 1 (chunks 2, 3 of block A), two per block-B slot 0..15
    auto badd = [&](auto SC) {
      constexpr int sl = decltype(SC)::value;
      if constexpr (kAddsInB && sl < 16) {
        constexpr int qh = sl >> 3, r = (sl & 7) * 2;
        rs[qh][0] += x[1][qh][r];
        rs[qh][1] += x[1][qh][r + 1];
      }
    };
    // block-A VALU of chunk cc = 2 t + j (8 S MFMAs): exp2 of x[t][.][8 j .. 8 j + 7] for both query halves, their
    // bf16 P fragments, and (key half 0 only) their row sums
    bf16x8 pb[2][4];
    auto fa = [&](auto CC) {
      constexpr int cc = decltype(CC)::value, t = cc >> 1, j = cc & 1;
#pragma unroll
      for (int qh = 0; qh < 2; ++qh)
#pragma unroll
        for (int r = 8 * j; r < 8 * j + 8; ++r) {
          x[t][qh][r] = fast_exp2(x[t][qh][r]);
          if constexpr (t == 0 || !kAddsInB) rs[qh][r & 1] += x[t][qh][r];
        }
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) pb[qh][2 * t + j] = j == 0 ? acc_to_b<0>(x[t][qh]) : acc_to_b<1>(x[t][qh]);
      // pin this chunk's results here: the exponentials are pure, and the optimizer would otherwise sink them past
      // the mask branch that follows block A, next to their first use in block B -- out of the S MFMAs they fill
      asm volatile("" : "+v"(pb[0][2 * t + j]), "+v"(pb[1][2 * t + j]), "+v"(rs[0][0]), "+v"(rs[0][1]), "+v"(rs[1][0]),
                   "+v"(rs[1][1]));
    };
    // variant 11: block A's VALU per S MFMA m = 8 g + 4 qh + i (g = 2 t + j): exp2 of x[t][qh][8 j + 2 i, + 1], their row
    // sums and ONE v_cvt_pk_bf16_f32 into dword i of P fragment (qh, g) -- "2 exp, 2 add, 1 cvt" in every gap
    uint32_t pw[2][4][4];
    // software-pipelined by one slot: slot m issues the exponentials of pair m and consumes (row sums, bf16 pack)
    // pair m - 1, whose v_exp_f32 results are an MFMA gap old -- at one wave per SIMD no other wave hides the
    // transcendental latency of a dependent add / cvt right behind it. Slot 32 (after the last MFMA) drains.
    auto fa_slot = [&](auto MC) {
      constexpr int m = decltype(MC)::value;
      if constexpr (m < 32) {
        constexpr int g = m >> 3, t = g >> 1, j = g & 1, qh = (m >> 2) & 1, i = m & 3, r = 8 * j + 2 * i;
        float ea, eb;
        if constexpr (DIAG_NOEXP) {
          ea = x[t][qh][r] * 0.5f;
          eb = x[t][qh][r + 1] * 0.5f;
        } else {
          ea = fast_exp2(x[t][qh][r]);
          eb = fast_exp2(x[t][qh][r + 1]);
        }
        asm volatile("" : "+v"(ea), "+v"(eb));  // issued in this slot
        x[t][qh][r] = ea;
        x[t][qh][r + 1] = eb;
      }
      if constexpr (m >= 1) {
        constexpr int mc = m - 1, g = mc >> 3, t = g >> 1, j = g & 1, qh = (mc >> 2) & 1, i = mc & 3;
        constexpr int r = 8 * j + 2 * i;
        const float ea = x[t][qh][r], eb = x[t][qh][r + 1];
        uint32_t wv;
        asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(wv) : "v"(ea), "v"(eb));
        pw[qh][g][i] = wv;
      }
    };
    // variant 11: the row sums of tile kt's exponentials run in block B (2 adds per P.V slot, its gaps have room:
    // stamps put block A at ~2,100 issue-bound cycles against block B's ~1,450); x holds them until the tile ends
    auto badd11 = [&](auto SC) {
      constexpr int sl = decltype(SC)::value, qh = sl >> 4, t = (sl >> 3) & 1, r = (sl & 7) * 2;
      float r0 = rs[qh][0] + x[t][qh][r], r1 = rs[qh][1] + x[t][qh][r + 1];
      asm volatile("" : "+v"(r0), "+v"(r1));  // stay in this slot
      rs[qh][0] = r0;
      rs[qh][1] = r1;
    };

    stage(smem + 0, p.k, p.sk, dk, kt_begin);
    stage(smem + 2 * TL, p.v, p.sv, dv, kt_begin);
    if (kt_begin + 1 < kt_end) {
      stage(smem + TL, p.k, p.sk, dk, kt_begin + 1);
      asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    }
    __syncthreads();
    if constexpr (MANUAL_A)
      s_tile_m(std::integral_constant<int, 0>{}, sn, no_fx);
    else
      s_tile(std::integral_constant<int, 0>{}, sn, no_fx);
    mask_tile(sn, kt_begin);
    static_for<32>([&](auto SC) { bvx(SC); });  // O = 0, l = 0: alpha is moot
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) x[t][qh] = sn[t][qh];

    // last tile this wave computes: past it every key follows the wave's last row (causal)
    const int kt_end_w = p.causal ? min(kt_end, wq_hi / BN + 1) : kt_end;
    auto tile = [&](auto BUFC, int kt) {
      constexpr int buf = decltype(BUFC)::value;
      constexpr int KN = (buf ^ 1) * TL;
      constexpr int VT = 2 * TL + buf * TL;
      stamp(std::integral_constant<int, 4>{});  // seg 4: the previous tile's tail (l, rescale, x = S)
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      stamp(std::integral_constant<int, 0>{});  // seg 0: DMA wait + barrier
      // V_{kt+1} and K_{kt+2} are staged by 8 LDS-DMA pieces per wave issued one per 4 P.V MFMAs in block B (its
      // vector-issue slack), not in a burst here: a piece costs its wave ~60-185 issue cycles in a burst. Past the
      // sequence end a piece re-reads the last tile into a buffer nobody reads (no branch in the MFMA block).
      const int ktv = min(kt + 1, kt_end - 1), ktk = min(kt + 2, kt_end - 1);
      // the pieces go through buffer descriptors of the two tiles (scalar base + byte count up to the end of the
      // tile's last row in the sequence): every lane keeps its constant offset dv / dk, and the rows past the end of
      // a partial last tile fail the descriptor's range check and land as zeros (masked keys, zero V rows) -- no
      // per-tile clamp of 8 per-lane offsets, each behind its own branch, between the barrier and block A
      const TileSrc rsv = tile_src<D>(p.v, p.sv, start, ktv, hk, len), rsk = tile_src<D>(p.k, p.sk, start, ktk, hk, len);
      char* const dstv = smem + 2 * TL + (buf ^ 1) * TL + w * PW * 1024;
      char* const dstk = smem + buf * TL + w * PW * 1024;
      if (kt >= kt_end_w) {  // idle tile: its keys all follow this wave's rows (causal); the wave still stages its
        // share of the tiles the other waves read and keeps the barrier count (stamps: the waves with the most mask
        // work on the diagonal tiles set the pace at every barrier)
#pragma unroll
        for (int j = 0; j < PW; ++j) {
          tile_dma(rsv, dstv + j * 1024, dv[j]);
          tile_dma(rsk, dstk + j * 1024, dk[j]);
        }
        return;
      }
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) rs[qh][0] = rs[qh][1] = 0.f;
      const bool more = kt + 1 < kt_end_w;
      // block A runs on the last tile too (S of a stale K buffer, discarded below): a branch around it would let the
      // optimizer hoist the exponentials, which both arms need, out of the MFMA block they are meant to fill
      const float m_keep[2] = {m[0], m[1]};
      bf16x8 vf[2][DT];  // V^T fragments of block B
      if constexpr (MANUAL_A) {
        // block A; the 8 LDS-DMA pieces of V_{kt+1} and K_{kt+2} go out in its first 16 slots (one per odd slot):
        // stamps (variant 12): issued in block B, the tile-start wait for them cost ~1,100 cycles per tile, issued
        // here ~770 (the rest is the barrier: waves with more mask work arrive later)
        s_tile_m(std::integral_constant<int, KN>{}, sn, [&](auto MC) {
          constexpr int m = decltype(MC)::value;
          if constexpr (!DIAG_NOVALU_A) fa_slot(MC);
          if constexpr (VPRE && m >= 24 && m < 32 && (m & 1) == 0) {  // past block A's last K wait (before m 24)
            constexpr int dt = (m - 24) >> 1;
            vf[0][dt] = lds_tr8<VT>(av0[dt], av1[dt]);
          }
          if constexpr (!DIAG_DMA_B && (SPREAD ? (m < 32 && (m & 3) == 1) : (m < 16 && (m & 1)))) {
            constexpr int j = SPREAD ? m >> 2 : m >> 1;
            if constexpr (j < PW)
              tile_dma(rsv, dstv + j * 1024, dv[j]);
            else
              tile_dma(rsk, dstk + (j - PW) * 1024, dk[j - PW]);
          }
        });
#pragma unroll
        for (int qh = 0; qh < 2; ++qh)
#pragma unroll
          for (int g = 0; g < 4; ++g)
            pb[qh][g] = __builtin_bit_cast(bf16x8, u32x4{pw[qh][g][0], pw[qh][g][1], pw[qh][g][2], pw[qh][g][3]});
      } else {
        s_tile(std::integral_constant<int, KN>{}, sn, fa);  // block A
      }
      stamp(std::integral_constant<int, 1>{});  // seg 1: DMA offsets + block A
      mask_tile(sn, kt + 1);
      stamp(std::integral_constant<int, 2>{});  // seg 2: P pack + mask
      // ---- block B: O += V_kt^T.P_kt, 32 asm MFMAs, each followed by its VALU slot (sched_barrier-fenced: hipcc
      // cannot see an asm MFMA, so the interleave is the source order) ----
      // (reading this first group in block A's last slots, or streaming K two tiles ahead through 3-slot rings so
      // block B could read the next block A's first K groups, both measured slower: 4,524-4,559 cycles per tile
      // against 4,364, profiles/r5/fa_fwd_stamps_*_r5ad/ae.txt)
      if constexpr (!VPRE) {
        static_for<DT>([&](auto DC) {
          constexpr int dt = decltype(DC)::value;
          vf[0][dt] = lds_tr8<VT>(av0[dt], av1[dt]);
        });
      }
      static_for<4>([&](auto STC) {
        constexpr int st = decltype(STC)::value;
        if constexpr (st + 1 < 4) {
          static_for<DT>([&](auto DC) {
            constexpr int dt = decltype(DC)::value;
            vf[(st + 1) & 1][dt] = lds_tr8<VT + 4096 * (st + 1)>(av0[dt], av1[dt]);
          });
          lds_wait_tie<8>(vf[st & 1][0], vf[st & 1][1], vf[st & 1][2], vf[st & 1][3]);
        } else {
          lds_wait_tie<0>(vf[st & 1][0], vf[st & 1][1], vf[st & 1][2], vf[st & 1][3]);
        }
        static_for<2 * DT>([&](auto IC) {
          constexpr int i = decltype(IC)::value, qh = i / DT, dt = i % DT, sl = 8 * st + i;
          if constexpr (sl == 0)
            mfma_pv_fresh(o[dt][qh], vf[st & 1][dt], pb[qh][st]);
          else
            mfma_pv(o[dt][qh], vf[st & 1][dt], pb[qh][st]);
          if constexpr (MANUAL_A)
            badd11(std::integral_constant<int, sl>{});
          else
            badd(std::integral_constant<int, sl>{});
          bvx(std::integral_constant<int, sl>{});
          if constexpr ((!MANUAL_A || DIAG_DMA_B) && sl % 4 == 1) {
            constexpr int j = sl / 4;
            if constexpr (j < PW)
              tile_dma(rsv, dstv + j * 1024, dv[j]);
            else
              tile_dma(rsk, dstk + (j - PW) * 1024, dk[j - PW]);
          }
          __builtin_amdgcn_sched_barrier(0);
        });
      });
      stamp(std::integral_constant<int, 3>{});  // seg 3: block B
      // l and O follow P_kt's reference max, then move to m_{kt+1} (alpha = 1 unless the max moved)
      if (!more) {  // the max update of the stale tile is void
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) {
          m[qh] = m_keep[qh];
          alpha[qh] = 1.f;
        }
        move_any = false;
      }
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) l[qh] = (l[qh] + xor32_sum(rs[qh][0] + rs[qh][1])) * alpha[qh];
      if (move_any) {  // rare: drain the P.V MFMAs before reading O back from the accumulator file
        xdl_drain();
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          o[dt][0] *= alpha[0];
          o[dt][1] *= alpha[1];
        }
      }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int qh = 0; qh < 2; ++qh) x[t][qh] = sn[t][qh];
    };
    stamp(std::integral_constant<int, -1>{});
    const uint64_t st_t0 = st_prev;
    int kt = kt_begin;
    for (; kt + 1 < kt_end; kt += 2) {
      tile(std::integral_constant<int, 0>{}, kt);
      tile(std::integral_constant<int, 1>{}, kt + 1);
    }
    if (kt < kt_end) tile(std::integral_constant<int, 0>{}, kt);
    stamp(std::integral_constant<int, 4>{});
#if HDS_FA_DIAG
    if constexpr (STAMPS) {
      st_acc[5] = st_prev - st_t0;  // the whole loop
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) atomicAdd(&g_w64_stamps[w][k], (unsigned long long)st_acc[k]);
        atomicAdd(&g_w64_stamps[w][6], (unsigned long long)(kt_end - kt_begin));
        atomicAdd(&g_w64_stamps[w][7], 1ull);
      }
    }
#endif
  } else {
  stage(smem + 0, p.k, p.sk, dk, kt_begin);
  stage(smem + 2 * TL, p.v, p.sv, dv, kt_begin);
  if (kt_begin + 1 < kt_end) {
    stage(smem + TL, p.k, p.sk, dk, kt_begin + 1);
    asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this wave's 4 K_0 pieces landed (V_0, K_1: 8 in flight)
  } else {
    asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  __syncthreads();
  f32x16 sc[2][2];
  s_tile(std::integral_constant<int, 0>{}, sc, no_fx);

  auto tile = [&](auto BUFC, int kt) {
    constexpr int buf = decltype(BUFC)::value;
    constexpr int KN = (buf ^ 1) * TL;     // K_{kt+1}
    constexpr int VT = 2 * TL + buf * TL;  // V_kt
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (kt + 1 < kt_end) stage(smem + 2 * TL + (buf ^ 1) * TL, p.v, p.sv, dv, kt + 1);
    if (kt + 2 < kt_end) stage(smem + buf * TL, p.k, p.sk, dk, kt + 2);

    const int k0 = kt * BN;
    const bool need_mask = (k0 + BN > len) || (p.causal && k0 + BN - 1 > wq_lo) ||
                           (p.window > 0 && k0 <= wq_hi - p.window) || (wq_hi >= len);
    if (need_mask) {
      // arithmetic mask (see mask_tile)
#pragma unroll
      for (int qh = 0; qh < 2; ++qh)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          const int base = k0 + 32 * t + 4 * h;
          const int A = base - klo[qh], B = khi[qh] - base;
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int ar = (r & 3) + 8 * (r >> 2);
            const int pen = ((A + ar) | (B - ar)) >> 31;
            sc[t][qh][r] = __builtin_fmaf((float)pen, kMaskPen, sc[t][qh][r]);
          }
        }
    }
    float alpha[2], muse[2];
    bool move_any = false;
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      float tm0 = -INFINITY, tm1 = -INFINITY;
#pragma unroll
      for (int r = 0; r < 16; r += 2) {
        tm0 = max3_raw(tm0, sc[0][qh][r], sc[0][qh][r + 1]);
        tm1 = max3_raw(tm1, sc[1][qh][r], sc[1][qh][r + 1]);
      }
      float tmax = fmaxf(tm0, tm1);
      tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64)) * c;
      const bool move = !__all(tmax <= m[qh] + kDeferThr);
      const float mnew = move ? fmaxf(m[qh], tmax) : m[qh];
      alpha[qh] = move ? ((m[qh] == -INFINITY) ? 0.f : fast_exp2(m[qh] - mnew)) : 1.f;
      m[qh] = mnew;
      muse[qh] = (mnew == -INFINITY) ? 0.f : mnew;
      move_any |= move;
    }
    if (move_any) {  // rare: O lives in the accumulator file, drain the last P.V MFMAs before reading it back
      xdl_drain();
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) {
        o[dt][0] *= alpha[0];
        o[dt][1] *= alpha[1];
      }
    }

    // ---- block A: S_{kt+1} (32 MFMAs) beside the whole softmax of tile kt: chunk c = 2 t + j exponentiates
    // sc[t][qh][8 j .. 8 j + 7] of both query halves (16 scores) and converts the finished bf16 P fragments ----
    float rs[2][2] = {{0.f, 0.f}, {0.f, 0.f}};
    bf16x8 pb[2][4];
    auto fx = [&](auto CC) {
      constexpr int cc = decltype(CC)::value, t = cc >> 1, j = cc & 1;
#pragma unroll
      for (int qh = 0; qh < 2; ++qh)
#pragma unroll
        for (int r = 8 * j; r < 8 * j + 8; ++r) {
          const float e = fast_exp2(__builtin_fmaf(sc[t][qh][r], c, -muse[qh]));
          sc[t][qh][r] = e;
          rs[qh][r & 1] += e;
        }
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) pb[qh][2 * t + j] = j == 0 ? acc_to_b<0>(sc[t][qh]) : acc_to_b<1>(sc[t][qh]);
    };
    f32x16 sn[2][2];
    if (kt + 1 < kt_end) {
      s_tile(std::integral_constant<int, KN>{}, sn, fx);
    } else {
      static_for<4>([&](auto CC) { fx(CC); });
    }

    // ---- block B: O += V_kt^T.P_kt (32 MFMAs, O in the accumulator file) ----
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
      for (int qh = 0; qh < 2; ++qh)
#pragma unroll
        for (int dt = 0; dt < DT; ++dt) {
          if (st == 0 && qh == 0 && dt == 0)
            mfma_pv_fresh(o[dt][qh], vf[st & 1][dt], pb[qh][st]);
          else
            mfma_pv(o[dt][qh], vf[st & 1][dt], pb[qh][st]);
        }
    });
#pragma unroll
    for (int qh = 0; qh < 2; ++qh) {
      float r = rs[qh][0] + rs[qh][1];
      r += __shfl_xor(r, 32, 64);
      l[qh] = l[qh] * alpha[qh] + r;
    }
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) sc[t][qh] = sn[t][qh];
  };
  int kt = kt_begin;
  for (; kt + 1 < kt_end; kt += 2) {
    tile(std::integral_constant<int, 0>{}, kt);
    tile(std::integral_constant<int, 1>{}, kt + 1);
  }
  if (kt < kt_end) tile(std::integral_constant<int, 0>{}, kt);

  }

  xdl_drain();
#pragma unroll
  for (int qh = 0; qh < 2; ++qh) {
    if (myq[qh] < len) {
      const float inv = l[qh] > 0.f ? 1.f / l[qh] : 0.f;
      bf16* op = p.o + (int64_t)(start + myq[qh]) * p.so + (int64_t)hq * D;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) store_row_block<D>(op, o[dt][qh], dt, h, inv);
      if (h == 0 && p.lse) {
        const float lse = (l[qh] > 0.f) ? (m[qh] + __log2f(l[qh])) / kLog2e : -INFINITY;
        p.lse[(int64_t)hq * p.total_tokens + start + myq[qh]] = lse;
      }
    }
  }
}

}  // namespace

int hds_attn_fwd_w64_launch(const void* params, size_t params_bytes, int batch, int max_len, int hq, int mode,
                            hipStream_t st) {
  if (params_bytes != sizeof(AttnParams)) return hipErrorInvalidValue;
  const AttnParams& p = *static_cast<const AttnParams*>(params);
  const dim3 grid((max_len + 255) / 256, hq, batch);
  switch (mode) {
    case 11: hipLaunchKernelGGL((attn_fwd_w64_kernel<128, 11>), grid, dim3(256), 0, st, p); break;
#if HDS_FA_DIAG
    case 0: hipLaunchKernelGGL((attn_fwd_w64_kernel<128, 0>), grid, dim3(256), 0, st, p); break;
    case 1: hipLaunchKernelGGL((attn_fwd_w64_kernel<128, 1>), grid, dim3(256), 0, st, p); break;
    case 2: hipLaunchKernelGGL((attn_fwd_w64_kernel<128, 2>), grid, dim3(256), 0, st, p); break;
    case 3: hipLaunchKernelGGL((attn_fwd_w64_kernel<128, 3>), grid, dim3(256), 0, st, p); break;
    case 4: hipLaunchKernelGGL((attn_fwd_w64_kernel<128, 4>), grid, dim3(256), 0, st, p); break;
    case 5: hipLaunchKernelGGL((attn_fwd_w64_kernel<128, 5>), grid, dim3(256), 0, st, p); break;
    case 6: hipLaunchKernelGGL((attn_fwd_w64_kernel<128, 6>), grid, dim3(256), 0, st, p); break;
    case 7: hipLaunchKernelGGL((attn_fwd_w64_kernel<128, 7>), grid, dim3(256), 0, st, p); break;
    case 8: hipLaunchKernelGGL((attn_fwd_w64_kernel<128, 8>), grid, dim3(256), 0, st, p); break;
    case 9: hipLaunchKernelGGL((attn_fwd_w64_kernel<128, 9>), grid, dim3(256), 0, st, p); break;
    case 10: hipLaunchKernelGGL((attn_fwd_w64_kernel<128, 10>), grid, dim3(256), 0, st, p); break;
    case 12: hipLaunchKernelGGL((attn_fwd_w64_kernel<128, 12>), grid, dim3(256), 0, st, p); break;
#endif
    default: return hipErrorInvalidValue;  // the shipped library holds only the default schedule (MODE 11)
  }
  return hipGetLastError();
}

#if HDS_FA_DIAG
// variant 12's (19's, 21's) stamps, out[32] = 4 wave indices x 8: [0..4] cycles per segment (DMA wait + barrier, block A, mask,
// block B, tail), [5] the whole loop, [6] tiles, [7] waves -- summed over the workgroups. reset != 0 zeroes them after.
HDS_EXPORT int hds_attn_w64_stamps(unsigned long long* out, int reset) {
  hipError_t e = hipMemcpyFromSymbol(out, HIP_SYMBOL(g_w64_stamps), sizeof(g_w64_stamps));
  if (e == hipSuccess && reset) {
    const unsigned long long z[32] = {};
    e = hipMemcpyToSymbol(HIP_SYMBOL(g_w64_stamps), z, sizeof(z));
  }
  return e;
}
#endif
