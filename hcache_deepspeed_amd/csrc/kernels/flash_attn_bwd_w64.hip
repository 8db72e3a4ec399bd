// FlashAttention backward dQ, one wave per SIMD, 64 query rows per wave (head_dim 128). Its own translation unit so it
// builds with the VGPR-form MFMA selection (ops/build.py FILE_FLAGS), like the forward's flash_attn_w64.hip.
//
// Why: the 8-wave dQ kernel (flash_attn.hip attn_bwd_dq_kernel) gives every wave 32 query rows, so each K / V / K^T
// fragment read from LDS feeds ONE MFMA -- 1 KiB of LDS per 32x32x16 MFMA per wave, i.e. the LDS port at 100 % when all
// four SIMDs run MFMAs back to back (PMC: ~1.0 PF/s). Here a wave owns 64 query rows (two 32-row halves qh), every LDS
// fragment feeds both halves (0.5 KiB per MFMA), and the wave runs alone on its SIMD with a 512-register budget:
//   accumulator file: Q and dO fragments (2 x 2 x 8 x 4 = 128, MFMA "a" operands) and dQ^T (4 x 2 x 16 = 128)
//   arch VGPRs: S^T / dP^T of two 32-key halves (the one being consumed and the one being produced, 128), the bf16
//               dS fragments, the K / V fragment ring, the K^T fragments
// Per 64-key tile and wave: 32 S + 32 dP + 32 dQ MFMAs. Software pipeline over 32-key halves:
//   block A (32 asm MFMAs: S and dP of the NEXT half) -- each followed by one score of THIS half: x = S c - lse2,
//            P = exp2(x), dS = P (dP - delta), and every second slot one v_cvt_pk_bf16_f32 (~22 issue cycles per gap)
//   block B (16 asm MFMAs: dQ^T += K^T . dS^T of this half) -- K^T transposed reads, the LDS-DMA pieces of tile kt+2
// K / V tiles are TRIPLE-buffered in LDS (96 KiB): tile kt+2 streams in during tile kt, one barrier per tile. The
// mask is one uniform branch per half on the diagonal / window / sequence-end halves (P = exp2(x - 2^20 c) = 0).
// hipcc neither models nor pads asm MFMA hazards: block A ends with 13 wait states before VALU reads S / dP, the first
// dQ MFMA after the dS conversion opens with s_nop 1, and dQ is read back (epilogue) after a full drain.
#include "flash_attn_shared.h"

namespace {

__device__ __forceinline__ void mfma_av_first(f32x16& s, const bf16x8& a, const bf16x8& b) {  // s = A . B (b in AGPRs)
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, 0" : "=&v"(s) : "v"(a), "a"(b));
}
__device__ __forceinline__ void mfma_av(f32x16& s, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+v"(s) : "v"(a), "a"(b));
}
__device__ __forceinline__ void mfma_acc(f32x16& o, const bf16x8& a, const bf16x8& b) {  // o (AGPRs) += A . B
  asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(o) : "v"(a), "v"(b));
}
__device__ __forceinline__ void mfma_acc_fresh(f32x16& o, const bf16x8& a, const bf16x8& b) {  // b just written
  asm volatile("s_nop 1\n\tv_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(o) : "v"(a), "v"(b));
}
__device__ __forceinline__ void xdl_drain_bw() { asm volatile("s_nop 15\n\ts_nop 15\n\ts_nop 3" ::: "memory"); }
constexpr float kPenBw = 1048576.f;  // 2^20: a masked score drops by this (exp2 -> 0; no -inf arithmetic)

__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(1, 1))) void attn_bwd_dq_w64_kernel(AttnParams p) {
  constexpr int D = 128, NW = 4, BM = 64 * NW, PW = 16 / NW;
  constexpr int KS = Dim<D>::KS, DT = Dim<D>::DT, TL = Dim<D>::TILE;  // 8 k-steps, 4 column blocks, 16 KiB tiles
  __shared__ __attribute__((aligned(1024))) char smem[6 * TL];       // (K, V) x 3 tiles
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
  float lse2[2], dlt[2];
  bf16x8 qf[2][KS], df[2][KS];  // accumulator file ("a" operands)
#pragma unroll
  for (int qh = 0; qh < 2; ++qh) {
    myq[qh] = wq_lo + 32 * qh + (lane & 31);
    key_span(p, myq[qh], len, klo[qh], khi[qh]);
    const int qr = myq[qh] < len ? myq[qh] : len - 1;
    const bf16* qp = p.q + (int64_t)(start + qr) * p.sq + (int64_t)hq * D + 8 * h;
    const bf16* dp = p.dout + (int64_t)(start + qr) * p.sdo + (int64_t)hq * D + 8 * h;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      qf[qh][ks] = *reinterpret_cast<const bf16x8*>(qp + 16 * ks);
      df[qh][ks] = *reinterpret_cast<const bf16x8*>(dp + 16 * ks);
    }
    lse2[qh] = p.lse2 ? p.lse2[(int64_t)hq * p.total_tokens + start + qr]
                      : p.lse[(int64_t)hq * p.total_tokens + start + qr] * kLog2e;
    dlt[qh] = p.delta[(int64_t)hq * p.total_tokens + start + qr];
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
  // LDS layout: K tiles in slots 0..2 at [0, 48 KiB), V tiles at [48, 96 KiB) -- every LDS read is an immediate offset
  // (< 64 KiB) on one of two per-lane base registers
  // K / V tile kt through buffer descriptors (flash_attn_shared.h tile_dma): every lane keeps its constant offsets
  // dk / dv, and the rows of a partial last tile past the sequence end land as zeros (range check) instead of being
  // clamped per lane and piece on every tile
  struct Dma {
    TileSrc k, v;
  };
  auto dma_prep = [&](int kt, Dma& d) {
    d.k = tile_src<D>(p.k, p.sk, start, kt, hk, len);
    d.v = tile_src<D>(p.v, p.sv, start, kt, hk, len);
  };
  auto dma_piece = [&](const Dma& d, int slot, int j) {  // j < PW: K piece j, else V piece j - PW
    if (j < PW)
      tile_dma(d.k, smem + slot * TL + (w * PW + j) * 1024, dk[j]);
    else
      tile_dma(d.v, smem + (3 + slot) * TL + (w * PW + j - PW) * 1024, dv[j - PW]);
  };
  const uint32_t sbase = (uint32_t)(uintptr_t)smem;
  uint32_t ar[KS], arv[KS], at0[DT], at1[DT];  // row-fragment (K, V) / transposed-fragment (K) lane addresses
  {
    const uint32_t P0 = rows_lane_off(0);
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      ar[ks] = sbase + (P0 ^ (32u * ks));
      arv[ks] = ar[ks] + 3 * TL;
    }
    uint32_t y0, y1;
    tr_lane_offs(y0, y1);
#pragma unroll
    for (int dt = 0; dt < DT; ++dt) {
      at0[dt] = sbase + (y0 ^ (64u * dt));
      at1[dt] = sbase + (y1 ^ (64u * dt));
    }
  }
  f32x16 dq[DT][2];  // dQ^T, accumulator file ("+a")
#pragma unroll
  for (int dt = 0; dt < DT; ++dt) dq[dt][0] = dq[dt][1] = f32x16{};

  // S^T / dP^T of a 32-key half, two halves in flight: sd[pair][0 = S, 1 = dP][qh]
  f32x16 sd[2][2][2];
  // block A: S and dP of the half (tile slot SLOT, key half T) into sd[PR]; each MFMA m = 0..31 followed by FX(m).
  // Fragment groups g: 0 = K k-steps 0-3, 1 = K 4-7, 2 = V 0-3, 3 = V 4-7, a ring of three (two in flight).
  auto block_a = [&](auto SLOTC, auto TC, auto PRC, auto&& FX) {
    constexpr int SLOT = decltype(SLOTC)::value, T = decltype(TC)::value, PR = decltype(PRC)::value;
    bf16x8 kr[3][4];
    auto issue = [&](auto GC) {
      constexpr int g = decltype(GC)::value, b3 = g % 3;
      constexpr int off = SLOT * TL + 8192 * T;  // on ar (K) or arv (V)
      static_for<4>([&](auto IC) {
        constexpr int i = decltype(IC)::value;
        kr[b3][i] = lds_b128<off>((g >> 1) ? arv[4 * (g & 1) + i] : ar[4 * (g & 1) + i]);
      });
    };
    issue(std::integral_constant<int, 0>{});
    issue(std::integral_constant<int, 1>{});
    static_for<4>([&](auto GC) {
      constexpr int g = decltype(GC)::value, b3 = g % 3, which = g >> 1, j = g & 1;
      if constexpr (g == 0) {
        issue(std::integral_constant<int, 2>{});
        lds_wait_tie<8>(kr[b3][0], kr[b3][1], kr[b3][2], kr[b3][3]);
      } else if constexpr (g == 1) {
        lds_wait_tie<4>(kr[b3][0], kr[b3][1], kr[b3][2], kr[b3][3]);
      } else if constexpr (g == 2) {
        issue(std::integral_constant<int, 3>{});  // into group 0's buffer: its MFMAs have issued
        lds_wait_tie<4>(kr[b3][0], kr[b3][1], kr[b3][2], kr[b3][3]);
      } else {
        lds_wait_tie<0>(kr[b3][0], kr[b3][1], kr[b3][2], kr[b3][3]);
      }
      static_for<8>([&](auto IC) {
        constexpr int ii = decltype(IC)::value, qh = ii >> 2, i = ii & 3, m = 8 * g + ii;
        const bf16x8& bq = which ? df[qh][4 * j + i] : qf[qh][4 * j + i];
        if constexpr (j == 0 && i == 0)
          mfma_av_first(sd[PR][which][qh], kr[b3][i], bq);
        else
          mfma_av(sd[PR][which][qh], kr[b3][i], bq);
        FX(std::integral_constant<int, m>{});
        __builtin_amdgcn_sched_barrier(0);
      });
    });
    FX(std::integral_constant<int, 32>{});  // drain of the one-slot software pipeline
    asm volatile("s_nop 7\n\ts_nop 4" ::: "memory");  // XDL result -> VALU read of S / dP
  };
  auto no_fx = [](auto) {};

  // mask of a half (key base k0h): uniform branch, only on halves that cross the diagonal / window / sequence end
  auto mask_half = [&](auto PRC, int k0h) {
    constexpr int PR = decltype(PRC)::value;
    const bool need = (k0h + 32 > len) || (p.causal && k0h + 31 > wq_lo) || (p.window > 0 && k0h <= wq_hi - p.window) ||
                      (wq_hi >= len);
    if (need) {
#pragma unroll
      for (int qh = 0; qh < 2; ++qh) {
        const int base = k0h + 4 * h;
        const int A = base - klo[qh], B = khi[qh] - base;
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int ar_ = (r & 3) + 8 * (r >> 2);
          const int pen = ((A + ar_) | (B - ar_)) >> 31;  // -1 outside [lo, hi]
          sd[PR][0][qh][r] = __builtin_fmaf((float)pen, kPenBw, sd[PR][0][qh][r]);
        }
      }
    }
  };

  // VALU of the half in sd[PR], element m = 16 qh + r, software-pipelined by one slot: slot m issues P_m =
  // exp2(S c - lse2) and dP_m - delta (kept in place), and consumes element m - 1: dS = P (dP - delta), every second
  // one packed with its predecessor into bf16 -- the exp result is an MFMA gap old when it is used (one wave per
  // SIMD: nothing else hides its latency). Slot 32 drains.
  uint32_t dsw[2][2][4];  // [qh][k-step j of the half][dword]
  auto make_fx = [&](auto PRC) {
    return [&](auto MC) {
      constexpr int PR = decltype(PRC)::value;
      constexpr int m = decltype(MC)::value;
      if constexpr (m < 32) {
        constexpr int qh = m >> 4, r = m & 15;
        float pr = fast_exp2(__builtin_fmaf(sd[PR][0][qh][r], c, -lse2[qh]));
        float dd = sd[PR][1][qh][r] - dlt[qh];
        asm volatile("" : "+v"(pr), "+v"(dd));  // issued in this slot
        sd[PR][0][qh][r] = pr;
        sd[PR][1][qh][r] = dd;
      }
      if constexpr (m >= 1) {
        constexpr int mc = m - 1, qh = mc >> 4, r = mc & 15;
        float ds = sd[PR][0][qh][r] * sd[PR][1][qh][r];
        if constexpr (r & 1) {
          uint32_t wv;
          const float prev = sd[PR][1][qh][r - 1];  // dS of r - 1, parked in dP's register by the previous slot
          asm volatile("v_cvt_pk_bf16_f32 %0, %1, %2" : "=v"(wv) : "v"(prev), "v"(ds));
          dsw[qh][r >> 3][(r & 7) >> 1] = wv;
        } else {
          asm volatile("" : "+v"(ds));  // stay in this slot
          sd[PR][1][qh][r] = ds;
        }
      }
    };
  };

  // block B: dQ^T += K^T . dS^T of the half (key half T of tile slot SLOT): 2 k-steps x 2 qh x 4 column blocks;
  // slot n = 8 j + 4 qh + dt, FXB(n) after each MFMA
  auto block_b = [&](auto SLOTC, auto TC, auto&& FXB) {
    constexpr int SLOT = decltype(SLOTC)::value, T = decltype(TC)::value;
    constexpr int KT = SLOT * TL;  // K tile of the slot
    bf16x8 dsb[2][2];
#pragma unroll
    for (int qh = 0; qh < 2; ++qh)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        dsb[qh][j] = __builtin_bit_cast(bf16x8, u32x4{dsw[qh][j][0], dsw[qh][j][1], dsw[qh][j][2], dsw[qh][j][3]});
    bf16x8 kt_[2][DT];
    static_for<DT>([&](auto DC) {
      constexpr int dt = decltype(DC)::value;
      kt_[0][dt] = lds_tr8<KT + 4096 * (2 * T)>(at0[dt], at1[dt]);
    });
    static_for<2>([&](auto JC) {
      constexpr int j = decltype(JC)::value;
      if constexpr (j == 0) {
        static_for<DT>([&](auto DC) {
          constexpr int dt = decltype(DC)::value;
          kt_[1][dt] = lds_tr8<KT + 4096 * (2 * T + 1)>(at0[dt], at1[dt]);
        });
        lds_wait_tie<8>(kt_[0][0], kt_[0][1], kt_[0][2], kt_[0][3]);
      } else {
        lds_wait_tie<0>(kt_[1][0], kt_[1][1], kt_[1][2], kt_[1][3]);
      }
      static_for<2 * DT>([&](auto IC) {
        constexpr int i = decltype(IC)::value, qh = i / DT, dt = i % DT, n = 8 * j + i;
        if constexpr (n == 0)
          mfma_acc_fresh(dq[dt][qh], kt_[j][dt], dsb[qh][j]);
        else
          mfma_acc(dq[dt][qh], kt_[j][dt], dsb[qh][j]);
        FXB(std::integral_constant<int, n>{});
        __builtin_amdgcn_sched_barrier(0);
      });
    });
  };

  // prologue: tiles kt_begin, kt_begin + 1 in flight; S / dP of the first half
  {
    Dma d0, d1;
    dma_prep(kt_begin, d0);
    dma_prep(min(kt_begin + 1, kt_end - 1), d1);
    for (int j = 0; j < 2 * PW; ++j) dma_piece(d0, 0, j);
    for (int j = 0; j < 2 * PW; ++j) dma_piece(d1, 1, j);
  }
  asm volatile("s_waitcnt vmcnt(8)" ::: "memory");  // this wave's pieces of tile kt_begin
  __syncthreads();
  block_a(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{}, no_fx);
  mask_half(std::integral_constant<int, 0>{}, kt_begin * BN);

  auto tile = [&](auto SLOTC, int kt) {
    constexpr int SLOT = decltype(SLOTC)::value, NXT = (SLOT + 1) % 3, FAR = (SLOT + 2) % 3;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tile kt + 1 (issued during tile kt - 1) landed
    __syncthreads();                                 // ... for every wave; tile kt - 1's slot is free
    Dma dfar;
    dma_prep(min(kt + 2, kt_end - 1), dfar);  // past the end: a harmless re-read into a dead slot
    // half 0 of tile kt consumed, half 1 produced
    block_a(SLOTC, std::integral_constant<int, 1>{}, std::integral_constant<int, 1>{},
            make_fx(std::integral_constant<int, 0>{}));
    mask_half(std::integral_constant<int, 1>{}, kt * BN + 32);
    block_b(SLOTC, std::integral_constant<int, 0>{}, [&](auto NC) {
      constexpr int n = decltype(NC)::value;
      if constexpr (n % 4 == 1) dma_piece(dfar, FAR, n / 4);  // pieces 0..3 (K)
    });
    // half 1 of tile kt consumed; half 0 of tile kt + 1 produced (past the end: a stale slot, discarded)
    block_a(std::integral_constant<int, NXT>{}, std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{},
            make_fx(std::integral_constant<int, 1>{}));
    mask_half(std::integral_constant<int, 0>{}, (kt + 1) * BN);
    block_b(SLOTC, std::integral_constant<int, 1>{}, [&](auto NC) {
      constexpr int n = decltype(NC)::value;
      if constexpr (n % 4 == 1) dma_piece(dfar, FAR, PW + n / 4);  // pieces 4..7 (V)
    });
  };
  int kt = kt_begin;
  for (; kt + 2 < kt_end; kt += 3) {
    tile(std::integral_constant<int, 0>{}, kt);
    tile(std::integral_constant<int, 1>{}, kt + 1);
    tile(std::integral_constant<int, 2>{}, kt + 2);
  }
  if (kt < kt_end) tile(std::integral_constant<int, 0>{}, kt);
  if (kt + 1 < kt_end) tile(std::integral_constant<int, 1>{}, kt + 1);

  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // no LDS-DMA in flight when the workgroup retires
  xdl_drain_bw();
#pragma unroll
  for (int qh = 0; qh < 2; ++qh) {
    if (myq[qh] < len) {
      bf16* qp = p.dq + (int64_t)(start + myq[qh]) * p.sdq + (int64_t)hq * D;
#pragma unroll
      for (int dt = 0; dt < DT; ++dt) store_row_block<D>(qp, dq[dt][qh], dt, h, p.scale);
    }
  }
}

}  // namespace

int hds_attn_bwd_dq_w64_launch(const void* params, size_t params_bytes, int batch, int max_len, int hq,
                               hipStream_t st) {
  if (params_bytes != sizeof(AttnParams)) return hipErrorInvalidValue;
  const AttnParams& p = *static_cast<const AttnParams*>(params);
  hipLaunchKernelGGL(attn_bwd_dq_w64_kernel, dim3((max_len + 255) / 256, hq, batch), dim3(256), 0, st, p);
  return hipGetLastError();
}
