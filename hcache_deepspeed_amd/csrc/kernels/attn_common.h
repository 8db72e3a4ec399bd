// MFMA / LDS building blocks shared by the attention kernels (flash_attn.hip, paged_attn.hip).
//
// All attention math uses v_mfma_f32_32x32x16_bf16 with the "query (or key) on the lane"
// orientation: for S^T = K . Q^T the accumulator column (lane & 31) is the query, so every
// softmax row statistic is lane-local (one cross-half exchange, no LDS round trip), and the
// accumulator registers are directly the B operand of the following P.V product
// (cdna_hip_programming.md §3 "An accumulator tile as the next MFMA's operand").
//
// K/V/Q/dO tiles live in LDS as 64 rows x 256 B (head_dim 128, bf16) in the XOR layout
//   off(row, ch) = 256*row + 16*(ch ^ (((row & 3) << 2) | ((row >> 2) & 3)))
// which serves both the row reads (ds_read_b128, A operand K-rows) and the transposed reads
// (ds_read_b64_tr_b16, A operand V^T) without bank conflicts (guide §5.5 T10 image (b)).
// Tiles are filled with global_load_lds_dwordx4 (LDS-DMA): the destination is lane-linear,
// so the XOR swizzle is applied to the per-lane GLOBAL source address (guide rule 21).
#pragma once
#include "hds_common.h"

namespace hds {
namespace attn {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

__device__ __forceinline__ int swz(int row) { return ((row & 3) << 2) | ((row >> 2) & 3); }
__device__ __forceinline__ int tile_off(int row, int ch) { return row * 256 + 16 * (ch ^ swz(row)); }

// row index of accumulator register r (0..15) for lane half h in a 32x32 MFMA tile
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

// Stage a 64-row x 128-col bf16 tile into LDS with LDS-DMA. `row_ptr(row)` gives the global
// address of logical row `row` (already clamped by the caller). 16 wave-instructions of 1 KiB,
// 16/NW per wave for an NW-wave block.
template <int NW = 4, typename RowPtr>
__device__ __forceinline__ void stage_tile64(char* lds_tile, RowPtr row_ptr) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 16 / NW; ++i) {
    const int n = w * (16 / NW) + i;
    const int row = 4 * n + (lane >> 4);
    const int pc = lane & 15;
    const int ch = pc ^ swz(row);
    const char* src = (const char*)row_ptr(row) + ch * 16;
    __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(lds_tile + n * 1024), 16, 0, 0);
  }
}

// A-operand fragment from a row-major tile: rows on lanes (row0 + (lane&31)), k = 16*ks + 8h .. +7
__device__ __forceinline__ bf16x8 read_rows(const char* lds_tile, int row0, int ks) {
  const int lane = threadIdx.x & 63;
  const int row = row0 + (lane & 31);
  const int ch = 2 * ks + (lane >> 5);
  return *reinterpret_cast<const bf16x8*>(lds_tile + tile_off(row, ch));
}

// A-operand fragment of the TRANSPOSED tile (tile^T: rows = tile columns d, k = tile rows)
// for k-step s (16 tile rows starting at 16*s) and column block dt (32 columns), in the permuted
// k order that matches accumulator-derived B operands (see acc_to_b):
//   element j of lane half h  <->  tile row 16*s + 8*(j>>2) + 4*h + (j&3)
__device__ __forceinline__ bf16x8 read_tr(const char* lds_tile, int s, int dt) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int row = 16 * s + 4 * (g >> 1) + q;
  const int ch = 4 * dt + 2 * (g & 1) + (p >> 1);
  const char* a0 = lds_tile + tile_off(row, ch) + 8 * (p & 1);
  const char* a1 = lds_tile + tile_off(row + 8, ch) + 8 * (p & 1);
  bf16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)(a0));
  bf16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4bf16((__attribute__((address_space(3))) bf16x4*)(a1));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// read_tr issued as inline asm: hipcc puts an `s_waitcnt vmcnt(0)` in front of every ds_read_b64_tr_b16 builtin
// that follows an LDS-DMA (it cannot tell the DMA's destination from the tile being read), which stalls a wave on
// its own prefetch of the NEXT tile. The asm form is invisible to that analysis; the caller retires it with
// lds_wait<N>() (lgkmcnt counts in issue order, so a count that also covers compiler-issued reads stays safe).
__device__ __forceinline__ bf16x4 ds_tr_asm(const char* a) {
  bf16x4 r;
  asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"((uint32_t)(uintptr_t)a) : "memory");
  return r;
}
__device__ __forceinline__ bf16x8 read_tr_asm(const char* lds_tile, int s, int dt) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int row = 16 * s + 4 * (g >> 1) + q;
  const int ch = 4 * dt + 2 * (g & 1) + (p >> 1);
  const bf16x4 lo = ds_tr_asm(lds_tile + tile_off(row, ch) + 8 * (p & 1));
  const bf16x4 hi = ds_tr_asm(lds_tile + tile_off(row + 8, ch) + 8 * (p & 1));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}
__device__ __forceinline__ bf16x8 tr_d_asm(const char* tile, int s, int dt) {
  return read_tr_asm(tile + (dt >> 2) * 16384, s, dt & 3);
}
// Closed-form addresses of the XOR layout, for kernels short of registers: with ch = 2ks + h,
//   tile_off(row, ch) = P ^ (32 ks),            P = row*256 | 16 (h ^ swz(row))          (row reads)
// and for the transposed reads of k-step s, column block dt (rows r0 = 4(g>>1) + q and r0 + 8, c = 2(g&1) + (p>>1)):
//   off = 4096 s + (Y ^ 64 dt),                 Y = (r*256 + 8(p&1)) | 16 (c ^ swz(r))
// so each read costs one XOR with a compile-time constant on ONE per-lane register instead of one precomputed
// offset register per k-step.
__device__ __forceinline__ uint32_t rows_lane_off(int row0) {
  const int lane = threadIdx.x & 63;
  const int row = row0 + (lane & 31);
  return (uint32_t)(row * 256) | (uint32_t)(16 * ((lane >> 5) ^ swz(row)));
}
__device__ __forceinline__ bf16x8 read_rows_off_asm(const char* tile, uint32_t P, int ks) {
  bf16x8 r;
  const uint32_t a = (uint32_t)(uintptr_t)tile + (P ^ (32u * (uint32_t)ks));
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"(a) : "memory");
  return r;
}
__device__ __forceinline__ void tr_lane_offs(uint32_t& y0, uint32_t& y1) {
  const int lane = threadIdx.x & 63;
  const int g = lane >> 4, i = lane & 15, q = i >> 2, p = i & 3;
  const int c = 2 * (g & 1) + (p >> 1);
  const int r0 = 4 * (g >> 1) + q, r1 = r0 + 8;
  y0 = (uint32_t)(r0 * 256 + 8 * (p & 1)) | (uint32_t)(16 * (c ^ swz(r0)));
  y1 = (uint32_t)(r1 * 256 + 8 * (p & 1)) | (uint32_t)(16 * (c ^ swz(r1)));
}
__device__ __forceinline__ bf16x8 read_tr_off_asm(const char* tile, uint32_t y0, uint32_t y1, int s, int dt) {
  const uint32_t base = (uint32_t)(uintptr_t)tile + 4096u * (uint32_t)s;
  const bf16x4 lo = ds_tr_asm((const char*)(uintptr_t)(base + (y0 ^ (64u * (uint32_t)dt))));
  const bf16x4 hi = ds_tr_asm((const char*)(uintptr_t)(base + (y1 ^ (64u * (uint32_t)dt))));
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// Reads on a pre-added base b = tile + lane offset: with 1 KiB-aligned LDS allocations every tile base has bits 0-9
// clear, so the k-step / column-block XOR (bits 5-7) commutes with the add -- ONE v_xor per read (none for k-step /
// column block 0), and slot / sub-block offsets ride in the ds_read immediate (OFF).
template <int OFF>
__device__ __forceinline__ bf16x8 rows_x(uint32_t b, int ks) {
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1 offset:%2" : "=v"(r) : "v"(b ^ (32u * (uint32_t)ks)), "n"(OFF) : "memory");
  return r;
}
template <int OFF>
__device__ __forceinline__ bf16x8 tr_x(uint32_t b0, uint32_t b1, int dt) {
  bf16x4 lo, hi;
  const uint32_t x = 64u * (uint32_t)dt;
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(lo) : "v"(b0 ^ x), "n"(OFF) : "memory");
  asm volatile("ds_read_b64_tr_b16 %0, %1 offset:%2" : "=v"(hi) : "v"(b1 ^ x), "n"(OFF) : "memory");
  return __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7);
}

// row fragment (read_rows) issued as inline asm, retired by lds_wait<N>() like read_tr_asm
__device__ __forceinline__ bf16x8 read_rows_asm(const char* lds_tile, int row0, int ks) {
  const int lane = threadIdx.x & 63;
  const int row = row0 + (lane & 31);
  const int ch = 2 * ks + (lane >> 5);
  bf16x8 r;
  asm volatile("ds_read_b128 %0, %1" : "=v"(r) : "v"((uint32_t)(uintptr_t)(lds_tile + tile_off(row, ch))) : "memory");
  return r;
}
template <int N>
__device__ __forceinline__ void lds_wait() {
  asm volatile("s_waitcnt lgkmcnt(%0)" ::"n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);  // keep the MFMAs that consume the asm reads behind the wait (guide rule 18)
}

// lds_wait<N>() that also TIES the fragments the retired reads produced: they are in/out operands of the
// s_waitcnt, so no use of them (an MFMA) can be placed above it. An inline-asm LDS read hands its destination
// registers to the compiler as if the data were already there; the sched_barrier in lds_wait stops only the machine
// scheduler, not IR-level motion of an MFMA (no memory effects) above an asm statement it has no data dependency on.
template <int N>
__device__ __forceinline__ void lds_wait_tie(bf16x8& a) {
  asm volatile("s_waitcnt lgkmcnt(%1)" : "+v"(a) : "n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
__device__ __forceinline__ void lds_wait_tie(bf16x8& a, bf16x8& b) {
  asm volatile("s_waitcnt lgkmcnt(%2)" : "+v"(a), "+v"(b) : "n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}
template <int N>
__device__ __forceinline__ void lds_wait_tie(bf16x8& a, bf16x8& b, bf16x8& c, bf16x8& d) {
  asm volatile("s_waitcnt lgkmcnt(%4)" : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "n"(N) : "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// B-operand fragment for k-step (s & 1) of a 32-row accumulator tile: registers 8*(s&1) .. +7.
template <int HALF>
__device__ __forceinline__ bf16x8 acc_to_b(const f32x16& acc) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (bf16)acc[8 * HALF + j];
  return r;
}

__device__ __forceinline__ f32x16 mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// max of three without the NaN-canonicalising v_max_f32 x,x that hipcc puts in front of every fmaxf on an MFMA
// result (two instructions per score); the scores are finite or -inf, so IEEE NaN handling is moot here
__device__ __forceinline__ float max3_raw(float a, float b, float c) {
  float r;
  asm("v_max3_f32 %0, %1, %2, %3" : "=v"(r) : "v"(a), "v"(b), "v"(c));
  return r;
}

// ---- head-dim generic tiles -------------------------------------------------------------------
// A D-wide 64-row tile is ceil(D/128) 128-column sub-tiles in the layout above; only the first D/8 16-byte
// chunks of each row are staged. Contractions over D use exactly D/16 k-steps; products that produce D
// columns compute ceil(D/32) 32-column blocks and never store columns >= D (those blocks only read
// unstaged LDS columns, and an MFMA output row depends on one A-operand row, so nothing leaks).
template <int D>
struct Dim {
  static constexpr int KS = D / 16;           // 16-wide k-steps of the head-dim contraction
  static constexpr int DT = (D + 31) / 32;    // 32-column output blocks
  static constexpr int NT = (D + 127) / 128;  // 128-column LDS sub-tiles
  static constexpr int TILE = NT * 16384;     // bytes of one 64-row tile
  static_assert(D % 16 == 0 && D <= 256, "head_dim must be a multiple of 16, at most 256");
};

// row-fragment (A or B operand) for k-step ks of a D-wide tile
__device__ __forceinline__ bf16x8 rows_d(const char* tile, int row0, int ks) {
  return read_rows(tile + (ks >> 3) * 16384, row0, ks & 7);
}
// transposed fragment for k-step s and 32-column block dt of a D-wide tile
__device__ __forceinline__ bf16x8 tr_d(const char* tile, int s, int dt) { return read_tr(tile + (dt >> 2) * 16384, s, dt & 3); }

// Stage a 64-row x D-column tile: sub-tile c holds columns [128c, 128c + 128); only valid 16-B chunks load.
template <int NW, int D, typename RowPtr>
__device__ __forceinline__ void stage_tile_d(char* tile, RowPtr row_ptr) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int c = 0; c < Dim<D>::NT; ++c) {
    constexpr int kFull = 16;
    const int nch = (D - 128 * c) >= 128 ? kFull : (D - 128 * c) / 8;
#pragma unroll
    for (int i = 0; i < 16 / NW; ++i) {
      const int n = w * (16 / NW) + i;
      const int row = 4 * n + (lane >> 4);
      const int ch = (lane & 15) ^ swz(row);
      if (nch == kFull || ch < nch) {
        const char* src = (const char*)(row_ptr(row) + 128 * c) + ch * 16;
        __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(tile + c * 16384 + n * 1024), 16, 0, 0);
      }
    }
  }
}

// Same as stage_tile_d, but staged by a GROUP of NWG waves: wi = this wave's index inside the group.
template <int NWG, int D, typename RowPtr>
__device__ __forceinline__ void stage_tile_dw(char* tile, RowPtr row_ptr, int wi) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int c = 0; c < Dim<D>::NT; ++c) {
    constexpr int kFull = 16;
    const int nch = (D - 128 * c) >= 128 ? kFull : (D - 128 * c) / 8;
#pragma unroll
    for (int i = 0; i < 16 / NWG; ++i) {
      const int n = wi * (16 / NWG) + i;
      const int row = 4 * n + (lane >> 4);
      const int ch = (lane & 15) ^ swz(row);
      if (nch == kFull || ch < nch) {
        const char* src = (const char*)(row_ptr(row) + 128 * c) + ch * 16;
        __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(tile + c * 16384 + n * 1024), 16, 0, 0);
      }
    }
  }
}

// store 32-column block dt of a lane's accumulator row (column = 32dt + 8g + 4h + j) with scale; cols >= D skipped.
// Lanes i and i+32 hold the two halves of every 8-column group of the SAME row, so one v_permlane32_swap per dword
// pairs group g of both halves in lanes 0-31 and group g+1 in lanes 32-63: two 16-B stores per block instead of four
// 8-B ones (guide T21: the epilogue tail is store-issue bound). Both lanes of a pair always share the row (and hence
// the branch taken here and the caller's row-validity test), as the swap requires.
template <int D>
__device__ __forceinline__ void store_row_block(bf16* dst, const f32x16& acc, int dt, int h, float mul) {
#ifndef HDS_NARROW_STORES  // A/B switch (ops/build.py file_flags): the 8-B stores only
  if constexpr (D % 32 == 0) {
    if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0) {
      u32x2 w[4];
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v4;
#pragma unroll
        for (int j = 0; j < 4; ++j) v4[j] = (bf16)(acc[4 * g + j] * mul);
        w[g] = __builtin_bit_cast(u32x2, v4);
      }
#pragma unroll
      for (int k = 0; k < 4; k += 2) {
#pragma unroll
        for (int d = 0; d < 2; ++d) {
          const auto r = __builtin_amdgcn_permlane32_swap(w[k][d], w[k + 1][d], false, false);
          w[k][d] = r[0];
          w[k + 1][d] = r[1];
        }
        const u32x4 v = {w[k][0], w[k][1], w[k + 1][0], w[k + 1][1]};
        *reinterpret_cast<u32x4*>(dst + 32 * dt + 8 * k + 8 * h) = v;
      }
      return;
    }
  }
#endif
#pragma unroll
  for (int g = 0; g < 4; ++g) {
    const int col = 32 * dt + 8 * g + 4 * h;
    if (D % 32 == 0 || col < D) {
      bf16x4 v4;
#pragma unroll
      for (int j = 0; j < 4; ++j) v4[j] = (bf16)(acc[4 * g + j] * mul);
      *reinterpret_cast<bf16x4*>(dst + col) = v4;
    }
  }
}


}  // namespace attn
}  // namespace hds
