// Dense bf16 GEMM on the CDNA4 matrix cores for the projection shapes of transformer training:
//   C[M, N] (+)= alpha * A[M, K] . B[N, K]^T       (A = activations, B = nn.Linear weight [out, in])
//
// Why a hand-written kernel next to hipBLASLt: at the Llama-3-8B forward shapes (M = 28672 tokens, K = 4096 /
// 14336) the library's heuristic tiles run at ~1.1 PF/s (profiles/rocprof_kernel_stats_r2_wgrad.csv); the
// structure below is built for one 256 x 256 tile per CU with the operand stream fully overlapped.
//
// Structure (guide §5 "256^2 8-phase template", rebuilt here around a 4-phase-per-K-tile schedule):
//   * 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns a 128 x 64 block of C = 8 x 4 tiles of
//     v_mfma_f32_16x16x32_bf16 (128 accumulator registers).
//   * BK = 64. LDS holds two K-tiles (2 x 64 KiB). Each K-tile is stored as four 16 KiB HALF-TILES:
//       A0 = tile rows {0-63, 128-191}, A1 = rows {64-127, 192-255}, B0 = columns {0-31, 64-95, ...} (32 of every
//       64), B1 = the other columns -- so that a wave's output QUADRANT (64 rows x 32 columns) reads exactly one A
//       half and one B half.
//   * A K-tile is consumed in 4 phases, one quadrant each (16 MFMAs): q0 = (A0, B0), q1 = (A0, B1),
//     q2 = (A1, B1), q3 = (A1, B0); fragments stay in registers between phases, so q0 reads A0 + B0, q1 reads
//     B1, q2 reads A1 and q3 reads nothing from LDS.
//   * A half-tile's LDS region is free one phase after its read, so the NEXT-but-one K-tile is restaged into it
//     right away (one half-tile = 2 LDS-DMA instructions per thread per phase): each half-tile gets 6-7 phases
//     of flight time, and a uniform counted `s_waitcnt vmcnt(10)` (5 half-tiles left in flight) before every
//     phase barrier retires exactly what the next phase reads. Barriers are raw s_barrier (no vmcnt(0) drain).
//   * LDS-DMA writes lane-linearly, so the bank-conflict XOR swizzle (16-B chunk c of row r stored at
//     c ^ ((r >> 1) & 7)) is applied to the per-lane GLOBAL source address and to the ds_read address (rule 21).
//     A 16-lane ds_read_b128 group then covers all 16 slots of the 256-B bank row.
//   * The MFMAs take the B (weight) fragment as their first operand, so the accumulator lane holds 4 consecutive
//     COLUMNS of one row of C: the epilogue stores 8 B per lane per tile, row-contiguous.
//   * Workgroup ids are remapped bijectively so the blocks that run on one XCD (hardware round-robin b % 8) form
//     a contiguous run of 8-row-tile groups and share A rows / B columns in that XCD's L2 (T1).
// Requirements (checked by the launcher): M % 256 == 0, N % 256 == 0, K % 128 == 0, rows 16-B aligned.
#include "hds_common.h"

using namespace hds;

namespace {

typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

constexpr int kHalf = 16384;     // bytes of one half-tile (128 rows x 64 bf16)
constexpr int kBuf = 4 * kHalf;  // one K-tile: A0 A1 B0 B1

struct GemmArgs {
  const bf16* A;
  const bf16* B;
  bf16* C;
  int M, N, K;
  int lda, ldb, ldc;
  float alpha;
  int accumulate;
};

__device__ __forceinline__ void vm_wait10() { asm volatile("s_waitcnt vmcnt(10)" ::: "memory"); }
__device__ __forceinline__ void vm_wait0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, const f32x4& c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// One half-tile (128 rows x 128 B) by LDS-DMA: thread (w, lane) moves pieces 2w and 2w+1 (8 rows each).
// src[i] already points at this lane's 16-B chunk of its row for K-tile 0; `koff` is the K-tile's element offset.
__device__ __forceinline__ void stage_half(char* dst_half, const bf16* const (&src)[2], long koff, int w) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    char* d = dst_half + (2 * w + i) * 1024;
    __builtin_amdgcn_global_load_lds((gbl_void*)(src[i] + koff), (lds_void*)d, 16, 0, 0);
  }
}

template <int Q>
__device__ __forceinline__ void read_frags(const char* buf, int lane_off0, int lane_off1, int wr, int wc,
                                           bf16x8 (&a)[2][4], bf16x8 (&b)[2][2][2]) {
  // q0: A0 + B0, q1: B1, q2: A1, q3: nothing
  if constexpr (Q == 0 || Q == 2) {
    const char* h = buf + (Q == 0 ? 0 : kHalf) + wr * 64 * 128;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[0][i] = *reinterpret_cast<const bf16x8*>(h + i * 16 * 128 + lane_off0);
      a[1][i] = *reinterpret_cast<const bf16x8*>(h + i * 16 * 128 + lane_off1);
    }
  }
  if constexpr (Q == 0 || Q == 1) {
    constexpr int nh = Q == 0 ? 0 : 1;
    const char* h = buf + 2 * kHalf + nh * kHalf + wc * 32 * 128;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      b[nh][0][j] = *reinterpret_cast<const bf16x8*>(h + j * 16 * 128 + lane_off0);
      b[nh][1][j] = *reinterpret_cast<const bf16x8*>(h + j * 16 * 128 + lane_off1);
    }
  }
}

template <int Q>
__device__ __forceinline__ void mfma_quadrant(const bf16x8 (&a)[2][4], const bf16x8 (&b)[2][2][2],
                                              f32x4 (&acc)[8][4]) {
  constexpr int mh = (Q == 0 || Q == 1) ? 0 : 1;
  constexpr int nh = (Q == 0 || Q == 3) ? 0 : 1;
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int ks = 0; ks < 2; ++ks)
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 2; ++j)
        acc[mh * 4 + i][nh * 2 + j] = mfma16(b[nh][ks][j], a[ks][i], acc[mh * 4 + i][nh * 2 + j]);
  __builtin_amdgcn_s_setprio(0);
}

__device__ __forceinline__ void lgkm_wait0() { asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory"); }

// Phase tail. Plain schedule (STG = false): one barrier per phase, every wave waits vmcnt(10) before it.
// Staggered schedule (STG = true, guide MI355X_MICROARCH "Two waves per SIMD" item 9): waves 4-7 run one barrier
// behind waves 0-3, so on every SIMD one wave's MFMA cluster runs beside its partner's LDS reads + DMA issue.
// Each phase is then READ | barrier | MFMA | barrier; the reads are retired (lgkmcnt 0) before the first barrier
// (a region is restaged one phase after its last read), waves 0-3 retire their DMA (vmcnt 10) before the second
// barrier and waves 4-7 before the first -- in both cases the barrier that precedes the other group's next reads.
template <bool STG>
__device__ __forceinline__ void after_reads(bool steady, int wr) {
  if constexpr (STG) {
    if (wr == 1) {
      if (steady) vm_wait10(); else vm_wait0();
    }
    lgkm_wait0();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  }
}

template <bool STG>
__device__ __forceinline__ void after_mfma(bool steady, int wr) {
  if (!STG || wr == 0) {
    if (steady) vm_wait10(); else vm_wait0();
  }
  __builtin_amdgcn_s_barrier();
}

// One K-tile (4 phases) reading LDS buffer CUR; stages A1(t+1) into the other buffer and A0/B0/B1(t+2) into CUR.
template <int CUR, bool STG>
__device__ __forceinline__ void k_tile(char* smem, int t, int nt, const bf16* const (&sa0)[2],
                                       const bf16* const (&sa1)[2], const bf16* const (&sb0)[2],
                                       const bf16* const (&sb1)[2], int w, int wr, int wc, int lane_off0,
                                       int lane_off1, bf16x8 (&a)[2][4], bf16x8 (&b)[2][2][2], f32x4 (&acc)[8][4]) {
  char* cur = smem + CUR * kBuf;
  char* nxt = smem + (CUR ^ 1) * kBuf;
  const bool steady = t + 2 < nt;
  // q0
  read_frags<0>(cur, lane_off0, lane_off1, wr, wc, a, b);
  if (t + 1 < nt) stage_half(nxt + kHalf, sa1, (long)(t + 1) * 64, w);
  after_reads<STG>(steady, wr);
  mfma_quadrant<0>(a, b, acc);
  after_mfma<STG>(steady, wr);
  // q1
  read_frags<1>(cur, lane_off0, lane_off1, wr, wc, a, b);
  if (steady) stage_half(cur, sa0, (long)(t + 2) * 64, w);
  after_reads<STG>(steady, wr);
  mfma_quadrant<1>(a, b, acc);
  after_mfma<STG>(steady, wr);
  // q2
  read_frags<2>(cur, lane_off0, lane_off1, wr, wc, a, b);
  if (steady) stage_half(cur + 2 * kHalf, sb0, (long)(t + 2) * 64, w);
  after_reads<STG>(steady, wr);
  mfma_quadrant<2>(a, b, acc);
  after_mfma<STG>(steady, wr);
  // q3
  if (steady) stage_half(cur + 3 * kHalf, sb1, (long)(t + 2) * 64, w);
  after_reads<STG>(steady, wr);
  mfma_quadrant<3>(a, b, acc);
  after_mfma<STG>(steady, wr);
}

template <bool ACC>
__device__ __forceinline__ void store_c(const GemmArgs& p, const f32x4 (&acc)[8][4], long m0, long n0, int wr, int wc,
                                        int lane) {
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const long row = m0 + wr * 128 + (i >> 2) * 64 + (i & 3) * 16 + (lane & 15);
    bf16* crow = p.C + row * p.ldc + n0 + wc * 64 + 4 * (lane >> 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16* dst = crow + (j >> 1) * 32 + (j & 1) * 16;
      f32x4 v = acc[i][j] * p.alpha;
      if constexpr (ACC) {
        const bf16x4 old = *reinterpret_cast<const bf16x4*>(dst);
        v[0] += (float)old[0];
        v[1] += (float)old[1];
        v[2] += (float)old[2];
        v[3] += (float)old[3];
      }
      bf16x4 o;
      o[0] = (bf16)v[0];
      o[1] = (bf16)v[1];
      o[2] = (bf16)v[2];
      o[3] = (bf16)v[3];
      *reinterpret_cast<bf16x4*>(dst) = o;
    }
  }
}

template <bool STG>
__global__ __launch_bounds__(512) void gemm_nt_kernel(GemmArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 2, wc = w & 3;

  // ---- bijective XCD remap, then 8-row-tile groups walked column-major ----
  const int tiles_m = p.M / 256, tiles_n = p.N / 256;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  constexpr int GM = 8;
  const int group = lid / (GM * tiles_n);
  const int first_m = group * GM;
  const int gm = min(tiles_m - first_m, GM);
  const int in_group = lid - group * GM * tiles_n;
  const int tm = first_m + in_group % gm;
  const int tn = in_group / gm;
  const long m0 = (long)tm * 256, n0 = (long)tn * 256;

  // ---- per-lane LDS-DMA sources (rows of piece 2w+i: rr = 16w + 8i + lane/8, chunk lane%8, swizzled) ----
  const bf16* sa0[2];
  const bf16* sa1[2];
  const bf16* sb0[2];
  const bf16* sb1[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rr = 16 * w + 8 * i + (lane >> 3);
    const int ch = (lane & 7) ^ ((rr >> 1) & 7);
    const long arow = m0 + (rr >> 6) * 128 + (rr & 63);
    const long brow = n0 + (rr >> 5) * 64 + (rr & 31);
    sa0[i] = p.A + arow * p.lda + ch * 8;
    sa1[i] = sa0[i] + 64L * p.lda;
    sb0[i] = p.B + brow * p.ldb + ch * 8;
    sb1[i] = sb0[i] + 32L * p.ldb;
  }
  // ---- per-lane fragment offsets inside a half-tile (row lane%16, chunk 4ks + lane/16, swizzled) ----
  const int sw = (lane >> 1) & 7;
  const int lane_off0 = (lane & 15) * 128 + 16 * ((0 + (lane >> 4)) ^ sw);
  const int lane_off1 = (lane & 15) * 128 + 16 * ((4 + (lane >> 4)) ^ sw);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 a[2][4];
  bf16x8 b[2][2][2];

  const int nt = p.K / 64;  // even (K % 128 == 0)
  // prologue: the stagings of phases -7 .. -1
  stage_half(smem + 0 * kHalf, sa0, 0, w);
  stage_half(smem + 2 * kHalf, sb0, 0, w);
  stage_half(smem + 3 * kHalf, sb1, 0, w);
  stage_half(smem + 1 * kHalf, sa1, 0, w);
  stage_half(smem + kBuf + 0 * kHalf, sa0, 64, w);
  stage_half(smem + kBuf + 2 * kHalf, sb0, 64, w);
  stage_half(smem + kBuf + 3 * kHalf, sb1, 64, w);
  vm_wait10();
  __builtin_amdgcn_s_barrier();
  if (STG && wr == 1) __builtin_amdgcn_s_barrier();  // waves 4-7 start one barrier behind

  for (int t = 0; t < nt; t += 2) {
    k_tile<0, STG>(smem, t, nt, sa0, sa1, sb0, sb1, w, wr, wc, lane_off0, lane_off1, a, b, acc);
    k_tile<1, STG>(smem, t + 1, nt, sa0, sa1, sb0, sb1, w, wr, wc, lane_off0, lane_off1, a, b, acc);
  }
  if (STG && wr == 0) __builtin_amdgcn_s_barrier();  // rejoin

  // ---- epilogue: lane holds C[row = m-tile row + lane%16][4 consecutive columns from 4*(lane/16)] ----
  if (p.accumulate)
    store_c<true>(p, acc, m0, n0, wr, wc, lane);
  else
    store_c<false>(p, acc, m0, n0, wr, wc, lane);
}

// =====================================================================================================
// MX-FP8 (OCP e4m3 elements, one e8m0 scale per 32 elements along K) GEMM on the block-scaled matrix core op
// v_mfma_scale_f32_16x16x128_f8f6f4 (2x the bf16 MFMA rate per clock):
//   C[M, N] = alpha * dequant(A)[M, K] . dequant(B)[N, K]^T,  bf16 out.
// Same tile / wave / half-tile structure as the bf16 kernel: a 128-element fp8 K-tile row is 128 B, exactly a
// bf16 64-element row, so staging and fragment reads are byte-identical (a lane's fragment is 16-B chunks g and
// g + 4 of its row, g = lane / 16 -- see the operand-order note in the kernel) and one MFMA covers the tile's K.
// Scales: tile-major [K/128][rows][4] bytes (the 4 K-blocks of a row for one K-tile form one dword, and the 256
// rows of a tile one contiguous KiB), staged per K-tile into a 2 KiB LDS region (SA | SB) by 8 single-dword
// LDS-DMA instructions (one per wave); each lane reads its (row, K-block) byte with ds_read_u8 and hands it to
// the MFMA's scale operand (OPSEL 0).
// Schedule per K-tile t (buffer CUR): q0 stages B0 + S of tile t+1 into the other buffer, q1..q3 stage A0, B1, A1
// of tile t+2 into CUR (each region one phase after its last read); ONE counted vmcnt(6) per K-tile, before the
// last phase barrier, retires everything the next K-tile reads (the S of tile t+1 is the newest of those; A0 / B1
// / A1 of tile t+1 had 7 phases of flight).
// =====================================================================================================
constexpr int kSBytes = 2048;            // SA (256 x 4 B) + SB (256 x 4 B)
constexpr int kBuf8 = 4 * kHalf + kSBytes;

typedef int i32x8 __attribute__((ext_vector_type(8)));
typedef int i32x4v __attribute__((ext_vector_type(4)));

struct MxArgs {
  const uint8_t* A;
  const uint8_t* B;
  const uint8_t* SA;  // [K/128][M][4]
  const uint8_t* SB;  // [K/128][N][4]
  bf16* C;
  int M, N, K;
  int lda, ldb, ldc;
  float alpha;
};

__device__ __forceinline__ void vm_wait6() { asm volatile("s_waitcnt vmcnt(6)" ::: "memory"); }

// 32-bit per-lane offsets on a wave-uniform base: the DMA uses the SGPR-base + VGPR-offset addressing form, one
// VGPR per source instead of a 64-bit pointer (the fp8 kernel needs the registers for its scale operands).
__device__ __forceinline__ void stage_half8(char* dst_half, const uint8_t* base, const uint32_t (&off)[2], int w) {
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    char* d = dst_half + (2 * w + i) * 1024;
    __builtin_amdgcn_global_load_lds((gbl_void*)(base + off[i]), (lds_void*)d, 16, 0, 0);
  }
}

// wave w < 4: SA rows 64w..64w+63; w >= 4: SB rows 64(w-4).. ; lane -> one row's dword
__device__ __forceinline__ void stage_scales(char* dst_s, const uint8_t* ssrc, long toff, int w) {
  char* d = dst_s + w * 256;
  __builtin_amdgcn_global_load_lds((gbl_void*)(ssrc + toff), (lds_void*)d, 4, 0, 0);
}

__device__ __forceinline__ i32x8 ld_frag8(const char* p0, const char* p1) {
  const i32x4v l = *reinterpret_cast<const i32x4v*>(p0);
  const i32x4v h = *reinterpret_cast<const i32x4v*>(p1);
  return __builtin_shufflevector(l, h, 0, 1, 2, 3, 4, 5, 6, 7);
}

// q0: A0 + B0, q1: B1, q2: A1, q3: B0 again (only the current B half is kept in registers: the fp8 kernel's
// scale operands need the 16 VGPRs that a second B half would take)
template <int Q>
__device__ __forceinline__ void read_frags8(const char* buf, int lane_off0, int lane_off1, int wr, int wc,
                                            i32x8 (&a)[4], i32x8 (&b)[2]) {
  if constexpr (Q == 0 || Q == 2) {
    const char* h = buf + (Q == 0 ? 0 : kHalf) + wr * 64 * 128;
#pragma unroll
    for (int i = 0; i < 4; ++i) a[i] = ld_frag8(h + i * 16 * 128 + lane_off0, h + i * 16 * 128 + lane_off1);
  }
  if constexpr (Q != 2) {
    constexpr int nh = Q == 1 ? 1 : 0;
    const char* h = buf + 2 * kHalf + nh * kHalf + wc * 32 * 128;
#pragma unroll
    for (int j = 0; j < 2; ++j) b[j] = ld_frag8(h + j * 16 * 128 + lane_off0, h + j * 16 * 128 + lane_off1);
  }
}

template <int Q>
__device__ __forceinline__ void read_scales(const char* sbuf, int lane, int wr, int wc, int (&sa)[4], int (&sb)[2]) {
  const int g = lane >> 4, r = lane & 15;
  if constexpr (Q == 0 || Q == 2) {
    constexpr int mh = Q == 0 ? 0 : 1;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int row = wr * 128 + mh * 64 + i * 16 + r;
      sa[i] = *reinterpret_cast<const uint8_t*>(sbuf + row * 4 + g);
    }
  }
  if constexpr (Q != 2) {
    constexpr int nh = Q == 1 ? 1 : 0;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = wc * 64 + nh * 32 + j * 16 + r;
      sb[j] = *reinterpret_cast<const uint8_t*>(sbuf + 1024 + row * 4 + g);
    }
  }
}

template <int Q>
__device__ __forceinline__ void mfma_quadrant8(const i32x8 (&a)[4], const i32x8 (&b)[2], const int (&sa)[4],
                                               const int (&sb)[2], f32x4 (&acc)[8][4]) {
  constexpr int mh = (Q == 0 || Q == 1) ? 0 : 1;
  constexpr int nh = (Q == 0 || Q == 3) ? 0 : 1;
  // hipcc sinks these MFMAs (register-only ops) past the phase barriers and hoists every phase's fragment reads
  // above them -- all fragments live at once, 180+ VGPRs spilled. The scheduling fences pin the cluster.
  __builtin_amdgcn_sched_barrier(0);
  __builtin_amdgcn_s_setprio(1);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
      acc[mh * 4 + i][nh * 2 + j] = __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(
          b[j], a[i], acc[mh * 4 + i][nh * 2 + j], 0, 0, 0, sb[j], 0, sa[i]);
  __builtin_amdgcn_s_setprio(0);
  __builtin_amdgcn_sched_barrier(0);
}

// s_waitcnt vmcnt(6) only when `on` (wave-uniform) -- the branch lives inside the asm so the loop body stays ONE
// basic block: with real branches hipcc sinks the (register-only) MFMAs into the block after the last phase and
// hoists every phase's fragment reads above them, which spills ~200 VGPRs.
__device__ __forceinline__ void vm_wait6_if(int on) {
  asm volatile("s_cmp_eq_u32 %0, 0\n\ts_cbranch_scc1 1f\n\ts_waitcnt vmcnt(6)\n1:" ::"s"(on) : "memory", "scc");
}

// K-tile t reading buffer CUR. Region reuse: A0 is free after q0, B1 after q1, A1 after q2, B0 and S after q3, so
// q1..q3 restage A0, B1, A1 of tile t+2 into CUR and q0 restages B0 + S of tile t+1 into the other buffer. Past the
// last tile the stagings re-load the last tile (clamped) into regions nobody reads again, which keeps the vmcnt
// arithmetic uniform and the body branch-free.
template <int CUR, bool STG>
__device__ __forceinline__ void k_tile8(char* smem, int t, int nt, const MxArgs& p, const uint32_t (&oa)[2],
                                        const uint32_t (&ob)[2], long a1_off, long b1_off, const uint8_t* ssrc,
                                        long sstride, int w, int wr, int wc, int lane, int lane_off0, int lane_off1,
                                        i32x8 (&a)[4], i32x8 (&b)[2], int (&sa)[4], int (&sb)[2],
                                        f32x4 (&acc)[8][4]) {
  char* cur = smem + CUR * kBuf8;
  char* nxt = smem + (CUR ^ 1) * kBuf8;
  const long k1 = (long)min(t + 1, nt - 1) * 128, k2 = (long)min(t + 2, nt - 1) * 128;
  const long s1 = (long)min(t + 1, nt - 1) * sstride;
  // q0
  read_frags8<0>(cur, lane_off0, lane_off1, wr, wc, a, b);
  read_scales<0>(cur + 4 * kHalf, lane, wr, wc, sa, sb);
  stage_half8(nxt + 2 * kHalf, p.B + k1, ob, w);
  stage_scales(nxt + 4 * kHalf, ssrc, s1, w);
  if constexpr (STG) {
    lgkm_wait0();
    __builtin_amdgcn_s_barrier();
  }
  mfma_quadrant8<0>(a, b, sa, sb, acc);
  __builtin_amdgcn_s_barrier();
  // q1
  read_frags8<1>(cur, lane_off0, lane_off1, wr, wc, a, b);
  read_scales<1>(cur + 4 * kHalf, lane, wr, wc, sa, sb);
  stage_half8(cur, p.A + k2, oa, w);
  if constexpr (STG) {
    lgkm_wait0();
    __builtin_amdgcn_s_barrier();
  }
  mfma_quadrant8<1>(a, b, sa, sb, acc);
  __builtin_amdgcn_s_barrier();
  // q2
  read_frags8<2>(cur, lane_off0, lane_off1, wr, wc, a, b);
  read_scales<2>(cur + 4 * kHalf, lane, wr, wc, sa, sb);
  stage_half8(cur + 3 * kHalf, p.B + b1_off + k2, ob, w);
  if constexpr (STG) {
    lgkm_wait0();
    __builtin_amdgcn_s_barrier();
  }
  mfma_quadrant8<2>(a, b, sa, sb, acc);
  __builtin_amdgcn_s_barrier();
  // q3 (retire the next K-tile's data: waves 4-7 before the read barrier, waves 0-3 before the last one)
  read_frags8<3>(cur, lane_off0, lane_off1, wr, wc, a, b);
  read_scales<3>(cur + 4 * kHalf, lane, wr, wc, sa, sb);
  stage_half8(cur + kHalf, p.A + a1_off + k2, oa, w);
  if constexpr (STG) {
    vm_wait6_if(wr);
    lgkm_wait0();
    __builtin_amdgcn_s_barrier();
  }
  mfma_quadrant8<3>(a, b, sa, sb, acc);
  if constexpr (STG) vm_wait6_if(wr ^ 1); else vm_wait6();
  __builtin_amdgcn_s_barrier();
}

template <bool STG>
__global__ __launch_bounds__(512) void gemm_mxfp8_kernel(MxArgs p) {
  __shared__ __attribute__((aligned(16))) char smem[2 * kBuf8];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wr = w >> 2, wc = w & 3;

  const int tiles_m = p.M / 256, tiles_n = p.N / 256;
  const int nwg = tiles_m * tiles_n;
  const int bid = blockIdx.x;
  const int xcd = bid % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  constexpr int GM = 8;
  const int group = lid / (GM * tiles_n);
  const int first_m = group * GM;
  const int gm = min(tiles_m - first_m, GM);
  const int in_group = lid - group * GM * tiles_n;
  const int tm = first_m + in_group % gm;
  const int tn = in_group / gm;
  const long m0 = (long)tm * 256, n0 = (long)tn * 256;

  // per-lane 32-bit DMA offsets (A0 / B0 rows); A1 = +64 rows, B1 = +32 rows, K-tile t = +128 B (all uniform)
  uint32_t oa[2], ob[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int rr = 16 * w + 8 * i + (lane >> 3);
    const int ch = (lane & 7) ^ ((rr >> 1) & 7);
    const long arow = m0 + (rr >> 6) * 128 + (rr & 63);
    const long brow = n0 + (rr >> 5) * 64 + (rr & 31);
    oa[i] = (uint32_t)(arow * p.lda + ch * 16);
    ob[i] = (uint32_t)(brow * p.ldb + ch * 16);
  }
  const long a1_off = 64L * p.lda, b1_off = 32L * p.ldb;
  // scale source: waves 0-3 -> SA rows m0 + 64w + lane, waves 4-7 -> SB rows n0 + 64(w-4) + lane
  const uint8_t* ssrc = w < 4 ? p.SA + (m0 + 64 * w + lane) * 4 : p.SB + (n0 + 64 * (w - 4) + lane) * 4;
  const long sstride = (w < 4 ? (long)p.M : (long)p.N) * 4;  // bytes per K-tile in the tile-major scale layout

  // Operand K order of v_mfma_scale_f32_16x16x128 (measured with exact data, tools/debug_mx.py): lane group
  // g = lane / 16 holds K [16g, 16g+16) in bytes 0-15 and K [64+16g, 64+16g+16) in bytes 16-31, and its scale
  // operand is the scale of K-block g ([32g, 32g+32)). So the fragment is 16-B chunks g and g+4 of the row --
  // the same chunks as the bf16 kernel's two k-steps.
  const int sw = (lane >> 1) & 7;
  const int g = lane >> 4;
  const int lane_off0 = (lane & 15) * 128 + 16 * (g ^ sw);
  const int lane_off1 = (lane & 15) * 128 + 16 * ((g + 4) ^ sw);

  f32x4 acc[8][4];
#pragma unroll
  for (int i = 0; i < 8; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  i32x8 a[4];
  i32x8 b[2];
  int sa[4];
  int sb[2];

  const int nt = p.K / 128;  // even (K % 256 == 0)
  // prologue: tile 0 (A0 B0 B1 A1 S) into buffer 0, tile 1 (A0 B0 B1) into buffer 1 -- the stagings the loop
  // would have issued in tiles -2 / -1; S and A1 of tile 1 follow in tile 0's q0.
  stage_half8(smem + 0 * kHalf, p.A, oa, w);
  stage_half8(smem + 3 * kHalf, p.B + b1_off, ob, w);
  stage_half8(smem + 1 * kHalf, p.A + a1_off, oa, w);
  stage_half8(smem + 2 * kHalf, p.B, ob, w);
  stage_scales(smem + 4 * kHalf, ssrc, 0, w);
  stage_half8(smem + kBuf8 + 0 * kHalf, p.A + 128, oa, w);
  stage_half8(smem + kBuf8 + 3 * kHalf, p.B + b1_off + 128, ob, w);
  stage_half8(smem + kBuf8 + 1 * kHalf, p.A + a1_off + 128, oa, w);
  vm_wait6();
  __builtin_amdgcn_s_barrier();
  if (STG && wr == 1) __builtin_amdgcn_s_barrier();

  for (int t = 0; t < nt; t += 2) {
    k_tile8<0, STG>(smem, t, nt, p, oa, ob, a1_off, b1_off, ssrc, sstride, w, wr, wc, lane, lane_off0, lane_off1, a,
                    b, sa, sb, acc);
    k_tile8<1, STG>(smem, t + 1, nt, p, oa, ob, a1_off, b1_off, ssrc, sstride, w, wr, wc, lane, lane_off0, lane_off1,
                    a, b, sa, sb, acc);
  }
  if (STG && wr == 0) __builtin_amdgcn_s_barrier();
  vm_wait0();  // the clamped tail stagings

  GemmArgs o{nullptr, nullptr, p.C, p.M, p.N, p.K, p.lda, p.ldb, p.ldc, p.alpha, 0};
  store_c<false>(o, acc, m0, n0, wr, wc, lane);
}

// ---- bf16 -> MX-FP8 quantization: one thread per 32-element block -------------------------------------
// shared exponent e = floor(log2(amax)) - 8 (e4m3 emax), scale byte = e + 127 (e8m0), q = sat_e4m3(x * 2^-e)
__global__ __launch_bounds__(256) void mx_quant_kernel(const bf16* __restrict__ x, uint8_t* __restrict__ q,
                                                       uint8_t* __restrict__ s, long rows, int K, long ldx) {
  const long blk = (long)blockIdx.x * 256 + threadIdx.x;
  const int kb_per_row = K / 32;
  if (blk >= rows * kb_per_row) return;
  const long r = blk / kb_per_row;
  const int kb = (int)(blk - r * kb_per_row);
  const bf16* src = x + r * ldx + kb * 32;
  float v[32];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const bf16x8 u = *reinterpret_cast<const bf16x8*>(src + 8 * c);
#pragma unroll
    for (int e = 0; e < 8; ++e) v[8 * c + e] = (float)u[e];
  }
  float amax = 0.f;
#pragma unroll
  for (int e = 0; e < 32; ++e) amax = fmaxf(amax, fabsf(v[e]));
  int ex = amax > 0.f ? (int)floorf(log2f(amax)) - 8 : -127;
  ex = ex < -127 ? -127 : (ex > 127 ? 127 : ex);
  const float inv = exp2f((float)-ex);
  int words[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) {
    float f[4];
#pragma unroll
    for (int e = 0; e < 4; ++e) f[e] = fminf(fmaxf(v[4 * c + e] * inv, -448.f), 448.f);
    int wv = __builtin_amdgcn_cvt_pk_fp8_f32(f[0], f[1], 0, false);
    words[c] = __builtin_amdgcn_cvt_pk_fp8_f32(f[2], f[3], wv, true);
  }
  uint8_t* dst = q + r * (long)K + kb * 32;
  *reinterpret_cast<i32x4v*>(dst) = i32x4v{words[0], words[1], words[2], words[3]};
  *reinterpret_cast<i32x4v*>(dst + 16) = i32x4v{words[4], words[5], words[6], words[7]};
  s[((long)(kb >> 2) * rows + r) * 4 + (kb & 3)] = (uint8_t)(ex + 127);
}

}  // namespace

HDS_EXPORT int hds_gemm_nt_supported(int M, int N, int K, int lda, int ldb, int ldc) {
  return M > 0 && N > 0 && K > 0 && M % 256 == 0 && N % 256 == 0 && K % 128 == 0 && lda % 8 == 0 &&
         ldb % 8 == 0 && ldc % 4 == 0 && lda >= K && ldb >= K && ldc >= N;
}

// C[M, N] (+)= alpha * A[M, K] . B[N, K]^T, all bf16, row-major with leading dimensions lda / ldb / ldc.
HDS_EXPORT int hds_gemm_nt(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                           float alpha, int accumulate, int variant, hipStream_t st) {
  if (!hds_gemm_nt_supported(M, N, K, lda, ldb, ldc)) return (int)hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B) & 15 || (uintptr_t)C & 7) return (int)hipErrorInvalidValue;
  GemmArgs p{(const bf16*)A, (const bf16*)B, (bf16*)C, M, N, K, lda, ldb, ldc, alpha, accumulate};
  const long nwg = (long)(M / 256) * (N / 256);
  if (nwg > 0x7fffffff) return (int)hipErrorInvalidValue;
  if (variant == 1)
    hipLaunchKernelGGL(gemm_nt_kernel<true>, dim3((unsigned)nwg), dim3(512), 0, st, p);
  else
    hipLaunchKernelGGL(gemm_nt_kernel<false>, dim3((unsigned)nwg), dim3(512), 0, st, p);
  return (int)hipGetLastError();
}

HDS_EXPORT int hds_gemm_mxfp8_supported(int M, int N, int K, int lda, int ldb, int ldc) {
  return M > 0 && N > 0 && K > 0 && M % 256 == 0 && N % 256 == 0 && K % 256 == 0 && lda % 16 == 0 &&
         ldb % 16 == 0 && ldc % 4 == 0 && lda >= K && ldb >= K && ldc >= N;
}

// C[M, N] = alpha * A . B^T with MX-FP8 operands (A [M, K] / B [N, K] e4m3 bytes, scales [K/128][rows][4] e8m0).
HDS_EXPORT int hds_gemm_mxfp8(const void* A, const void* SA, const void* B, const void* SB, void* C, int M, int N,
                              int K, int lda, int ldb, int ldc, float alpha, int variant, hipStream_t st) {
  if (!hds_gemm_mxfp8_supported(M, N, K, lda, ldb, ldc)) return (int)hipErrorInvalidValue;
  if (((uintptr_t)A | (uintptr_t)B) & 15 || ((uintptr_t)SA | (uintptr_t)SB) & 3 || (uintptr_t)C & 7)
    return (int)hipErrorInvalidValue;
  MxArgs p{(const uint8_t*)A, (const uint8_t*)B, (const uint8_t*)SA, (const uint8_t*)SB, (bf16*)C, M, N, K,
           lda, ldb, ldc, alpha};
  const long nwg = (long)(M / 256) * (N / 256);
  if (nwg > 0x7fffffff) return (int)hipErrorInvalidValue;
  if (variant == 1)
    hipLaunchKernelGGL(gemm_mxfp8_kernel<true>, dim3((unsigned)nwg), dim3(512), 0, st, p);
  else
    hipLaunchKernelGGL(gemm_mxfp8_kernel<false>, dim3((unsigned)nwg), dim3(512), 0, st, p);
  return (int)hipGetLastError();
}

// bf16 [rows, K] (row stride ldx) -> e4m3 bytes [rows, K] + e8m0 scales [K/128][rows][4]; K % 128 == 0.
HDS_EXPORT int hds_mx_quant(const void* x, void* q, void* s, long rows, int K, long ldx, hipStream_t st) {
  if (rows <= 0 || K <= 0 || K % 128 || ldx % 8 || ((uintptr_t)x & 15) || ((uintptr_t)q & 15))
    return (int)hipErrorInvalidValue;
  const long blocks = rows * (K / 32);
  const long grid = (blocks + 255) / 256;
  if (grid > 0x7fffffff) return (int)hipErrorInvalidValue;
  hipLaunchKernelGGL(mx_quant_kernel, dim3((unsigned)grid), dim3(256), 0, st, (const bf16*)x, (uint8_t*)q,
                     (uint8_t*)s, rows, K, ldx);
  return (int)hipGetLastError();
}
