// Grouped (MoE) GEMM for gfx950: for every expert e, Y[o_e : o_{e+1}] = X[o_e : o_{e+1}] . W[e]^T
// with X [T, K] expert-contiguous rows (the permuted token order), W [E, N, K] (nn.Linear layout) and
// o = exclusive prefix of the per-expert row counts, kept ON THE DEVICE (no host sync on the routing).
//
// Reference parity: SURVEY.md §2.10 N15 / §2.11 K37 — the CUTLASS grouped MoE GEMM of
// inference/v2/kernels/cutlass_ops/moe_gemm (external libdeepspeedft). Not a translation: one launch covers
// every expert's ragged row block, no capacity padding (dropless), and the tile schedule is built on the GPU.
//
// Design (cdna_hip_programming.md §3/§5):
//   * a tiny planning kernel turns the device offsets into a tile list (expert, m0) and a tile count;
//     the GEMM grid is the host-side upper bound ceil(T/128)+E, blocks past the count exit at once;
//   * 128(N) x 128(tokens) block tile, BK = 128, 4 waves each owning a 64 x 64 quadrant = 2 x 2
//     v_mfma_f32_32x32x16_bf16 accumulators. Operand orientation D = W . X^T puts the token on the lane
//     and 4 consecutive output features in consecutive accumulator registers, so the epilogue writes
//     8-byte bf16x4 vectors of one output row;
//   * both operands are K-contiguous, staged by LDS-DMA (global_load_lds_dwordx4) into the XOR-swizzled
//     64 x 256 B tiles of attn_common.h (conflict-free ds_read_b128 A/B fragments), double-buffered:
//     the next K tile streams in while the current one feeds the MFMAs;
//   * blockIdx.x walks N tiles fastest so the (consecutively dispatched, XCD-round-robin) blocks of one
//     token tile share the X tile in L2 while W[e] streams.
#include "attn_common.h"

using namespace hds;
using namespace hds::attn;

namespace {

constexpr int BM = 128;  // tokens per block tile
constexpr int BN = 128;  // output features per block tile
constexpr int BK = 128;  // reduction depth per stage (one 256-byte bf16 row per tile row)

template <int TM>
__global__ __launch_bounds__(64) void gg_plan_kernel(const int* __restrict__ offs, int E, int T,
                                                     int* __restrict__ tile_e, int* __restrict__ tile_m,
                                                     int* __restrict__ n_tiles, int max_tiles) {
  // single wave: serial prefix over experts (E <= a few hundred), lanes fill each expert's tiles
  const int lane = threadIdx.x;
  int base = 0;
  for (int e = 0; e < E; ++e) {
    const int lo = min(max(offs[e], 0), T), hi = min(max(offs[e + 1], lo), T);  // never trust offsets
    const int t = (hi - lo + TM - 1) / TM;
    for (int i = lane; i < t; i += 64) {
      if (base + i < max_tiles) {
        tile_e[base + i] = e;
        tile_m[base + i] = i * TM;
      }
    }
    base += t;
  }
  if (lane == 0) *n_tiles = base < max_tiles ? base : max_tiles;
}

__global__ __launch_bounds__(256) void gg_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                 bf16* __restrict__ y, const int* __restrict__ offs,
                                                 const int* __restrict__ tile_e, const int* __restrict__ tile_m,
                                                 const int* __restrict__ n_tiles, int T, int N, int K, int ldy) {
  const int t = blockIdx.y;
  if (t >= *n_tiles) return;  // block-uniform exit before any barrier
  const int e = tile_e[t];
  const int m0 = tile_m[t];
  const int row0 = min(max(offs[e], 0), T);
  const int rows = min(max(offs[e + 1], row0), T) - row0;  // >= 1: the plan only emits tiles of non-empty experts
  const int n0 = blockIdx.x * BN;

  __shared__ __attribute__((aligned(16))) char smem[2 * 65536];
  // buffer b: W tile halves at [b*64K, +16K, ...], X tile halves at [b*64K + 32K, +16K]
  const bf16* wb = w + (int64_t)e * N * K + (int64_t)n0 * K;
  const bf16* xb = x + (int64_t)row0 * K;
  auto wrow = [&](int half, int kt) {
    return [=](int r) { return wb + (int64_t)(64 * half + r) * K + (int64_t)kt * BK; };
  };
  auto xrow = [&](int half, int kt) {
    return [=](int r) {
      int m = m0 + 64 * half + r;
      m = m < rows ? m : rows - 1;
      return xb + (int64_t)m * K + (int64_t)kt * BK;
    };
  };
  auto stage = [&](int buf, int kt) {
    char* s = smem + buf * 65536;
    stage_tile64<4>(s, wrow(0, kt));
    stage_tile64<4>(s + 16384, wrow(1, kt));
    stage_tile64<4>(s + 32768, xrow(0, kt));
    stage_tile64<4>(s + 49152, xrow(1, kt));
  };

  const int wv = threadIdx.x >> 6;
  const int wn = wv & 1, wm = wv >> 1;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  const int KT = K / BK;
  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) stage(buf ^ 1, kt + 1);
    const char* Wt = smem + buf * 65536 + wn * 16384;
    const char* Xt = smem + buf * 65536 + 32768 + wm * 16384;
#pragma unroll
    for (int ks = 0; ks < 8; ++ks) {
      const bf16x8 a0 = read_rows(Wt, 0, ks), a1 = read_rows(Wt, 32, ks);
      const bf16x8 b0 = read_rows(Xt, 0, ks), b1 = read_rows(Xt, 32, ks);
      acc[0][0] = mfma(a0, b0, acc[0][0]);
      acc[0][1] = mfma(a0, b1, acc[0][1]);
      acc[1][0] = mfma(a1, b0, acc[1][0]);
      acc[1][1] = mfma(a1, b1, acc[1][1]);
    }
    __syncthreads();
  }

  // epilogue: lane = token, registers 4g..4g+3 = 4 consecutive output features
  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = m0 + 64 * wm + 32 * j + (lane & 31);
    if (m >= rows) continue;
    bf16* yr = y + (int64_t)(row0 + m) * ldy + n0 + 64 * wn;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v;
#pragma unroll
        for (int q = 0; q < 4; ++q) v[q] = (bf16)acc[i][j][4 * g + q];
        *reinterpret_cast<bf16x4*>(yr + 32 * i + acc_row(4 * g, h)) = v;
      }
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Large-expert variant: 256 x 256 block tile, BK = 64, 8 waves (2 along N x 4 along tokens, 128 x 64 per wave =
// 4 x 2 accumulators). The per-wave tile halves the LDS bytes per MFMA of the 128^2 kernel (6 ds_read_b128 per
// 8 MFMA instead of 4 per 4), which is what bounds the small tile. LDS: two buffers of (256 + 256) rows x 128 B
// = 128 KB; rows of 128 B use the XOR swizzle chunk ^ ((row >> 1) & 7): a 16-lane ds_read_b128 group reading 16
// consecutive rows at one logical chunk hits 16 distinct 16-B bank slots (row & 1 selects the half of the
// 256-B bank line). Staging is LDS-DMA (lane-linear destination, swizzle applied to the source address).
// Blocks are remapped so each XCD works on a contiguous range of (token tile, N tile) pairs, rastered in groups of
// 4 token tiles so co-resident blocks share X and W panels in the same L2.
// ---------------------------------------------------------------------------------------------------------------
constexpr int BM2 = 256, BN2 = 256, BK2 = 64;

__device__ __forceinline__ int off128(int row, int ch) { return row * 128 + 16 * (ch ^ ((row >> 1) & 7)); }

// stage `rows` x 128 B (rows % 64 == 0) with an NW-wave block: one wave-instruction fills 8 rows
template <int NW, int ROWS, typename RowPtr>
__device__ __forceinline__ void stage128(char* lds, RowPtr row_ptr) {
  const int lane = threadIdx.x & 63;
  const int w = threadIdx.x >> 6;
  constexpr int PER = ROWS / 8 / NW;
#pragma unroll
  for (int i = 0; i < PER; ++i) {
    const int n = w * PER + i;
    const int row = 8 * n + (lane >> 3);
    const int ch = (lane & 7) ^ ((row >> 1) & 7);
    const char* src = (const char*)row_ptr(row) + ch * 16;
    __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(lds + n * 1024), 16, 0, 0);
  }
}

__device__ __forceinline__ bf16x8 frag128(const char* lds, int row0, int ks) {
  const int lane = threadIdx.x & 63;
  return *reinterpret_cast<const bf16x8*>(lds + off128(row0 + (lane & 31), 2 * ks + (lane >> 5)));
}

__global__ __launch_bounds__(512) void gg_big_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                     bf16* __restrict__ y, const int* __restrict__ offs,
                                                     const int* __restrict__ tile_e, const int* __restrict__ tile_m,
                                                     const int* __restrict__ n_tiles, int T, int N, int K, int ldy,
                                                     int ntn) {
  // XCD-contiguous remap of the 1-D grid (bijective for any size)
  const int nwg = gridDim.x, orig = blockIdx.x;
  const int q = nwg / 8, r = nwg % 8, xcd = orig % 8;
  const int id = (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
  // grouped raster: consecutive ids sweep GT token tiles before moving to the next N tile, so the ~32 blocks an
  // XCD runs at once cover a GT x (32/GT) rectangle and share both X and W K-slices in its L2
  constexpr int GT = 4;
  const int mt = gridDim.x / ntn;  // token-tile slots (host upper bound)
  const int grp = id / (GT * ntn), rem = id % (GT * ntn);
  const int gsz = min(GT, mt - grp * GT);
  const int t = grp * GT + rem % gsz;
  if (t >= *n_tiles) return;  // block-uniform exit before any barrier
  const int n0 = (rem / gsz) * BN2;
  const int e = tile_e[t];
  const int m0 = tile_m[t];
  const int row0 = min(max(offs[e], 0), T);
  const int rows = min(max(offs[e + 1], row0), T) - row0;

  __shared__ __attribute__((aligned(16))) char smem[2 * 65536];  // [buf][W 32 KB | X 32 KB]
  const bf16* wb = w + (int64_t)e * N * K + (int64_t)n0 * K;
  const bf16* xb = x + (int64_t)row0 * K;
  auto stage = [&](int buf, int kt) {
    char* s = smem + buf * 65536;
    const int64_t k0 = (int64_t)kt * BK2;
    stage128<8, 256>(s, [=](int rr) { return wb + (int64_t)rr * K + k0; });
    stage128<8, 256>(s + 32768, [=](int rr) {
      int m = m0 + rr;
      m = m < rows ? m : rows - 1;
      return xb + (int64_t)m * K + k0;
    });
  };

  const int wv = threadIdx.x >> 6;
  const int wn = wv & 1, wm = wv >> 1;  // 128 features x 64 tokens per wave
  f32x16 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = f32x16{};

  const int KT = K / BK2;
  stage(0, 0);
  __syncthreads();
  for (int kt = 0; kt < KT; ++kt) {
    const int buf = kt & 1;
    if (kt + 1 < KT) stage(buf ^ 1, kt + 1);
    const char* Wt = smem + buf * 65536 + wn * 128 * 128;
    const char* Xt = smem + buf * 65536 + 32768 + wm * 64 * 128;
#pragma unroll
    for (int ks = 0; ks < 4; ++ks) {
      bf16x8 a[4], b[2];
#pragma unroll
      for (int i = 0; i < 4; ++i) a[i] = frag128(Wt, 32 * i, ks);
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = frag128(Xt, 32 * j, ks);
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = mfma(a[i], b[j], acc[i][j]);
    }
    __syncthreads();
  }

  const int lane = threadIdx.x & 63;
  const int h = lane >> 5;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int m = m0 + 64 * wm + 32 * j + (lane & 31);
    if (m >= rows) continue;
    bf16* yr = y + (int64_t)(row0 + m) * ldy + n0 + 128 * wn;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v;
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) v[qq] = (bf16)acc[i][j][4 * g + qq];
        *reinterpret_cast<bf16x4*>(yr + 32 * i + acc_row(4 * g, h)) = v;
      }
  }
}

}  // namespace

// Upper bound of the tile count for T rows over E experts (host-side grid size / scratch sizing).
HDS_EXPORT int hds_grouped_gemm_max_tiles(int T, int E) { return (T + BM - 1) / BM + E; }

// Y [T, ldy>=N] = per-expert X . W[e]^T.  x [T, K], w [E, N, K], offs [E+1] (device, int32),
// work = int32 scratch of 2*hds_grouped_gemm_max_tiles(T, E) + 1 elements. Requires N % 128 == 0, K % 128 == 0.
// variant: 0 = auto (256^2 tiles when N % 256 == 0 and the average expert has >= 256 rows), 1 = 128^2, 2 = 256^2.
HDS_EXPORT int hds_grouped_gemm(const void* x, const void* w, void* y, const int* offs, int* work, int T, int N, int K,
                                int E, int ldy, int variant, hipStream_t st) {
  if (T <= 0 || E <= 0) return 0;
  if (N % BN || K % BK || ldy < N || ldy % 8) return hipErrorInvalidValue;
  bool big = variant == 2 || (variant == 0 && N % BN2 == 0 && T >= BM2 * E);
  if (big && N % BN2) return hipErrorInvalidValue;
  const int cap = hds_grouped_gemm_max_tiles(T, E);
  int* tile_e = work;
  int* tile_m = work + cap;
  int* n_tiles = work + 2 * cap;
  if (big) {
    const int max_tiles = (T + BM2 - 1) / BM2 + E;  // <= cap
    const int ntn = N / BN2;
    hipLaunchKernelGGL(gg_plan_kernel<BM2>, dim3(1), dim3(64), 0, st, offs, E, T, tile_e, tile_m, n_tiles, max_tiles);
    hipLaunchKernelGGL(gg_big_kernel, dim3(ntn * max_tiles), dim3(512), 0, st, (const bf16*)x, (const bf16*)w,
                       (bf16*)y, offs, tile_e, tile_m, n_tiles, T, N, K, ldy, ntn);
  } else {
    hipLaunchKernelGGL(gg_plan_kernel<BM>, dim3(1), dim3(64), 0, st, offs, E, T, tile_e, tile_m, n_tiles, cap);
    hipLaunchKernelGGL(gg_kernel, dim3(N / BN, cap), dim3(256), 0, st, (const bf16*)x, (const bf16*)w, (bf16*)y,
                       offs, tile_e, tile_m, n_tiles, T, N, K, ldy);
  }
  return hipGetLastError();
}
