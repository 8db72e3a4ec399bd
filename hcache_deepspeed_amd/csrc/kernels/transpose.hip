// 2-D bf16 transpose dst[c][r] = src[r][c] (src row stride lds elements, dst contiguous [cols, rows]).
// Used to put weight-gradient GEMMs dW = dY^T X into hipBLASLt's fast NT layout (ops/gemm.py wgrad): the transposed
// copies are written once at HBM rate instead of the TN GEMM running ~25 % below the NT one at the bench shapes.
// Tile 64 x 64 through LDS: 16-B global loads along src rows, 16-B global stores along dst rows; the LDS tile is
// padded to 66 elements per row so the column reads of the store phase spread over the banks.
#include "hds_common.h"

namespace {
using namespace hds;

constexpr int TT = 64, PAD = 66;

__global__ __launch_bounds__(256) void transpose_bf16_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                             int rows, int cols, int64_t lds) {
  __shared__ bf16 tile[TT * PAD];
  const int r0 = blockIdx.y * TT, c0 = blockIdx.x * TT;
  const int tid = threadIdx.x;
  // load: 64 rows x 8 vectors of 8 -> 512 vectors, 2 per thread
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + 256 * i, rr = v >> 3, cc = (v & 7) * 8;
    const int r = r0 + rr, c = c0 + cc;
    bf16x8 x;
    if (r < rows && c + 7 < cols) {
      x = *reinterpret_cast<const bf16x8*>(src + (int64_t)r * lds + c);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (r < rows && c + j < cols) ? src[(int64_t)r * lds + c + j] : (bf16)0.f;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) tile[rr * PAD + cc + j] = x[j];
  }
  __syncthreads();
  // store: dst row = source column c0 + cr, 8 consecutive source rows per vector
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int v = tid + 256 * i, cr = v >> 3, rc = (v & 7) * 8;
    const int c = c0 + cr, r = r0 + rc;
    if (c >= cols) continue;
    bf16x8 y;
#pragma unroll
    for (int j = 0; j < 8; ++j) y[j] = tile[(rc + j) * PAD + cr];
    if (r + 7 < rows) {
      *reinterpret_cast<bf16x8*>(dst + (int64_t)c * rows + r) = y;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j)
        if (r + j < rows) dst[(int64_t)c * rows + r + j] = y[j];
    }
  }
}

// v2 (default): tile 64 rows x 128 columns, 256 threads, every LDS access 8 or 16 B wide.
//   load : 16-B global loads along src rows (16 lanes = one 256-B row), one ds_write_b128 each -- a 16-lane group
//          writes a whole 256-B LDS row, conflict-free.
//   store: thread (lr = t / 32, lc = t % 32) owns the 8 x 4 block rows 8lr..8lr+7, columns 4lc..4lc+3: eight
//          ds_read_b64 (a half-wave reads the 32 8-B granules of one LDS row -> all 64 banks), 16 v_perm_b32 pack the
//          four transposed 8-element vectors, four 16-B stores to dst rows c0 + 4lc + i.
// v1's LDS traffic was one 2-B write and one 2-B read per element (32 LDS instructions per thread per 16 B moved).
constexpr int TR = 64, TC = 128;

__global__ __launch_bounds__(256) void transpose_bf16_v2_kernel(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                                int rows, int cols, int64_t lds) {
  __shared__ __attribute__((aligned(16))) bf16 tile[TR * TC];
  const int r0 = blockIdx.y * TR, c0 = blockIdx.x * TC;
  const int tid = threadIdx.x;
  const bool full = (r0 + TR <= rows) && (c0 + TC <= cols);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int v = tid + 256 * i, rr = v >> 4, cc = (v & 15) * 8;
    const int r = r0 + rr, c = c0 + cc;
    bf16x8 x;
    if (full || (r < rows && c + 7 < cols)) {
      x = *reinterpret_cast<const bf16x8*>(src + (int64_t)r * lds + c);
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) x[j] = (r < rows && c + j < cols) ? src[(int64_t)r * lds + c + j] : (bf16)0.f;
    }
    *reinterpret_cast<bf16x8*>(&tile[rr * TC + cc]) = x;
  }
  __syncthreads();
  const int lr = tid >> 5, lc = tid & 31;
  u32x2 v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = *reinterpret_cast<const u32x2*>(&tile[(8 * lr + j) * TC + 4 * lc]);
  const int r = r0 + 8 * lr;
  if (r >= rows) return;  // rows % 8 == 0: a block row is all in or all out
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int c = c0 + 4 * lc + i;
    if (!full && c >= cols) break;
    // element i of row j sits in dword i/2 of v[j], low half for even i; pack rows (2k, 2k+1) into word k
    const uint32_t sel = (i & 1) ? 0x07060302u : 0x05040100u;
    u32x4 y;
#pragma unroll
    for (int k = 0; k < 4; ++k) y[k] = __builtin_amdgcn_perm(v[2 * k + 1][i >> 1], v[2 * k][i >> 1], sel);
    *reinterpret_cast<u32x4*>(dst + (int64_t)c * rows + r) = y;
  }
}

}  // namespace

// rows % 8 == 0 and lds % 8 == 0 keep the vector accesses aligned (checked by the caller)
// variant 1: 64 x 64 tile, 2-B LDS accesses; variant 2 (default): 64 x 128 tile, 16-B writes / 8-B reads + v_perm
HDS_EXPORT int hds_transpose_bf16_var(const void* src, void* dst, int rows, int cols, long lds, int variant,
                                      hipStream_t st) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  if (rows % 8 || lds % 8 || ((uintptr_t)src & 15) || ((uintptr_t)dst & 15)) return hipErrorInvalidValue;
  if (variant == 1) {
    dim3 grid((cols + TT - 1) / TT, (rows + TT - 1) / TT);
    hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, st, (const bf16*)src, (bf16*)dst, rows, cols,
                       (int64_t)lds);
  } else {
    dim3 grid((cols + TC - 1) / TC, (rows + TR - 1) / TR);
    hipLaunchKernelGGL(transpose_bf16_v2_kernel, grid, dim3(256), 0, st, (const bf16*)src, (bf16*)dst, rows, cols,
                       (int64_t)lds);
  }
  return hipGetLastError();
}

HDS_EXPORT int hds_transpose_bf16(const void* src, void* dst, int rows, int cols, long lds, hipStream_t st) {
  return hds_transpose_bf16_var(src, dst, rows, cols, lds, 2, st);
}
