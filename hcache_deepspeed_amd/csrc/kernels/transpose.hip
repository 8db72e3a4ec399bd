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

}  // namespace

// rows % 8 == 0 and lds % 8 == 0 keep the vector accesses aligned (checked by the caller)
HDS_EXPORT int hds_transpose_bf16(const void* src, void* dst, int rows, int cols, long lds, hipStream_t st) {
  if (rows <= 0 || cols <= 0) return hipSuccess;
  if (rows % 8 || lds % 8) return hipErrorInvalidValue;
  dim3 grid((cols + TT - 1) / TT, (rows + TT - 1) / TT);
  hipLaunchKernelGGL(transpose_bf16_kernel, grid, dim3(256), 0, st, (const bf16*)src, (bf16*)dst, rows, cols,
                     (int64_t)lds);
  return hipGetLastError();
}
