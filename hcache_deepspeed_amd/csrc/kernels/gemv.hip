// Decode-sized bf16 linear: y[M, N] = x[M, K] . W[N, K]^T (+ bias) for M <= 8 token rows.
//
// Capability parity: the reference's inference kernels run decode projections through cuBLAS GEMV-shaped GEMMs
// (csrc/transformer/inference/csrc/pt_binding.cpp qkv_gemm / vector_matmul). At M <= 8 the
// product is a pure weight stream (N * K * 2 bytes); hipBLASLt reaches 6+ TB/s on the wide projections but
// only ~2.7 TB/s on the narrow ones (Llama-3-8B qkv 6144 x 4096: 18.9 us for 50 MB), where a few hundred
// workgroups cannot cover its launch / tail latency (profiles/int_gemv_bench_r1.log).
//
// Structure: a wave owns R consecutive weight rows; each lane streams 16-B chunks (8 bf16) of those rows, two
// k-chunks per iteration so 2R loads are in flight per lane, and contracts them with the matching x chunks
// (x is tiny and L2/L1-resident) by v_dot2_f32_bf16 (4 per chunk per token row). The per-(row, token) partial
// sums are reduced across the wave once at the end.
#include "hds_common.h"

namespace {
using namespace hds;

typedef __bf16 bf16x2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float dot8(const bf16x8& a, const bf16x8& b, float c) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const bf16x2 a2 = {a[2 * j], a[2 * j + 1]}, b2 = {b[2 * j], b[2 * j + 1]};
    c = __builtin_amdgcn_fdot2_f32_bf16(a2, b2, c, false);
  }
  return c;
}

template <int MAXM, int R>
__global__ __launch_bounds__(256) void gemv_bf16_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                        const bf16* __restrict__ bias, bf16* __restrict__ y, int M,
                                                        int N, int K, int64_t ldx, int64_t ldy) {
  const int lane = threadIdx.x & 63;
  const int n0 = (blockIdx.x * 4 + (threadIdx.x >> 6)) * R;
  if (n0 >= N) return;
  float acc[R][MAXM];
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < MAXM; ++m) acc[r][m] = 0.f;
  const bf16* wr[R];
#pragma unroll
  for (int r = 0; r < R; ++r) wr[r] = w + (int64_t)min(n0 + r, N - 1) * K;  // tail rows re-read row N-1 (unused)
  int k0 = 8 * lane;
  for (; k0 + 512 < K; k0 += 1024) {
    bf16x8 wa[R], wb[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      wa[r] = *reinterpret_cast<const bf16x8*>(wr[r] + k0);
      wb[r] = *reinterpret_cast<const bf16x8*>(wr[r] + k0 + 512);
    }
#pragma unroll
    for (int m = 0; m < MAXM; ++m) {
      if (m < M) {
        const bf16x8 xa = *reinterpret_cast<const bf16x8*>(x + m * ldx + k0);
        const bf16x8 xb = *reinterpret_cast<const bf16x8*>(x + m * ldx + k0 + 512);
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][m] = dot8(xb, wb[r], dot8(xa, wa[r], acc[r][m]));
      }
    }
  }
  if (k0 < K) {  // K / 8 not a multiple of 128 chunks: one last single chunk per lane
    bf16x8 wa[R];
#pragma unroll
    for (int r = 0; r < R; ++r) wa[r] = *reinterpret_cast<const bf16x8*>(wr[r] + k0);
#pragma unroll
    for (int m = 0; m < MAXM; ++m) {
      if (m < M) {
        const bf16x8 xa = *reinterpret_cast<const bf16x8*>(x + m * ldx + k0);
#pragma unroll
        for (int r = 0; r < R; ++r) acc[r][m] = dot8(xa, wa[r], acc[r][m]);
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < MAXM; ++m) {
      if (m < M && n0 + r < N) {
        float v = wave_sum(acc[r][m]);
        if (lane == 0) {
          if (bias) v += (float)bias[n0 + r];
          y[m * ldy + n0 + r] = (bf16)v;
        }
      }
    }
}

}  // namespace

// Shapes the kernel takes: M <= 8 rows, K a multiple of 8 (16-B rows), 16-B aligned operands (checked by the caller).
HDS_EXPORT int hds_gemv_bf16_supported(int M, int N, int K) { return M >= 1 && M <= 8 && N >= 1 && K >= 8 && K % 8 == 0; }

HDS_EXPORT int hds_gemv_bf16(const void* x, const void* w, const void* bias, void* y, int M, int N, int K, int64_t ldx,
                             int64_t ldy, hipStream_t st) {
  if (!hds_gemv_bf16_supported(M, N, K) || ldx % 8) return hipErrorInvalidValue;
  // R = 4 rows per wave while that still leaves >= 2 waves per SIMD on 256 CUs, else 2 / 1 (parallelism)
#define HDS_GV(MM, RR)                                                                                        \
  hipLaunchKernelGGL((gemv_bf16_kernel<MM, RR>), dim3((N + 4 * RR - 1) / (4 * RR)), dim3(256), 0, st,        \
                     (const bf16*)x, (const bf16*)w, (const bf16*)bias, (bf16*)y, M, N, K, ldx, ldy)
#define HDS_GVM(RR)                                                                                           \
  if (M == 1) HDS_GV(1, RR); else if (M <= 2) HDS_GV(2, RR); else if (M <= 4) HDS_GV(4, RR); else HDS_GV(8, RR);
  if (N >= 8192) {
    HDS_GVM(4)
  } else if (N >= 4096) {
    HDS_GVM(2)
  } else {
    HDS_GVM(1)
  }
#undef HDS_GVM
#undef HDS_GV
  return hipGetLastError();
}
