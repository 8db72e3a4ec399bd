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

// ---------------------------------------------------------------------------------------------------------------
// Fused decode GEMV: the pre-norm and the gated activation of a decoder layer folded into its projection GEMVs, so a
// decode step launches neither the RMSNorm nor the GLU kernel (each ~4-5 us per call in a decode graph, i.e. about a
// tenth of a Llama-3-8B B = 1 step, for kernels that move a few KB).
//
// NORM: the input rows are x = bf16(r * rstd * gamma), r = bf16(h + res) (or h without a residual) -- the arithmetic
// of norm.hip's RMSNorm forward. rstd is one scalar per row, so x . w = rstd * (bf16(r * gamma) . w): a wave streams
// its weight rows against bf16(r * gamma) chunks built on the fly (r and gamma are L2-resident, K * 2 bytes) and, since
// its 64 lanes together walk the whole row, accumulates sum(r^2) in the same loop; rstd scales the reduced dot
// products at the end. No workgroup-wide prologue (row reduction, LDS, barriers) sits ahead of the weight stream: that
// serial prologue cost what a separate RMSNorm launch did (fused qkv 15.4 us vs 10.9 us plain GEMV + 4.6 us norm).
// Workgroup 0 also writes r (the new residual stream) and, when asked, x (the normed rows: HCache's hidden-state
// latents) once its waves know rstd.
// GLU: the weight is [gate; up] ([2I, K]) and the output y[M, I] = bf16(act(bf16(x.g_j)) * bf16(x.u_j)) (silu): a wave
// owns R output columns and streams their gate AND up rows, so the [M, 2I] intermediate never exists.
__device__ __forceinline__ float silu_f(float v) { return v * __builtin_amdgcn_rcpf(1.f + __expf(-v)); }

// r = bf16(h + res) (h without res) for 8 elements at k
__device__ __forceinline__ bf16x8 load_r(const bf16* __restrict__ h, const bf16* __restrict__ res, int64_t off, int k) {
  bf16x8 hv = *reinterpret_cast<const bf16x8*>(h + off + k);
  if (res != nullptr) {
    const bf16x8 rv = *reinterpret_cast<const bf16x8*>(res + off + k);
#pragma unroll
    for (int j = 0; j < 8; ++j) hv[j] = (bf16)((float)hv[j] + (float)rv[j]);  // round like the unfused add
  }
  return hv;
}

// the GEMV operand chunk: bf16(r * gamma) with sum(r^2) accumulated into ss (NORM), else h itself
template <bool NORM>
__device__ __forceinline__ bf16x8 load_x(const bf16* __restrict__ h, const bf16* __restrict__ res,
                                         const bf16* __restrict__ gamma, int64_t off, int k, float& ss) {
  if constexpr (!NORM) {
    return *reinterpret_cast<const bf16x8*>(h + off + k);
  } else {
    const bf16x8 r = load_r(h, res, off, k);
    const bf16x8 g = *reinterpret_cast<const bf16x8*>(gamma + k);
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float v = (float)r[j];
      ss += v * v;
      o[j] = (bf16)(v * (float)g[j]);
    }
    return o;
  }
}

template <int MAXM, int R, bool NORM, bool GLU>
__global__ __launch_bounds__(256) void gemv_fused_kernel(const bf16* __restrict__ h, const bf16* __restrict__ res,
                                                         const bf16* __restrict__ gamma, float eps,
                                                         const bf16* __restrict__ w, bf16* __restrict__ y,
                                                         bf16* __restrict__ r_out, bf16* __restrict__ x_out, int M,
                                                         int N, int K, int64_t ldh, int64_t ldy) {
  const int lane = threadIdx.x & 63;
  const int wid = threadIdx.x >> 6;
  const int n0 = (blockIdx.x * 4 + wid) * R;  // output columns [n0, n0 + R)
  const bool writes_rows = NORM && blockIdx.x == 0 && (r_out != nullptr || x_out != nullptr);
  if (n0 >= N && !writes_rows) return;  // (workgroup 0's waves all run: they share the row writes below)
  constexpr int RR = GLU ? 2 * R : R;   // weight rows streamed per wave: the gate rows, then the up rows
  float acc[RR][MAXM], ss[MAXM];
#pragma unroll
  for (int m = 0; m < MAXM; ++m) {
    ss[m] = 0.f;
#pragma unroll
    for (int r = 0; r < RR; ++r) acc[r][m] = 0.f;
  }
  const bf16* wr[RR];
#pragma unroll
  for (int r = 0; r < R; ++r) {
    const int n = min(n0 + r, N - 1);  // tail columns re-read column N-1 (unused)
    wr[r] = w + (int64_t)n * K;
    if constexpr (GLU) wr[R + r] = w + (int64_t)(N + n) * K;
  }
  int k0 = 8 * lane;
  for (; k0 + 512 < K; k0 += 1024) {
    bf16x8 wa[RR], wb[RR];
#pragma unroll
    for (int r = 0; r < RR; ++r) {
      wa[r] = *reinterpret_cast<const bf16x8*>(wr[r] + k0);
      wb[r] = *reinterpret_cast<const bf16x8*>(wr[r] + k0 + 512);
    }
#pragma unroll
    for (int m = 0; m < MAXM; ++m) {
      if (m < M) {
        const bf16x8 xa = load_x<NORM>(h, res, gamma, m * ldh, k0, ss[m]);
        const bf16x8 xb = load_x<NORM>(h, res, gamma, m * ldh, k0 + 512, ss[m]);
#pragma unroll
        for (int r = 0; r < RR; ++r) acc[r][m] = dot8(xb, wb[r], dot8(xa, wa[r], acc[r][m]));
      }
    }
  }
  if (k0 < K) {
    bf16x8 wa[RR];
#pragma unroll
    for (int r = 0; r < RR; ++r) wa[r] = *reinterpret_cast<const bf16x8*>(wr[r] + k0);
#pragma unroll
    for (int m = 0; m < MAXM; ++m) {
      if (m < M) {
        const bf16x8 xa = load_x<NORM>(h, res, gamma, m * ldh, k0, ss[m]);
#pragma unroll
        for (int r = 0; r < RR; ++r) acc[r][m] = dot8(xa, wa[r], acc[r][m]);
      }
    }
  }
  float rstd[MAXM];
#pragma unroll
  for (int m = 0; m < MAXM; ++m) rstd[m] = NORM ? rsqrtf(wave_sum(ss[m]) / (float)K + eps) : 1.f;
  if (writes_rows) {  // the 4 waves of workgroup 0 split the rows' chunks
    for (int c = (wid * 64 + lane) * 8; c < K; c += 2048) {
#pragma unroll
      for (int m = 0; m < MAXM; ++m) {
        if (m < M) {
          const bf16x8 r = load_r(h, res, m * ldh, c);
          if (r_out != nullptr && res != nullptr) *reinterpret_cast<bf16x8*>(r_out + m * ldh + c) = r;
          if (x_out != nullptr) {
            const bf16x8 g = *reinterpret_cast<const bf16x8*>(gamma + c);
            bf16x8 o;
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = (bf16)((float)r[j] * rstd[m] * (float)g[j]);
            *reinterpret_cast<bf16x8*>(x_out + m * ldh + c) = o;
          }
        }
      }
    }
  }
#pragma unroll
  for (int r = 0; r < R; ++r)
#pragma unroll
    for (int m = 0; m < MAXM; ++m) {
      if (m < M && n0 + r < N) {
        const float v = rstd[m] * wave_sum(acc[r][m]);
        if constexpr (GLU) {
          const float u = rstd[m] * wave_sum(acc[R + r][m]);
          if (lane == 0) y[m * ldy + n0 + r] = (bf16)(silu_f((float)(bf16)v) * (float)(bf16)u);
        } else {
          if (lane == 0) y[m * ldy + n0 + r] = (bf16)v;
        }
      }
    }
}

// ---------------------------------------------------------------------------------------------------------------
// Skinny GEMM for 2..16 token rows on the matrix cores: y[M, N] = x[M, K] . W[N, K]^T (+ bias).
// The VALU GEMV above spends 4 dot2 instructions per 16-B weight chunk PER ROW, so from a few rows on it is VALU-bound
// (o projection at M = 8: 1.7 TB/s) and hipBLASLt's small-M tiles stream at 3.5-3.7 TB/s. Here one
// mfma_f32_16x16x32_bf16 contracts a 16-column x 32-k weight tile with all (up to 16) token rows at once, so the
// kernel is a pure weight stream: A = W rows (lane l: row n0 + (l & 15), k = 8 (l >> 4) .. +8, one 16-B load), B = x^T
// (lane l: token l & 15, same k; zero past M), C: token = l & 15, column n0 + 4 (l >> 4) + reg. A workgroup owns 16
// output columns; its 4 waves split K four ways with 8 weight loads per lane in flight, and the partial tiles are
// summed through LDS.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

template <int U>
__global__ __launch_bounds__(256) void skinny_mfma_kernel(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                          const bf16* __restrict__ bias, bf16* __restrict__ y, int M,
                                                          int N, int K, int64_t ldx, int64_t ldy) {
  __shared__ f32x4 red[3][64];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int n0 = blockIdx.x * 16;
  const int row = min(n0 + (lane & 15), N - 1);  // tail columns re-read column N-1 (not stored)
  const int tok = lane & 15;
  const int kq = K >> 2;  // this wave's quarter of K (K % 128 == 0)
  const int kb = wid * kq + 8 * (lane >> 4);
  const bf16* wp = w + (int64_t)row * K + kb;
  const bf16* xp = x + (int64_t)min(tok, M - 1) * ldx + kb;
  const bool tok_ok = tok < M;
  f32x4 acc = {0.f, 0.f, 0.f, 0.f};
  int k = 0;
  for (; k + 32 * U <= kq; k += 32 * U) {
    bf16x8_t a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) a[u] = *reinterpret_cast<const bf16x8_t*>(wp + k + 32 * u);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      b[u] = *reinterpret_cast<const bf16x8_t*>(xp + k + 32 * u);
      if (!tok_ok) b[u] = bf16x8_t{};
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[u], b[u], acc, 0, 0, 0);
  }
  for (; k < kq; k += 32) {
    const bf16x8_t a = *reinterpret_cast<const bf16x8_t*>(wp + k);
    bf16x8_t b = *reinterpret_cast<const bf16x8_t*>(xp + k);
    if (!tok_ok) b = bf16x8_t{};
    acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, acc, 0, 0, 0);
  }
  if (wid > 0) red[wid - 1][lane] = acc;
  __syncthreads();
  if (wid == 0) {
#pragma unroll
    for (int v = 0; v < 3; ++v) acc += red[v][lane];
    if (tok_ok) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int n = n0 + 4 * (lane >> 4) + r;
        if (n < N) {
          float v = acc[r];
          if (bias) v += (float)bias[n];
          y[(int64_t)tok * ldy + n] = (bf16)v;
        }
      }
    }
  }
}

int g_skinny_u = 16;

}  // namespace

// Skinny matrix-core GEMM (skinny_mfma_kernel): 1 <= M <= 16, K % 128 == 0, 16-B aligned rows
HDS_EXPORT int hds_skinny_gemm_bf16(const void* x, const void* w, const void* bias, void* y, int M, int N, int K,
                                    int64_t ldx, int64_t ldy, hipStream_t st) {
  if (M < 1 || M > 16 || N < 1 || K < 128 || K % 128 || ldx % 8) return hipErrorInvalidValue;
  if (g_skinny_u == 32 && (K >> 2) % 1024 == 0)
    hipLaunchKernelGGL(skinny_mfma_kernel<32>, dim3((N + 15) / 16), dim3(256), 0, st, (const bf16*)x,
                       (const bf16*)w, (const bf16*)bias, (bf16*)y, M, N, K, ldx, ldy);
  else if (g_skinny_u >= 16)
    hipLaunchKernelGGL(skinny_mfma_kernel<16>, dim3((N + 15) / 16), dim3(256), 0, st, (const bf16*)x,
                       (const bf16*)w, (const bf16*)bias, (bf16*)y, M, N, K, ldx, ldy);
  else
    hipLaunchKernelGGL(skinny_mfma_kernel<8>, dim3((N + 15) / 16), dim3(256), 0, st, (const bf16*)x,
                       (const bf16*)w, (const bf16*)bias, (bf16*)y, M, N, K, ldx, ldy);
  return hipGetLastError();
}

// weight loads per lane in flight in the skinny GEMM (8, 16 or 32); returns the previous value
HDS_EXPORT int hds_skinny_set_unroll(int u) {
  const int prev = g_skinny_u;
  g_skinny_u = u >= 32 ? 32 : (u >= 16 ? 16 : 8);
  return prev;
}

// Fused decode GEMV (see gemv_fused_kernel): y[M, N] = norm(h (+ res)) . W^T, or with glu != 0, y[M, N] =
// silu(x . Wg^T) * (x . Wu^T) for W = [Wg; Wu] of 2N rows (x normed when gamma is given, else h itself). r_out /
// x_out (workgroup 0, with gamma): the new residual rows and the normed rows. ldh: row stride of h / res / r_out /
// x_out (elements); ldy: row stride of y. Shapes: M <= 8, K % 8 == 0, 16-B aligned operands (checked by the caller).
HDS_EXPORT int hds_gemv_fused_bf16(const void* h, const void* res, const void* gamma, float eps, const void* w,
                                   void* y, void* r_out, void* x_out, int glu, int M, int N, int K, int64_t ldh,
                                   int64_t ldy, hipStream_t st) {
  if (M < 1 || M > 8 || N < 1 || K < 8 || K % 8 || ldh % 8) return hipErrorInvalidValue;
  if (gamma == nullptr && (r_out != nullptr || x_out != nullptr || res != nullptr)) return hipErrorInvalidValue;
  const int R = N >= 8192 ? (glu ? 2 : 4) : (N >= 4096 ? 2 : 1);
#define HDS_GF(MM, RR, NN, GG)                                                                                   \
  hipLaunchKernelGGL((gemv_fused_kernel<MM, RR, NN, GG>), dim3((N + 4 * RR - 1) / (4 * RR)), dim3(256), 0, st,  \
                     (const bf16*)h, (const bf16*)res, (const bf16*)gamma, eps, (const bf16*)w, (bf16*)y,      \
                     (bf16*)r_out, (bf16*)x_out, M, N, K, ldh, ldy)
#define HDS_GFM(RR, NN, GG)                                                                                    \
  if (M == 1) HDS_GF(1, RR, NN, GG); else if (M <= 2) HDS_GF(2, RR, NN, GG);                                   \
  else if (M <= 4) HDS_GF(4, RR, NN, GG); else HDS_GF(8, RR, NN, GG);
#define HDS_GFR(NN, GG)                                                                                        \
  if (R == 4) { HDS_GFM(4, NN, GG) } else if (R == 2) { HDS_GFM(2, NN, GG) } else { HDS_GFM(1, NN, GG) }
  if (gamma != nullptr) {
    if (glu) { HDS_GFR(true, true) } else { HDS_GFR(true, false) }
  } else {
    if (glu) { HDS_GFR(false, true) } else { return hipErrorInvalidValue; }  // plain GEMV: hds_gemv_bf16
  }
#undef HDS_GFR
#undef HDS_GFM
#undef HDS_GF
  return hipGetLastError();
}

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
