// Mixed-input GEMM on the gfx950 matrix cores: C[M, N] = A[M, K] (bf16) x dequant(W)[N, K]^T for weight-only
// quantized W (symmetric group INT8, INT4, or FP6 e3m2 / e2m3 with fp32 group scales along k), bf16 out.
//
// Reference parity: the CUTLASS mixed-input GEMM (inference/v2 mixed_gemm) and the
// FP6-LLM tensor-core kernel (N12 / K29, inference/v2/kernels/core_ops/cuda_linear). Those decode packed weights
// in the mainloop so the weight stream stays at 8 / 6 / 4 bits; this kernel does the same on MFMA.
//
// Regime: 8 < M <= a few hundred rows (batched decode, chunked prefill) where a bf16 GEMM is bound by the 16-bit
// weight stream. Decode-sized M (<= 8) runs the GEMVs (quant.hip / fpq.hip); prefill-sized M dequantizes once and
// runs hipBLASLt (compute-bound there, so the weight bytes no longer matter).
//
// Structure: workgroup = 4 waves = 512 weight rows (wave = 4 fragments of 32 rows, the weight row on the MFMA lane)
// x 32*MB activation rows, over one K split. Per 64-k chunk a lane reads 32 consecutive k of each of its 4 weight
// rows (32 B int8, 16 B int4, 24 B fp6), applies the group scale and converts to bf16x8 B fragments; the
// contraction order inside a chunk is permuted (half h of the lane group takes k = 32h .. 32h + 31, fragment j = 8
// of them) and the A fragments are read with the same permutation, so the sum is unchanged. The A chunk is staged
// once per workgroup in LDS (padded rows, conflict-free ds_read_b128) and every A fragment feeds 4 MFMAs: a first
// version that read A per 32-row wave from L2 moved 2x (M = 16) to 30x (M = 256) more A bytes than weight bytes
// and ran at 0.2-0.8x the bf16 GEMM. The next chunk's weights and A are loaded before the current chunk's MFMAs.
// K splits (grid.z) write fp32 partials reduced by wmix_reduce_kernel.
#include "hds_common.h"

namespace {
using namespace hds;

__device__ __forceinline__ f32x16 mma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

enum WFmt : int { kInt8 = 0, kInt4 = 1, kFp6 = 2 };

template <int FMT> struct WRaw;
template <> struct WRaw<kInt8> { uint4 a, b; };
template <> struct WRaw<kInt4> { uint4 a; };
template <> struct WRaw<kFp6> { uint2 a, b, c; };

// raw bytes of the 32 weights k = ks .. ks + 31 of row n
template <int FMT>
__device__ __forceinline__ WRaw<FMT> load_w(const uint8_t* __restrict__ w, int64_t n, int K, int ks) {
  WRaw<FMT> r;
  if constexpr (FMT == kInt8) {
    const uint4* p = reinterpret_cast<const uint4*>(w + n * K + ks);
    r.a = p[0];
    r.b = p[1];
  } else if constexpr (FMT == kInt4) {
    r.a = *reinterpret_cast<const uint4*>(w + (n * K + ks) / 2);
  } else {
    const uint2* p = reinterpret_cast<const uint2*>(w + (n * K + ks) * 3 / 4);
    r.a = p[0];
    r.b = p[1];
    r.c = p[2];
  }
  return r;
}

// FP6 magnitude (E exponent bits, M mantissa bits, no inf/nan) -> float, without ldexp:
// normal codes become an fp32 bit pattern directly; subnormals (e == 0) are m * 2^(1 - bias - M)
template <int E, int M>
__device__ __forceinline__ float fp6_val(uint32_t c) {
  constexpr int bias = (1 << (E - 1)) - 1;
  const uint32_t e = (c >> M) & ((1u << E) - 1), m = c & ((1u << M) - 1);
  const float nrm = __uint_as_float(((e + 127 - bias) << 23) | (m << (23 - M)));
  const float sub = (float)m * __uint_as_float((uint32_t)(127 + 1 - bias - M) << 23);
  const float v = e ? nrm : sub;
  return (c >> (E + M)) & 1u ? -v : v;
}

// fragment j (weights 8j .. 8j+7 of the lane's 32) scaled by s, as bf16
template <int FMT, int E>
__device__ __forceinline__ bf16x8 frag(const WRaw<FMT>& r, int j, float s) {
  bf16x8 out;
  if constexpr (FMT == kInt8) {
    const uint32_t dw[8] = {r.a.x, r.a.y, r.a.z, r.a.w, r.b.x, r.b.y, r.b.z, r.b.w};
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int e = 8 * j + t;
      out[t] = (bf16)((float)(int8_t)((dw[e >> 2] >> (8 * (e & 3))) & 0xff) * s);
    }
  } else if constexpr (FMT == kInt4) {
    const uint32_t dw[4] = {r.a.x, r.a.y, r.a.z, r.a.w};
#pragma unroll
    for (int t = 0; t < 8; ++t) out[t] = (bf16)((float)((int)((dw[j] >> (4 * t)) & 0xf) ^ 8) - 8.f) * s;
  } else {
    const uint64_t q[3] = {((uint64_t)r.a.y << 32) | r.a.x, ((uint64_t)r.b.y << 32) | r.b.x,
                           ((uint64_t)r.c.y << 32) | r.c.x};
#pragma unroll
    for (int t = 0; t < 8; ++t) {
      const int b = 6 * (8 * j + t), wi = b >> 6, o = b & 63;
      uint64_t v = q[wi] >> o;
      if (o > 58) v |= q[wi + 1] << (64 - o);
      out[t] = (bf16)(fp6_val<E, 5 - E>((uint32_t)v & 63u) * s);
    }
  }
  return out;
}

constexpr int kArow = 144;             // LDS bytes per A row of a 64-k chunk (128 + 16 pad: conflict-free b128 reads)

template <int FMT, int MB, int E, int kNF>
__global__ __launch_bounds__(256) void wmix_gemm_kernel(const bf16* __restrict__ A, const uint8_t* __restrict__ W,
                                                        const float* __restrict__ scales,
                                                        const bf16* __restrict__ bias, bf16* __restrict__ C,
                                                        float* __restrict__ part, int M, int N, int K, int G,
                                                        int kc) {
  constexpr int BM = 32 * MB;
  constexpr int kBN = 4 * 32 * kNF;  // weight rows per workgroup
  __shared__ __attribute__((aligned(16))) char As[2][BM * kArow];
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6, h = lane >> 5;
  const int nb = blockIdx.x * kBN + 32 * kNF * w + (lane & 31);  // row of fragment f: nb + 32 f
  const int m0 = blockIdx.y * BM;
  const int k_begin = blockIdx.z * kc, k_end = min(K, k_begin + kc);
  int nr[kNF];
#pragma unroll
  for (int f = 0; f < kNF; ++f) nr[f] = min(nb + 32 * f, N - 1);
  // A staging: thread -> (row, 16-B piece) of the chunk, MB rows of 32 apart
  const int ar = tid >> 3, ap = tid & 7;
  const bf16* asrc[MB];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb) asrc[mb] = A + (int64_t)min(m0 + 32 * mb + ar, M - 1) * K + 8 * ap;

  f32x16 acc[MB][kNF];
#pragma unroll
  for (int mb = 0; mb < MB; ++mb)
#pragma unroll
    for (int f = 0; f < kNF; ++f) acc[mb][f] = f32x16{};

  WRaw<FMT> wc[kNF], wn[kNF];
  float sc[kNF], sn[kNF];
  auto load_wf = [&](WRaw<FMT> (&wr)[kNF], float (&sr)[kNF], int k0) {
#pragma unroll
    for (int f = 0; f < kNF; ++f) {
      wr[f] = load_w<FMT>(W, nr[f], K, k0 + 32 * h);
      sr[f] = scales[(int64_t)nr[f] * (K / G) + (k0 + 32 * h) / G];
    }
  };
  bf16x8 ag[MB];
  auto load_ag = [&](int k0) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) ag[mb] = *reinterpret_cast<const bf16x8*>(asrc[mb] + k0);
  };
  auto store_ag = [&](int buf) {
#pragma unroll
    for (int mb = 0; mb < MB; ++mb) *reinterpret_cast<bf16x8*>(&As[buf][(32 * mb + ar) * kArow + 16 * ap]) = ag[mb];
  };

  load_wf(wc, sc, k_begin);
  load_ag(k_begin);
  store_ag(0);
  __syncthreads();
  int buf = 0;
  for (int k0 = k_begin; k0 < k_end; k0 += 64) {
    const bool more = k0 + 64 < k_end;
    if (more) {
      load_wf(wn, sn, k0 + 64);
      load_ag(k0 + 64);
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      bf16x8 af[MB];
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
        af[mb] = *reinterpret_cast<const bf16x8*>(&As[buf][(32 * mb + (lane & 31)) * kArow + 64 * h + 16 * j]);
#pragma unroll
      for (int f = 0; f < kNF; ++f) {
        const bf16x8 b = frag<FMT, E>(wc[f], j, sc[f]);
#pragma unroll
        for (int mb = 0; mb < MB; ++mb) acc[mb][f] = mma(af[mb], b, acc[mb][f]);
      }
    }
    if (more) {
      store_ag(buf ^ 1);
#pragma unroll
      for (int f = 0; f < kNF; ++f) {
        wc[f] = wn[f];
        sc[f] = sn[f];
      }
    }
    __syncthreads();
    buf ^= 1;
  }
#pragma unroll
  for (int f = 0; f < kNF; ++f) {
    const int n = nb + 32 * f;
    if (n >= N) continue;
    if (part == nullptr) {
      const float bv = bias ? (float)bias[n] : 0.f;
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + 32 * mb + acc_row(r, h);
          if (m < M) C[(int64_t)m * N + n] = (bf16)(acc[mb][f][r] + bv);
        }
    } else {
      float* P = part + (int64_t)blockIdx.z * M * N;
#pragma unroll
      for (int mb = 0; mb < MB; ++mb)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const int m = m0 + 32 * mb + acc_row(r, h);
          if (m < M) P[(int64_t)m * N + n] = acc[mb][f][r];
        }
    }
  }
}

// C = sum_z part[z] (+ bias): 4 outputs per thread
__global__ __launch_bounds__(256) void wmix_reduce_kernel(const float* __restrict__ part,
                                                          const bf16* __restrict__ bias, bf16* __restrict__ C, int M,
                                                          int N, int splits) {
  const int64_t i = ((int64_t)blockIdx.x * 256 + threadIdx.x) * 4;
  const int64_t MN = (int64_t)M * N;
  if (i >= MN) return;
  f32x4 a = *reinterpret_cast<const f32x4*>(part + i);
  for (int z = 1; z < splits; ++z) a += *reinterpret_cast<const f32x4*>(part + z * MN + i);
  const int n = (int)(i % N);
  bf16x4 o;
#pragma unroll
  for (int t = 0; t < 4; ++t) o[t] = (bf16)(a[t] + (bias ? (float)bias[n + t] : 0.f));
  *reinterpret_cast<bf16x4*>(C + i) = o;
}

int pick_mb(int M) { return M <= 32 ? 1 : 2; }
// weight fragments per wave: 1 at small M (more workgroups in flight for the weight stream), 4 once the A chunk
// re-reads and the per-fragment MFMA chain matter (measured, profiles/wmix_bench_r2.log)
int pick_nf(int M) { return M <= 64 ? 1 : 4; }

}  // namespace

// number of K splits (grid.z) for a problem; the caller provides an fp32 workspace of splits * M * N when > 1
HDS_EXPORT int hds_wmix_splits(int M, int N, int K) {
  const int mb = pick_mb(M), kBN = 128 * pick_nf(M);
  const int base = ((N + kBN - 1) / kBN) * ((M + 32 * mb - 1) / (32 * mb));
  int splits = (512 + base - 1) / base;
  const int max_splits = K / 256 > 1 ? K / 256 : 1;  // >= 4 chunks of 64 k per split
  if (splits > max_splits) splits = max_splits;
  if (splits > 16) splits = 16;
  if (splits < 1) splits = 1;
  const int kc = ((K / 64 + splits - 1) / splits) * 64;
  return (K + kc - 1) / kc;
}

HDS_EXPORT int hds_wmix_supported(int M, int N, int K, int G) {
  return M > 0 && N % 4 == 0 && K % 64 == 0 && G % 32 == 0 && K % G == 0;
}

// fmt: 0 int8, 1 int4, 2 fp6 (ebits 3 -> e3m2, ebits 2 -> e2m3). A [M, K] bf16 row-major, W packed [N, K], scales
// [N, K / G] fp32, bias [N] bf16 or null, C [M, N] bf16, ws fp32 [splits, M, N] (null when splits == 1)
HDS_EXPORT int hds_wmix_gemm(const void* A, const void* W, const float* scales, const void* bias, void* C, float* ws,
                             int M, int N, int K, int G, int fmt, int ebits, hipStream_t st) {
  if (!hds_wmix_supported(M, N, K, G)) return hipErrorInvalidValue;
  const int splits = hds_wmix_splits(M, N, K);
  if (splits > 1 && ws == nullptr) return hipErrorInvalidValue;
  const int kc = ((K / 64 + splits - 1) / splits) * 64;
  const int mb = pick_mb(M), nf = pick_nf(M), kBN = 128 * nf;
  dim3 grid((N + kBN - 1) / kBN, (M + 32 * mb - 1) / (32 * mb), splits);
  float* part = splits > 1 ? ws : nullptr;
  auto launch = [&](auto kern) {
    hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, (const bf16*)A, (const uint8_t*)W, scales, (const bf16*)bias,
                       (bf16*)C, part, M, N, K, G, kc);
  };
#define HDS_WMIX(F, E)                                                 \
  do {                                                                 \
    if (mb == 1 && nf == 1) launch(wmix_gemm_kernel<F, 1, E, 1>);      \
    else if (mb == 1) launch(wmix_gemm_kernel<F, 1, E, 4>);            \
    else if (nf == 1) launch(wmix_gemm_kernel<F, 2, E, 1>);            \
    else launch(wmix_gemm_kernel<F, 2, E, 4>);                         \
  } while (0)
  if (fmt == 0) HDS_WMIX(kInt8, 0);
  else if (fmt == 1) HDS_WMIX(kInt4, 0);
  else if (fmt == 2 && ebits == 3) HDS_WMIX(kFp6, 3);
  else if (fmt == 2 && ebits == 2) HDS_WMIX(kFp6, 2);
  else return hipErrorInvalidValue;
#undef HDS_WMIX
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || splits == 1) return e;
  const int64_t MN = (int64_t)M * N;
  hipLaunchKernelGGL(wmix_reduce_kernel, dim3((unsigned)((MN / 4 + 255) / 256)), dim3(256), 0, st, ws,
                     (const bf16*)bias, (bf16*)C, M, N, splits);
  return hipGetLastError();
}
