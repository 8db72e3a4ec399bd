// Evoformer attention forward with MSA-mask and pair biases (DS4Sci_EvoformerAttention), gfx950.
//
// Reference parity: csrc/deepspeed4science/evoformer_attn (CUTLASS memory-efficient attention with bias, SURVEY.md
// §2.10 N16 / §2.11 K24). Not a translation: one wave64 owns 32 queries of one (b, n, h) and streams the keys in
// 32-row tiles through v_mfma_f32_32x32x16_bf16 with the FlashAttention orientation of attn_common.h:
//   S^T = K . Q^T puts the QUERY on the lane, so the online-softmax statistics are lane-local (one cross-half
//   shuffle), and the S^T accumulator is directly the B operand of O^T = V^T . P^T (acc_to_b) — no LDS round trip.
// Evoformer heads are small (D = 32 or 64, L ~ 256-1024), so the operands come straight from global memory /
// L2 as 16-byte rows (Q, K) and coalesced per-key rows (V^T: lanes = 32 consecutive d of one key); the grid is
// (B*N*H, query tiles), tens of thousands of waves for MSA row attention. Biases (same dtype as Q) are added in
// fp32 before the softmax: bias1[b, n, key] (mask, broadcast over heads/queries), bias2[b, h, q, key] (pair bias,
// broadcast over the N rows). The kernel also writes the natural-log LSE per query for the memory-efficient
// backward (ops/deepspeed4science/evoformer_attn.py recomputes P from it chunk by chunk).
#include "attn_common.h"

using namespace hds;
using namespace hds::attn;

namespace {

template <typename T>
__device__ __forceinline__ float ld(const T* p) { return to_f(*p); }

template <int D, typename T>
__global__ __launch_bounds__(64) void evo_fwd_kernel(const bf16* __restrict__ q, const bf16* __restrict__ k,
                                                     const bf16* __restrict__ v, const T* __restrict__ b1,
                                                     const T* __restrict__ b2, bf16* __restrict__ o,
                                                     float* __restrict__ lse, int N, int L, int H, float scale) {
  const int lane = threadIdx.x;
  const int hf = lane >> 5, j = lane & 31;
  const int q0 = blockIdx.y * 32;
  const int bnh = blockIdx.x;  // (b * N + n) * H + h
  const int h = bnh % H, bn = bnh / H, b = bn / N;
  const int64_t tok = (int64_t)H * D;  // stride between tokens
  const bf16* qb = q + (int64_t)bn * L * tok + (int64_t)h * D;
  const bf16* kb = k + (int64_t)bn * L * tok + (int64_t)h * D;
  const bf16* vb = v + (int64_t)bn * L * tok + (int64_t)h * D;
  const int myq = q0 + j;
  const int qc = myq < L ? myq : L - 1;
  constexpr float kLog2e = 1.4426950408889634f;
  const float c = scale * kLog2e;

  bf16x8 qf[D / 16];
#pragma unroll
  for (int ks = 0; ks < D / 16; ++ks) qf[ks] = *reinterpret_cast<const bf16x8*>(qb + qc * tok + 16 * ks + 8 * hf);

  f32x16 acc[D / 32];
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt) acc[dt] = f32x16{};
  float m = -INFINITY, l = 0.f;
  const T* b1r = b1 ? b1 + (int64_t)bn * L : nullptr;
  const T* b2r = b2 ? b2 + ((int64_t)(b * H + h) * L + qc) * L : nullptr;

  for (int k0 = 0; k0 < L; k0 += 32) {
    // S^T tile: rows = keys k0 + acc_row(r, hf), column = this lane's query
    const int kr = min(k0 + j, L - 1);
    f32x16 s = f32x16{};
#pragma unroll
    for (int ks = 0; ks < D / 16; ++ks)
      s = mfma(*reinterpret_cast<const bf16x8*>(kb + kr * tok + 16 * ks + 8 * hf), qf[ks], s);
    float tmax = -INFINITY;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int key = k0 + acc_row(r, hf);
      float x = s[r] * c;
      if (key < L) {
        if (b1r) x += ld(b1r + key) * kLog2e;
        if (b2r) x += ld(b2r + key) * kLog2e;
      } else {
        x = -INFINITY;
      }
      s[r] = x;
      tmax = fmaxf(tmax, x);
    }
    tmax = fmaxf(tmax, __shfl_xor(tmax, 32, 64));
    const float mnew = fmaxf(m, tmax);
    const float alpha = (m == -INFINITY) ? 0.f : fast_exp2(m - mnew);
    m = mnew;
    float rs = 0.f;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const float e = fast_exp2(s[r] - m);
      s[r] = e;
      rs += e;
    }
    rs += __shfl_xor(rs, 32, 64);
    l = l * alpha + rs;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt) acc[dt] *= alpha;
    const bf16x8 pb[2] = {acc_to_b<0>(s), acc_to_b<1>(s)};
    // A operand = V^T: lane row d = 32*dt + j, element e of half hf <-> key 16*st + 8*(e>>2) + 4*hf + (e&3)
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int st = 0; st < 2; ++st) {
        bf16x8 va;
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const int key = min(k0 + 16 * st + 8 * (e >> 2) + 4 * hf + (e & 3), L - 1);
          va[e] = vb[key * tok + 32 * dt + j];
        }
        acc[dt] = mfma(va, pb[st], acc[dt]);
      }
  }

  if (myq < L) {
    const float inv = l > 0.f ? 1.f / l : 0.f;
    bf16* orow = o + (int64_t)bn * L * tok + (int64_t)myq * tok + (int64_t)h * D;
#pragma unroll
    for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        bf16x4 v4;
#pragma unroll
        for (int t = 0; t < 4; ++t) v4[t] = (bf16)(acc[dt][4 * g + t] * inv);
        *reinterpret_cast<bf16x4*>(orow + 32 * dt + acc_row(4 * g, hf)) = v4;
      }
    if (hf == 0) lse[(int64_t)bnh * L + myq] = (m + log2f(l)) / kLog2e;
  }
}

}  // namespace

// q/k/v/o [B, N, L, H, D] bf16; b1 [B, N, 1, 1, L] or null; b2 [B, 1, H, L, L] or null (bias dtype: 1 = bf16,
// 0 = fp32); lse [B, N, H, L] fp32 (natural log of the softmax normaliser of the scaled+biased scores).
HDS_EXPORT int hds_evoformer_fwd(const void* q, const void* k, const void* v, const void* b1, const void* b2,
                                 int bias_dtype, void* o, float* lse, int B, int N, int L, int H, int D, float scale,
                                 hipStream_t st) {
  if (B <= 0 || N <= 0 || L <= 0 || H <= 0) return 0;
  if (D != 32 && D != 64 && D != 128) return hipErrorInvalidValue;
  if ((L + 31) / 32 > 65535) return hipErrorInvalidValue;
  const dim3 grid(B * N * H, (L + 31) / 32);
#define HDS_EVO(DD, TT)                                                                                             \
  hipLaunchKernelGGL((evo_fwd_kernel<DD, TT>), grid, dim3(64), 0, st, (const bf16*)q, (const bf16*)k,             \
                     (const bf16*)v, (const TT*)b1, (const TT*)b2, (bf16*)o, lse, N, L, H, scale)
#define HDS_EVO_D(TT)                                                                                               \
  if (D == 32) HDS_EVO(32, TT); else if (D == 64) HDS_EVO(64, TT); else HDS_EVO(128, TT);
  if (bias_dtype == kBF16) {
    HDS_EVO_D(bf16)
  } else if (bias_dtype == kF32) {
    HDS_EVO_D(float)
  } else {
    return hipErrorInvalidValue;
  }
#undef HDS_EVO_D
#undef HDS_EVO
  return hipGetLastError();
}
