// Generic minifloat (FP6 e3m2 / e2m3, FP12 e4m7, any E+M<=11) group quantization with bit packing, optional
// stochastic rounding, dequantization, and a weight-only FP6 x bf16 skinny GEMM for decode-sized batches.
//
// Capability parity: csrc/fp_quantizer/fp_quantize.cu (K21: apply_quantization / apply_dequantization /
// apply_selective_dequantization for FP8/FP6/FP12 with stochastic rounding) and the FP6-LLM
// weight-only GEMM of inference/v2/kernels/core_ops/cuda_linear (K29, PTX mma.sync + cp.async there).
// OCP FP8 uses the hardware v_cvt_pk_fp8 path in quant.hip; this file covers the widths the chip has no
// per-element conversion for, with an exact round-to-nearest-even (or stochastic) encoder.
//
// Packing (little-endian bit stream inside each 4-element chunk): 6-bit -> 3 bytes, 8-bit -> 4, 12-bit -> 6.
// Layout: one wave per quantization group; lane l owns 4-element chunks l, l + 64, ... of its group, so a group
// of G elements uses min(64, G/4) lanes per pass; the group's abs-max is a wave reduction.
#include "hds_common.h"

using namespace hds;

namespace {

struct MiniFmt {
  int E, M, bias;
  float maxval;
};

__device__ __forceinline__ MiniFmt make_fmt(int ebits, int mbits) {
  MiniFmt f;
  f.E = ebits;
  f.M = mbits;
  f.bias = (1 << (ebits - 1)) - 1;
  // no inf / nan encodings: the top exponent is a normal binade (saturating formats, like OCP FP6)
  f.maxval = (2.f - ldexpf(1.f, -mbits)) * ldexpf(1.f, (1 << ebits) - 1 - f.bias);
  return f;
}

__device__ __forceinline__ uint32_t hash32(uint32_t a, uint32_t b) {
  uint32_t h = a * 0x9E3779B1u ^ (b + 0x7F4A7C15u + (a << 6) + (a >> 2));
  h ^= h >> 16;
  h *= 0x85EBCA6Bu;
  h ^= h >> 13;
  h *= 0xC2B2AE35u;
  h ^= h >> 16;
  return h;
}

// |x| <= maxval expected (scaled); returns sign|exp|mant code
__device__ __forceinline__ uint32_t encode(float x, const MiniFmt& f, bool stochastic, float u) {
  const uint32_t sign = x < 0.f ? 1u : 0u;
  float a = fabsf(x);
  if (!(a > 0.f)) return sign << (f.E + f.M);
  a = fminf(a, f.maxval);
  int k;
  frexpf(a, &k);
  int e = k - 1;  // a in [2^e, 2^(e+1))
  const int emin = 1 - f.bias;
  uint32_t expf_, mant;
  const float mscale = ldexpf(1.f, f.M);
  if (e < emin) {  // subnormal: value = m * 2^(emin - M)
    float mf = ldexpf(a, f.M - emin);
    float m = stochastic ? floorf(mf + u) : rintf(mf);
    if (m >= mscale) {
      expf_ = 1;
      mant = 0;
    } else {
      expf_ = 0;
      mant = (uint32_t)m;
    }
  } else {
    float mf = (ldexpf(a, -e) - 1.f) * mscale;
    float m = stochastic ? floorf(mf + u) : rintf(mf);
    if (m >= mscale) {
      m = 0.f;
      e += 1;
    }
    int ef = e + f.bias;
    if (ef > (1 << f.E) - 1) {  // saturate
      ef = (1 << f.E) - 1;
      m = mscale - 1.f;
    }
    expf_ = (uint32_t)ef;
    mant = (uint32_t)m;
  }
  return (sign << (f.E + f.M)) | (expf_ << f.M) | mant;
}

__device__ __forceinline__ float decode(uint32_t c, const MiniFmt& f) {
  const uint32_t mant = c & ((1u << f.M) - 1);
  const uint32_t ef = (c >> f.M) & ((1u << f.E) - 1);
  const bool neg = (c >> (f.E + f.M)) & 1u;
  float v = ef == 0 ? ldexpf((float)mant, 1 - f.bias - f.M)
                    : ldexpf(1.f + (float)mant * ldexpf(1.f, -f.M), (int)ef - f.bias);
  return neg ? -v : v;
}

// 4 codes of `bits` each -> bytes of the chunk (bits/2 bytes)
__device__ __forceinline__ void store_chunk(uint8_t* dst, const uint32_t (&c)[4], int bits) {
  if (bits == 8) {
    uint32_t w = c[0] | (c[1] << 8) | (c[2] << 16) | (c[3] << 24);
    *reinterpret_cast<uint32_t*>(dst) = w;
    return;
  }
  if (bits == 6) {
    const uint32_t w = c[0] | (c[1] << 6) | (c[2] << 12) | (c[3] << 18);
    dst[0] = w & 0xFF;
    dst[1] = (w >> 8) & 0xFF;
    dst[2] = (w >> 16) & 0xFF;
    return;
  }
  // 12-bit: two 24-bit words
  const uint32_t w0 = c[0] | (c[1] << 12), w1 = c[2] | (c[3] << 12);
  dst[0] = w0 & 0xFF;
  dst[1] = (w0 >> 8) & 0xFF;
  dst[2] = (w0 >> 16) & 0xFF;
  dst[3] = w1 & 0xFF;
  dst[4] = (w1 >> 8) & 0xFF;
  dst[5] = (w1 >> 16) & 0xFF;
}

__device__ __forceinline__ void load_chunk(const uint8_t* src, uint32_t (&c)[4], int bits) {
  if (bits == 8) {
    const uint32_t w = *reinterpret_cast<const uint32_t*>(src);
    c[0] = w & 0xFF;
    c[1] = (w >> 8) & 0xFF;
    c[2] = (w >> 16) & 0xFF;
    c[3] = w >> 24;
    return;
  }
  if (bits == 6) {
    const uint32_t w = src[0] | (src[1] << 8) | (src[2] << 16);
    c[0] = w & 63;
    c[1] = (w >> 6) & 63;
    c[2] = (w >> 12) & 63;
    c[3] = (w >> 18) & 63;
    return;
  }
  const uint32_t w0 = src[0] | (src[1] << 8) | (src[2] << 16), w1 = src[3] | (src[4] << 8) | (src[5] << 16);
  c[0] = w0 & 0xFFF;
  c[1] = w0 >> 12;
  c[2] = w1 & 0xFFF;
  c[3] = w1 >> 12;
}

template <typename T>
__global__ __launch_bounds__(256) void minifloat_quant_kernel(const T* __restrict__ x, uint8_t* __restrict__ q,
                                                              float* __restrict__ scales, int64_t n_groups, int G,
                                                              int ebits, int mbits, int stochastic, uint32_t seed) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= n_groups) return;
  const MiniFmt f = make_fmt(ebits, mbits);
  const int bits = 1 + ebits + mbits;
  const T* xg = x + g * G;
  float amax = 0.f;
  for (int c = lane; 4 * c < G; c += 64) {
#pragma unroll
    for (int j = 0; j < 4; ++j) amax = fmaxf(amax, fabsf(to_f(xg[4 * c + j])));
  }
  amax = wave_max(amax);
  const float scale = amax > 0.f ? amax / f.maxval : 1.f;
  uint8_t* qg = q + g * (int64_t)G * bits / 8;
  for (int c = lane; 4 * c < G; c += 64) {
    uint32_t code[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      float u = 0.f;
      if (stochastic) u = (float)(hash32(seed, (uint32_t)(g * G + 4 * c + j)) >> 8) * (1.f / 16777216.f);
      code[j] = encode(to_f(xg[4 * c + j]) / scale, f, stochastic != 0, u);
    }
    store_chunk(qg + (int64_t)c * bits / 2, code, bits);
  }
  if (lane == 0) scales[g] = scale;
}

template <typename T>
__global__ __launch_bounds__(256) void minifloat_dequant_kernel(const uint8_t* __restrict__ q,
                                                                const float* __restrict__ scales, T* __restrict__ y,
                                                                int64_t n_groups, int G, int ebits, int mbits) {
  const int lane = threadIdx.x & 63;
  const int64_t g = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (g >= n_groups) return;
  const MiniFmt f = make_fmt(ebits, mbits);
  const int bits = 1 + ebits + mbits;
  const float s = scales[g];
  const uint8_t* qg = q + g * (int64_t)G * bits / 8;
  T* yg = y + g * G;
  for (int c = lane; 4 * c < G; c += 64) {
    uint32_t code[4];
    load_chunk(qg + (int64_t)c * bits / 2, code, bits);
#pragma unroll
    for (int j = 0; j < 4; ++j) yg[4 * c + j] = from_f<T>(decode(code[j], f) * s);
  }
}

// y[m, n] = sum_k x[m, k] * W[n, k]; W: FP6 (e3m2 / e2m3) rows packed 3 bytes per 4 weights, group scales
// [N, K / G] along k. One wave per output feature, lane = 16 consecutive k (12 packed bytes = 3 dwords),
// M <= 8 activation rows held as fp32 partial sums; wave reduction at the end. Memory bound on the 6-bit
// weight stream (2.67x fewer bytes than bf16 weights) -- the decode-time regime FP6-LLM targets.
template <int MAXM>
__global__ __launch_bounds__(256) void fp6_gemv_kernel(const bf16* __restrict__ x, const uint8_t* __restrict__ w,
                                                       const float* __restrict__ scales, bf16* __restrict__ y, int M,
                                                       int N, int K, int G, int ebits, int mbits) {
  const int lane = threadIdx.x & 63;
  const int n = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (n >= N) return;
  const MiniFmt f = make_fmt(ebits, mbits);
  const uint8_t* wr = w + (int64_t)n * K * 3 / 4;
  const float* sr = scales + (int64_t)n * (K / G);
  float acc[MAXM];
#pragma unroll
  for (int m = 0; m < MAXM; ++m) acc[m] = 0.f;
  for (int k0 = 16 * lane; k0 < K; k0 += 16 * 64) {
    const uint32_t* p = reinterpret_cast<const uint32_t*>(wr + (int64_t)k0 * 3 / 4);
    const uint32_t d0 = p[0], d1 = p[1], d2 = p[2];
    const float s = sr[k0 / G];
    float wv[16];
    // 96-bit stream: weights j at bits [6j, 6j+6)
#pragma unroll
    for (int j = 0; j < 16; ++j) {
      const int b = 6 * j;
      uint32_t code;
      if (b + 6 <= 32)
        code = (d0 >> b) & 63;
      else if (b < 32)
        code = ((d0 >> b) | (d1 << (32 - b))) & 63;
      else if (b + 6 <= 64)
        code = (d1 >> (b - 32)) & 63;
      else if (b < 64)
        code = ((d1 >> (b - 32)) | (d2 << (64 - b))) & 63;
      else
        code = (d2 >> (b - 64)) & 63;
      wv[j] = decode(code, f) * s;
    }
#pragma unroll
    for (int m = 0; m < MAXM; ++m) {
      if (m < M) {
        float xv[8], xw[8];
        Vec8<bf16>::load(x + (int64_t)m * K + k0, xv);
        Vec8<bf16>::load(x + (int64_t)m * K + k0 + 8, xw);
        float a = 0.f;
#pragma unroll
        for (int j = 0; j < 8; ++j) a += xv[j] * wv[j] + xw[j] * wv[8 + j];
        acc[m] += a;
      }
    }
  }
#pragma unroll
  for (int m = 0; m < MAXM; ++m) {
    if (m < M) {
      const float r = wave_sum(acc[m]);
      if (lane == 0) y[(int64_t)m * N + n] = (bf16)r;
    }
  }
}

}  // namespace

static bool fpq_fmt_ok(int G, int ebits, int mbits) {
  const int bits = 1 + ebits + mbits;
  return G > 0 && G % 4 == 0 && ebits >= 2 && mbits >= 1 && (bits == 6 || bits == 8 || bits == 12);
}

// x: [n_groups * G] -> q: packed bytes [n_groups * G * bits / 8], scales [n_groups]
HDS_EXPORT int hds_quant_minifloat(int dtype, const void* x, void* q, float* scales, int64_t n_groups, int G,
                                   int ebits, int mbits, int stochastic, int seed, hipStream_t st) {
  if (!fpq_fmt_ok(G, ebits, mbits)) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((n_groups + 3) / 4));
  switch (dtype) {
    case kF32:
      hipLaunchKernelGGL(minifloat_quant_kernel<float>, grid, dim3(256), 0, st, (const float*)x, (uint8_t*)q, scales,
                         n_groups, G, ebits, mbits, stochastic, (uint32_t)seed);
      break;
    case kBF16:
      hipLaunchKernelGGL(minifloat_quant_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)x, (uint8_t*)q, scales,
                         n_groups, G, ebits, mbits, stochastic, (uint32_t)seed);
      break;
    case kF16:
      hipLaunchKernelGGL(minifloat_quant_kernel<_Float16>, grid, dim3(256), 0, st, (const _Float16*)x, (uint8_t*)q,
                         scales, n_groups, G, ebits, mbits, stochastic, (uint32_t)seed);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

HDS_EXPORT int hds_dequant_minifloat(int dtype, const void* q, const float* scales, void* y, int64_t n_groups, int G,
                                     int ebits, int mbits, hipStream_t st) {
  if (!fpq_fmt_ok(G, ebits, mbits)) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((n_groups + 3) / 4));
  switch (dtype) {
    case kF32:
      hipLaunchKernelGGL(minifloat_dequant_kernel<float>, grid, dim3(256), 0, st, (const uint8_t*)q, scales,
                         (float*)y, n_groups, G, ebits, mbits);
      break;
    case kBF16:
      hipLaunchKernelGGL(minifloat_dequant_kernel<bf16>, grid, dim3(256), 0, st, (const uint8_t*)q, scales, (bf16*)y,
                         n_groups, G, ebits, mbits);
      break;
    case kF16:
      hipLaunchKernelGGL(minifloat_dequant_kernel<_Float16>, grid, dim3(256), 0, st, (const uint8_t*)q, scales,
                         (_Float16*)y, n_groups, G, ebits, mbits);
      break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

// x [M, K] bf16 (M <= 8), w packed FP6 [N, K * 3 / 4], scales [N, K / G] -> y [M, N] bf16. K % 16 == 0, G % 16 == 0.
HDS_EXPORT int hds_fp6_gemv(const void* x, const void* w, const float* scales, void* y, int M, int N, int K, int G,
                            int ebits, int mbits, hipStream_t st) {
  if (M < 1 || M > 8 || K % 16 || G % 16 || K % G || 1 + ebits + mbits != 6) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fp6_gemv_kernel<8>, dim3((N + 3) / 4), dim3(256), 0, st, (const bf16*)x, (const uint8_t*)w,
                     scales, (bf16*)y, M, N, K, G, ebits, mbits);
  return hipGetLastError();
}
