// Rotary position embedding (rotate-half / NeoX-Llama form and interleaved GPT-J form),
// forward and backward, applied IN PLACE on a packed QKV activation.
//
// Capability parity: reference csrc/transformer/inference/csrc/apply_rotary_pos_emb.cu
// (`apply_rotary_pos_half`) and the rotary half of
// deepspeed/inference/v2/kernels/ragged_ops/linear_blocked_kv_rotary (K31). The reference
// only has inference RoPE; this file also provides the backward (inverse rotation) used by
// training.
//
// Layout: x is [T, n_heads_total, D] with a row stride (in elements) of `row_stride`; the first
// `n_rot_heads` heads of every token are rotated (q heads followed by k heads when this is the
// fused QKV GEMM output), the rest (v) are untouched. This lets the training path run RoPE on
// the QKV GEMM output without any split/transpose copies: FlashAttention then reads q/k/v as
// strided views of the same buffer.
//
// cos/sin come from a host-precomputed fp32 table [max_pos, rot_dim/2] (no on-device trig:
// keeps the kernel memory-bound, cdna_hip_programming Appendix B "Element-wise").
#include "hds_common.h"

using namespace hds;

namespace {

// One thread handles 8 rotation pairs (16 bf16 values) of one head.
template <typename T, bool INTERLEAVED>
__global__ __launch_bounds__(256) void rope_kernel(T* __restrict__ x, const float* __restrict__ cos_t,
                                                   const float* __restrict__ sin_t, const int* __restrict__ pos_ids,
                                                   int64_t n_tok, int n_rot_heads, int head_dim, int rot_dim,
                                                   int64_t row_stride, int seq_len, int pos_offset, float sign) {
  const int half = rot_dim / 2;
  const int groups_per_head = half / 8;  // 8 pairs per thread
  const int64_t per_tok = (int64_t)n_rot_heads * groups_per_head;
  const int64_t total = n_tok * per_tok;
  for (int64_t idx = (int64_t)blockIdx.x * 256 + threadIdx.x; idx < total; idx += (int64_t)gridDim.x * 256) {
    const int64_t t = idx / per_tok;
    const int rem = (int)(idx - t * per_tok);
    const int hd = rem / groups_per_head;
    const int g = rem - hd * groups_per_head;
    const int pos = pos_ids ? pos_ids[t] : (int)(t % seq_len) + pos_offset;
    const float* cr = cos_t + (int64_t)pos * half + g * 8;
    const float* sr = sin_t + (int64_t)pos * half + g * 8;
    float c[8], s[8];
    Vec8<float>::load(cr, c);
    Vec8<float>::load(sr, s);
    T* base = x + t * row_stride + (int64_t)hd * head_dim;
    if constexpr (!INTERLEAVED) {
      float a[8], b[8];
      Vec8<T>::load(base + g * 8, a);
      Vec8<T>::load(base + half + g * 8, b);
      float oa[8], ob[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const float sj = sign * s[j];
        oa[j] = a[j] * c[j] - b[j] * sj;
        ob[j] = b[j] * c[j] + a[j] * sj;
      }
      Vec8<T>::store(base + g * 8, oa);
      Vec8<T>::store(base + half + g * 8, ob);
    } else {
      // pairs (2i, 2i+1): thread g covers elements [16g, 16g+16)
      float v0[8], v1[8];
      Vec8<T>::load(base + g * 16, v0);
      Vec8<T>::load(base + g * 16 + 8, v1);
      float o0[8], o1[8];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const float s0 = sign * s[j], s1 = sign * s[j + 4];
        o0[2 * j] = v0[2 * j] * c[j] - v0[2 * j + 1] * s0;
        o0[2 * j + 1] = v0[2 * j + 1] * c[j] + v0[2 * j] * s0;
        o1[2 * j] = v1[2 * j] * c[j + 4] - v1[2 * j + 1] * s1;
        o1[2 * j + 1] = v1[2 * j + 1] * c[j + 4] + v1[2 * j] * s1;
      }
      Vec8<T>::store(base + g * 16, o0);
      Vec8<T>::store(base + g * 16 + 8, o1);
    }
  }
}

}  // namespace

// sign = +1 forward, -1 backward (inverse rotation of the incoming gradient)
HDS_EXPORT int hds_rope(int dtype, int interleaved, void* x, const float* cos_t, const float* sin_t,
                        const int* pos_ids, int64_t n_tok, int n_rot_heads, int head_dim, int rot_dim,
                        int64_t row_stride, int seq_len, int pos_offset, float sign, hipStream_t st) {
  if (rot_dim % 16 || rot_dim > head_dim) return hipErrorInvalidValue;
  const int64_t work = n_tok * n_rot_heads * (rot_dim / 16);
  dim3 grid(stream_grid(work, 256, 4096)), block(256);
#define L(T, I)                                                                                               \
  hipLaunchKernelGGL((rope_kernel<T, I>), grid, block, 0, st, (T*)x, cos_t, sin_t, pos_ids, n_tok, n_rot_heads, \
                     head_dim, rot_dim, row_stride, seq_len, pos_offset, sign)
  if (dtype == kBF16) {
    if (interleaved) L(bf16, true); else L(bf16, false);
  } else if (dtype == kF32) {
    if (interleaved) L(float, true); else L(float, false);
  } else if (dtype == kF16) {
    if (interleaved) L(_Float16, true); else L(_Float16, false);
  } else {
    return hipErrorInvalidValue;
  }
#undef L
  return hipGetLastError();
}
