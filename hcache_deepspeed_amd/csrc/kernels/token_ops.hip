// Token-routing kernels for random layerwise token dropping (random-LTD) and channels-last bias fusions for
// diffusion UNet / VAE blocks.
//
// Capability parity:
//   * csrc/random_ltd/{gather_scatter.cu,token_sort.cu,slice_attn_masks.cu}:
//     token_sort_ (sort the sampled indices of every (layer, batch) row), token_gather / token_scatter
//     ([B, S, H] <-> [B, R, H] rows), slice_gpt_mask / slice_bert_mask.
//   * csrc/spatial/csrc/opt_bias_add.cu (N19): nhwc_bias_add, nhwc_bias_add_add, nhwc_bias_add_bias_add.
// Design: every row moves with 16-byte vectors (8 x bf16 per lane); the sort is one LDS bitonic network per row
// (a workgroup per row, up to 16384 keys = 64 KB of the 160 KB LDS); mask slicing gathers rows and columns in one
// pass. All are bandwidth kernels, so the grids have one workgroup per row (B * R >> 256 for real shapes).
#include "hds_common.h"

using namespace hds;

namespace {

// out[b, r, :] = x[b, idx[b, r], :]   (x: [B, S, H], idx: [B, R] int32)
template <typename T>
__global__ __launch_bounds__(256) void token_gather_kernel(const T* __restrict__ x, const int* __restrict__ idx,
                                                           T* __restrict__ out, int S, int R, int H) {
  const int row = blockIdx.x;  // b * R + r
  const int b = row / R;
  const int s = idx[row];
  if (s < 0 || s >= S) return;
  const T* src = x + ((int64_t)b * S + s) * H;
  T* dst = out + (int64_t)row * H;
  for (int c = threadIdx.x * 8; c < H; c += 256 * 8) {
    float v[8];
    Vec8<T>::load(src + c, v);
    Vec8<T>::store(dst + c, v);
  }
}

// out[b, idx[b, r], :] = part[b, r, :]   (out already holds the full [B, S, H] input)
template <typename T>
__global__ __launch_bounds__(256) void token_scatter_kernel(const T* __restrict__ part, const int* __restrict__ idx,
                                                            T* __restrict__ out, int S, int R, int H) {
  const int row = blockIdx.x;
  const int b = row / R;
  const int s = idx[row];
  if (s < 0 || s >= S) return;
  const T* src = part + (int64_t)row * H;
  T* dst = out + ((int64_t)b * S + s) * H;
  for (int c = threadIdx.x * 8; c < H; c += 256 * 8) {
    float v[8];
    Vec8<T>::load(src + c, v);
    Vec8<T>::store(dst + c, v);
  }
}

// Ascending in-place sort of each row of `keys` [rows, n] (n <= 16384) with an LDS bitonic network.
__global__ __launch_bounds__(1024) void token_sort_kernel(int* __restrict__ keys, int n, int npow2) {
  extern __shared__ int sk[];
  int* row = keys + (int64_t)blockIdx.x * n;
  for (int i = threadIdx.x; i < npow2; i += blockDim.x) sk[i] = i < n ? row[i] : 0x7fffffff;
  __syncthreads();
  for (int k = 2; k <= npow2; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < npow2; i += blockDim.x) {
        const int p = i ^ j;
        if (p > i) {
          const int a = sk[i], c = sk[p];
          const bool up = (i & k) == 0;
          if ((a > c) == up) {
            sk[i] = c;
            sk[p] = a;
          }
        }
      }
      __syncthreads();
    }
  }
  for (int i = threadIdx.x; i < n; i += blockDim.x) row[i] = sk[i];
}

// out[l, b, i, j] = mask[b', idx[l, b, i], idx[l, b, j]]  (mask [Bm, S, S], Bm in {1, B}; out [L, B, R, R])
template <typename T>
__global__ __launch_bounds__(256) void slice_mask_kernel(const T* __restrict__ mask, const int* __restrict__ idx,
                                                         T* __restrict__ out, int B, int Bm, int S, int R) {
  const int row = blockIdx.x;  // (l * B + b) * R + i
  const int lb = row / R, i = row - lb * R;
  const int b = lb % B;
  const int* ix = idx + (int64_t)lb * R;
  const T* src = mask + ((int64_t)(Bm == 1 ? 0 : b) * S + ix[i]) * S;
  T* dst = out + (int64_t)row * R;
  for (int j = threadIdx.x; j < R; j += 256) dst[j] = src[ix[j]];
}

// Channels-last bias fusions over [N*H*W, C] rows (C % 8 == 0):
//   mode 0: out = a + bias;  mode 1: out = a + bias + other;  mode 2: out = a + bias + other + other_bias
template <typename T>
__global__ __launch_bounds__(256) void nhwc_bias_add_kernel(const T* __restrict__ a, const T* __restrict__ bias,
                                                            const T* __restrict__ other,
                                                            const T* __restrict__ other_bias, T* __restrict__ out,
                                                            int64_t n_vec, int C, int mode) {
  const int cv = C / 8;
  for (int64_t v = (int64_t)blockIdx.x * 256 + threadIdx.x; v < n_vec; v += (int64_t)gridDim.x * 256) {
    const int c = (int)(v % cv) * 8;
    float x[8], bb[8];
    Vec8<T>::load(a + v * 8, x);
    Vec8<T>::load(bias + c, bb);
#pragma unroll
    for (int i = 0; i < 8; ++i) x[i] += bb[i];
    if (mode >= 1) {
      float o[8];
      Vec8<T>::load(other + v * 8, o);
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] += o[i];
    }
    if (mode == 2) {
      float ob[8];
      Vec8<T>::load(other_bias + c, ob);
#pragma unroll
      for (int i = 0; i < 8; ++i) x[i] += ob[i];
    }
    Vec8<T>::store(out + v * 8, x);
  }
}

// Embedding weight gradient, accumulated in place: grad[id, :] += sum of dy[t, :] over tokens t with ids[t] == id.
// ``sorted``/``perm`` come from a stable sort of the ids, so every id's tokens are one contiguous run and the
// first position of each run owns the row: one read-modify-write per touched row, fp32 sums in a fixed
// (token) order -- deterministic, no atomics, and no dense [V, D] temporary (the sort-based framework path
// materialises and then adds one). One workgroup per sorted position; non-leading positions exit at once.
template <typename T>
__global__ __launch_bounds__(256) void embed_bwd_kernel(const T* __restrict__ dy, const int64_t* __restrict__ sorted,
                                                        const int64_t* __restrict__ perm, T* __restrict__ grad,
                                                        int64_t n, int D, int64_t V, int64_t pad_idx) {
  const int64_t i = blockIdx.x;
  const int64_t id = sorted[i];
  if ((i > 0 && sorted[i - 1] == id) || id == pad_idx || id < 0 || id >= V) return;
  int64_t end = i + 1;
  while (end < n && sorted[end] == id) ++end;
  T* g = grad + id * (int64_t)D;
  for (int c = threadIdx.x * 8; c < D; c += 256 * 8) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int64_t j = i; j < end; ++j) {
      float v[8];
      Vec8<T>::load(dy + perm[j] * (int64_t)D + c, v);
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += v[e];
    }
    float old[8];
    Vec8<T>::load(g + c, old);
#pragma unroll
    for (int e = 0; e < 8; ++e) old[e] += acc[e];
    Vec8<T>::store(g + c, old);
  }
}

#define HDS_TOK_DISPATCH(dtype, ...)                  \
  switch (dtype) {                                    \
    case kF32: { typedef float T; __VA_ARGS__; break; }    \
    case kBF16: { typedef bf16 T; __VA_ARGS__; break; }    \
    case kF16: { typedef _Float16 T; __VA_ARGS__; break; } \
    default: return (int)hipErrorInvalidValue;       \
  }

}  // namespace

HDS_EXPORT int hds_token_gather(int dtype, const void* x, const int* idx, void* out, int B, int S, int R, int H,
                                hipStream_t st) {
  if (H % 8 || B <= 0 || R <= 0) return (int)hipErrorInvalidValue;
  HDS_TOK_DISPATCH(dtype, hipLaunchKernelGGL(token_gather_kernel<T>, dim3(B * R), dim3(256), 0, st,
                                             (const T*)x, idx, (T*)out, S, R, H));
  return (int)hipGetLastError();
}

HDS_EXPORT int hds_token_scatter(int dtype, const void* part, const int* idx, void* out, int B, int S, int R, int H,
                                 hipStream_t st) {
  if (H % 8 || B <= 0 || R <= 0) return (int)hipErrorInvalidValue;
  HDS_TOK_DISPATCH(dtype, hipLaunchKernelGGL(token_scatter_kernel<T>, dim3(B * R), dim3(256), 0, st,
                                             (const T*)part, idx, (T*)out, S, R, H));
  return (int)hipGetLastError();
}

HDS_EXPORT int hds_token_sort(int* keys, int rows, int n, hipStream_t st) {
  if (n <= 0 || n > 16384 || rows <= 0) return (int)hipErrorInvalidValue;
  int p = 1;
  while (p < n) p <<= 1;
  const int nt = p < 1024 ? (p < 64 ? 64 : p) : 1024;
  hipLaunchKernelGGL(token_sort_kernel, dim3(rows), dim3(nt), p * sizeof(int), st, keys, n, p);
  return (int)hipGetLastError();
}

HDS_EXPORT int hds_slice_mask(int dtype, const void* mask, const int* idx, void* out, int L, int B, int Bm, int S,
                              int R, hipStream_t st) {
  if (L <= 0 || B <= 0 || R <= 0 || (Bm != 1 && Bm != B)) return (int)hipErrorInvalidValue;
  HDS_TOK_DISPATCH(dtype, hipLaunchKernelGGL(slice_mask_kernel<T>, dim3(L * B * R), dim3(256), 0, st,
                                             (const T*)mask, idx, (T*)out, B, Bm, S, R));
  return (int)hipGetLastError();
}

HDS_EXPORT int hds_nhwc_bias_add(int dtype, const void* a, const void* bias, const void* other, const void* other_bias,
                                 void* out, int64_t rows, int C, int mode, hipStream_t st) {
  if (C % 8 || rows <= 0 || mode < 0 || mode > 2) return (int)hipErrorInvalidValue;
  const int64_t n_vec = rows * (C / 8);
  const int64_t want = (n_vec + 255) / 256;
  const int grid = (int)(want < 256 * 32 ? want : 256 * 32);
  HDS_TOK_DISPATCH(dtype, hipLaunchKernelGGL(nhwc_bias_add_kernel<T>, dim3(grid), dim3(256), 0, st, (const T*)a,
                                             (const T*)bias, (const T*)other, (const T*)other_bias, (T*)out, n_vec,
                                             C, mode));
  return (int)hipGetLastError();
}

HDS_EXPORT int hds_embed_bwd(int dtype, const void* dy, const int64_t* sorted, const int64_t* perm, void* grad,
                             int64_t n, int D, int64_t V, int64_t pad_idx, hipStream_t st) {
  if (n <= 0) return 0;
  if (D % 8 || n > 0x7fffffff) return (int)hipErrorInvalidValue;
  HDS_TOK_DISPATCH(dtype, hipLaunchKernelGGL(embed_bwd_kernel<T>, dim3((unsigned)n), dim3(256), 0, st, (const T*)dy,
                                             sorted, perm, (T*)grad, n, D, V, pad_idx));
  return (int)hipGetLastError();
}
