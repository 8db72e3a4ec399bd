// Fused softmax cross-entropy over a (chunk of) logits with the gradient written in place.
//
// Capability parity: the reference has no fused training loss kernel (HF Llama runs
// F.cross_entropy on materialised fp32 logits; SURVEY §2.11 "fused ops the new framework
// needs", chunked CE over a 128k vocabulary). Used by ops/cross_entropy.py, which runs the
// LM-head GEMM chunk by chunk so the [T, 128256] logits never exist at once.
//
// One 256-thread workgroup per row: pass 1 is an online (max, sum-exp) sweep with 16-byte
// loads; pass 2 rewrites the row as dlogits = (softmax - onehot) * grad_scale (bf16) in place,
// re-reading a row that was just streamed (256 KB at V=128256: served from L2/Infinity Cache).
#include "hds_common.h"

using namespace hds;

namespace {

template <typename T>
__global__ __launch_bounds__(256) void xent_kernel(T* __restrict__ logits, const int64_t* __restrict__ target,
                                                   float* __restrict__ loss, float* __restrict__ lse_out, int V,
                                                   int64_t ld, int ignore_index, float grad_scale, int write_grad,
                                                   float label_smoothing) {
  __shared__ float red[4];
  const int64_t row = blockIdx.x;
  T* x = logits + row * ld;
  const int64_t tgt = target[row];
  float mx = -INFINITY, se = 0.f, sum_x = 0.f;
  const int nvec = ((ld % 8) == 0) ? V / 8 : 0;  // 16-byte path only for aligned rows
  for (int i = threadIdx.x; i < nvec; i += 256) {
    float v[8];
    Vec8<T>::load(x + i * 8, v);
    float lm = v[0];
#pragma unroll
    for (int j = 1; j < 8; ++j) lm = fmaxf(lm, v[j]);
    if (lm > mx) {
      se *= __expf(mx - lm);
      mx = lm;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      se += __expf(v[j] - mx);
      sum_x += v[j];
    }
  }
  for (int i = nvec * 8 + threadIdx.x; i < V; i += 256) {
    const float v = to_f(x[i]);
    if (v > mx) {
      se *= __expf(mx - v);
      mx = v;
    }
    se += __expf(v - mx);
    sum_x += v;
  }
  const float gmx = block_max<256>(mx, red);
  se = (mx == -INFINITY) ? 0.f : se * __expf(mx - gmx);
  se = block_sum<256>(se, red);
  const float lse = gmx + __logf(se);
  float sx = 0.f;
  if (label_smoothing > 0.f) sx = block_sum<256>(sum_x, red);
  const bool valid = tgt != ignore_index && tgt >= 0 && tgt < V;
  if (threadIdx.x == 0) {
    float l = 0.f;
    if (valid) {
      const float xt = to_f(x[tgt]);
      l = (1.f - label_smoothing) * (lse - xt);
      if (label_smoothing > 0.f) l += label_smoothing * (lse - sx / V);
    }
    loss[row] = l;
    if (lse_out) lse_out[row] = lse;
  }
  if (!write_grad) return;
  __syncthreads();  // everyone has read x[tgt] before it is overwritten
  const float gs = valid ? grad_scale : 0.f;
  const float smooth = label_smoothing / V;
  for (int i = threadIdx.x; i < nvec; i += 256) {
    float v[8];
    Vec8<T>::load(x + i * 8, v);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int col = i * 8 + j;
      float pr = __expf(v[j] - lse);
      float t = (col == tgt) ? (1.f - label_smoothing) : 0.f;
      v[j] = (pr - t - smooth) * gs;
    }
    Vec8<T>::store(x + i * 8, v);
  }
  for (int i = nvec * 8 + threadIdx.x; i < V; i += 256) {
    const float pr = __expf(to_f(x[i]) - lse);
    const float t = (i == tgt) ? (1.f - label_smoothing) : 0.f;
    x[i] = from_f<T>((pr - t - smooth) * gs);
  }
}

}  // namespace

HDS_EXPORT int hds_xent(int dtype, void* logits, const int64_t* target, float* loss, float* lse, int64_t rows, int V,
                        int64_t ld, int ignore_index, float grad_scale, int write_grad, float label_smoothing,
                        hipStream_t st) {
  if (rows <= 0) return 0;
  dim3 grid(rows), block(256);
  if (dtype == kBF16)
    hipLaunchKernelGGL(xent_kernel<bf16>, grid, block, 0, st, (bf16*)logits, target, loss, lse, V, ld, ignore_index,
                       grad_scale, write_grad, label_smoothing);
  else if (dtype == kF32)
    hipLaunchKernelGGL(xent_kernel<float>, grid, block, 0, st, (float*)logits, target, loss, lse, V, ld,
                       ignore_index, grad_scale, write_grad, label_smoothing);
  else if (dtype == kF16)
    hipLaunchKernelGGL(xent_kernel<_Float16>, grid, block, 0, st, (_Float16*)logits, target, loss, lse, V, ld,
                       ignore_index, grad_scale, write_grad, label_smoothing);
  else
    return hipErrorInvalidValue;
  return hipGetLastError();
}
