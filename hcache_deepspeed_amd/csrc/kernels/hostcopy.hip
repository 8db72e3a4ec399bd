// Device -> pinned-host copy by a kernel with a SMALL, fixed number of workgroups.
//
// Why: on this ROCm stack a hipMemcpyAsync device->host runs as the runtime's blit kernel (__amd_rocclr_copyBuffer),
// which spreads over as many workgroups as the copy has chunks. Activation spills overlap compute by design, and a
// wide blit grid takes CUs from the FlashAttention / GEMM kernels it runs beside: in a 32k-token step that spills
// ~25 GB, the forward stretched from 708 to 1103 ms while the GPU stayed 99.8 % busy (profiles/r4/). PCIe (~56 GB/s),
// not the CU count, bounds the copy, so a handful of workgroups streaming 16-byte vectors saturate the link; they hold
// few registers and no LDS, so the compute kernels' waves keep co-residing on those CUs.
//
// The host buffer is hipHostMalloc memory mapped into the GPU address space; stores are non-temporal (no L2
// allocation for data the GPU never reads back) and each thread ends with a system-scope fence, so the bytes are in
// host memory when the stream's completion event fires.
#include "hds_common.h"

namespace {
using namespace hds;

constexpr int kThreads = 256;
constexpr int kUnroll = 4;

__global__ __launch_bounds__(kThreads) void d2h_kernel(const u32x4* __restrict__ src, u32x4* __restrict__ dst,
                                                        int64_t nvec, const uint8_t* __restrict__ src_tail,
                                                        uint8_t* __restrict__ dst_tail, int tail) {
  const int64_t stride = (int64_t)gridDim.x * kThreads;
  int64_t i = (int64_t)blockIdx.x * kThreads + threadIdx.x;
  for (; i + (kUnroll - 1) * stride < nvec; i += kUnroll * stride) {
    u32x4 v[kUnroll];
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) v[u] = __builtin_nontemporal_load(src + i + u * stride);
#pragma unroll
    for (int u = 0; u < kUnroll; ++u) __builtin_nontemporal_store(v[u], dst + i + u * stride);
  }
  for (; i < nvec; i += stride) __builtin_nontemporal_store(__builtin_nontemporal_load(src + i), dst + i);
  if (blockIdx.x == 0 && threadIdx.x < tail) dst_tail[threadIdx.x] = src_tail[threadIdx.x];
  __threadfence_system();
}

}  // namespace

// dst: pinned host pointer (device-accessible), src: device pointer; both 16-byte aligned. n_wg workgroups.
HDS_EXPORT int hds_copy_d2h(void* dst, const void* src, int64_t nbytes, int n_wg, hipStream_t st) {
  if (nbytes <= 0) return hipSuccess;
  if ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) % 16 || n_wg < 1)
    return hipErrorInvalidValue;
  const int64_t nvec = nbytes / 16;
  const int tail = (int)(nbytes - nvec * 16);
  if (tail > kThreads) return hipErrorInvalidValue;
  int64_t need = (nvec + kThreads - 1) / kThreads;
  const int grid = (int)(need < n_wg ? (need < 1 ? 1 : need) : n_wg);
  hipLaunchKernelGGL(d2h_kernel, dim3(grid), dim3(kThreads), 0, st, reinterpret_cast<const u32x4*>(src),
                     reinterpret_cast<u32x4*>(dst), nvec, static_cast<const uint8_t*>(src) + nvec * 16,
                     static_cast<uint8_t*>(dst) + nvec * 16, tail);
  return hipGetLastError();
}
