// Device -> pinned-host copy by a kernel with a SMALL, fixed number of workgroups (opt-in: ops/hostcopy.py HDS_D2H_WG).
//
// On this ROCm stack a hipMemcpyAsync device->host runs as the runtime's blit kernel (__amd_rocclr_copyBuffer), which
// spreads over as many workgroups as the copy has chunks and takes CUs from the FlashAttention / GEMM kernels an
// activation spill overlaps: a 32k-token step spilling ~25 GB stretched its forward from 708 to 1103 ms at 99.8 % GPU
// busy. PCIe (~56 GB/s), not the CU count, bounds the copy, so few workgroups suffice. Measured in situ, though, the
// runtime blit LIMITED to 8-32 workgroups (DEBUG_CLR_LIMIT_BLIT_WG, set by the package) cost ~0.01 ms of forward per
// spilled GB and this kernel ~14 (profiles/r4/copy_engine_ab_r4f.txt), so the limited blit is the default.
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

// ---------------------------------------------------------------------------------------------------------------------
// HCache latents inside a captured decode graph (inference/v2/model.py _DecodeGraph): every layer's latent rows are
// stored into a DEVICE ring at a slot read from device memory, so the graph (fixed addresses) writes a different slot
// on every replay; a one-thread kernel at the end of the graph advances the slot. The host drains filled halves of the
// ring with one D2H each on the copy stream instead of 32 per-layer D2H copies per token.
namespace {

// rows x row_bytes from src (row stride src_stride bytes) -> dst_base + slot * slot_stride (contiguous rows), in
// VT-sized pieces: 16 B when every row and stride is a multiple of 16, else 4 B (the packed fp8 / int8 latents are
// H + 4 and H + H/32 bytes per row)
template <typename VT>
__global__ __launch_bounds__(256) void latent_slot_store_kernel(const char* __restrict__ src, int64_t src_stride,
                                                                char* __restrict__ dst_base,
                                                                const int* __restrict__ slot, int64_t slot_stride,
                                                                int rows, int64_t row_bytes) {
  char* dst = dst_base + (int64_t)(*slot) * slot_stride;
  const int64_t nvec = row_bytes / (int64_t)sizeof(VT);
  const int64_t total = (int64_t)rows * nvec;
  for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < total; i += (int64_t)gridDim.x * 256) {
    const int64_t r = i / nvec, v = i - r * nvec;
    *reinterpret_cast<VT*>(dst + r * row_bytes + v * (int64_t)sizeof(VT)) =
        *reinterpret_cast<const VT*>(src + r * src_stride + v * (int64_t)sizeof(VT));
  }
}

__global__ void slot_advance_kernel(int* slot, int mod) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    const int s = *slot + 1;
    *slot = s >= mod ? 0 : s;
  }
}

}  // namespace

HDS_EXPORT int hds_latent_slot_store(const void* src, int64_t src_stride, void* dst_base, const int* slot,
                                     int64_t slot_stride, int rows, int64_t row_bytes, hipStream_t st) {
  if (rows <= 0 || row_bytes <= 0) return hipSuccess;
  const uintptr_t al = reinterpret_cast<uintptr_t>(src) | reinterpret_cast<uintptr_t>(dst_base) |
                       (uintptr_t)row_bytes | (uintptr_t)src_stride | (uintptr_t)slot_stride;
  if (al & 3) return hipErrorInvalidValue;
  const bool wide = (al & 15) == 0;
  const int64_t total = (int64_t)rows * (row_bytes / (wide ? 16 : 4));
  int64_t grid = (total + 255) / 256;
  if (grid > 1024) grid = 1024;
  if (wide)
    hipLaunchKernelGGL(latent_slot_store_kernel<u32x4>, dim3((unsigned)grid), dim3(256), 0, st,
                       static_cast<const char*>(src), src_stride, static_cast<char*>(dst_base), slot, slot_stride, rows,
                       row_bytes);
  else
    hipLaunchKernelGGL(latent_slot_store_kernel<uint32_t>, dim3((unsigned)grid), dim3(256), 0, st,
                       static_cast<const char*>(src), src_stride, static_cast<char*>(dst_base), slot, slot_stride, rows,
                       row_bytes);
  return hipGetLastError();
}

HDS_EXPORT int hds_slot_advance(int* slot, int mod, hipStream_t st) {
  if (mod < 1) return hipErrorInvalidValue;
  hipLaunchKernelGGL(slot_advance_kernel, dim3(1), dim3(64), 0, st, slot, mod);
  return hipGetLastError();
}
