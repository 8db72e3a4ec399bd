// Symmetric-memory collectives over xGMI: one-shot all-reduce, direct-read all-gather and reduce-scatter between the
// GPUs of one node, for the small / latency-bound collectives where a ring's 2(W-1) steps dominate.
//
// Reference parity: DeepCompile's SymmetricMemory all-gather (csrc/compile/z3.cpp:91-110, compile config
// ``symmetric_memory``) and the one-shot small-message all-reduce SURVEY.md §5.8 asks for. The reference rides
// torch's SymmetricMemory over NVLink; here every rank allocates ONE uncached device buffer (hipExtMallocWithFlags
// hipDeviceMallocUncached: stores bypass L2, so a peer reading it over xGMI never sees a stale line), exports it
// with hipIpcGetMemHandle, and maps every peer's buffer (hipIpcOpenMemHandle). xGMI is point-to-point, so a kernel
// that reads all W-1 peers at once drives all 7 links concurrently instead of one ring neighbour per step.
//
// Buffer layout (per rank): flags [kMaxRanks][kMaxBlocks] u32 | error word | data parity 0 [cap] | data parity 1.
// Protocol of one collective with epoch e (host counter, same on every rank; parity = e & 1):
//   block b copies its chunk of the input into its OWN data[parity], fences at system scope, then stores e into
//   flags[rank][b] of every peer's buffer; it then waits until its own flags[src][b] >= e for every peer src and
//   reads chunk b of each peer's data[parity]. Per-block flags need no grid-wide barrier (every rank splits the
//   message into the same blocks). Two parities make reuse safe: a rank rewrites data[parity] only at epoch e+2,
//   after every peer signalled e+1, which a peer does only after its epoch-e kernel (all reads of e) has finished.
// Every wait is bounded (kSpinMax polls): a missing peer sets the error word and the grid still drains -- no wave can
// spin forever. A timeout is FATAL for the buffer: the error word is sticky (every later collective on it re-reports
// it), and it is also written to two status words the caller passes: a host-mapped pinned word the host polls at no
// cost before every call (comm/symmetric.py raises), and an optional device flag the ZeRO optimizer folds into its
// step's skip flag, so a step whose collective read stale peer data never updates the weights.
#include <cstring>

#include "hds_common.h"

namespace {
using namespace hds;

constexpr int kMaxRanks = 8;
constexpr int kMaxBlocks = 256;
constexpr int64_t kFlagBytes = (int64_t)kMaxRanks * kMaxBlocks * 4;
constexpr int64_t kErrOff = kFlagBytes;
constexpr int64_t kDataOff = kFlagBytes + 256;
constexpr int kSpinMax = 1 << 22;
constexpr int kThreads = 512;

struct SymmArgs {
  char* base[kMaxRanks];  // every rank's mapped buffer (own included)
  int rank, world;
  int64_t cap;            // bytes per parity
  uint32_t epoch;
  const void* in;
  void* out;
  int64_t n;              // all-reduce: elements; all-gather: bytes per rank; reduce-scatter: elements per rank
  uint32_t* host_status;  // host-mapped pinned word (may be null): error code on timeout
  int32_t* dev_status;    // device flag (may be null): error code on timeout
};

__device__ __forceinline__ uint32_t* err_ptr(char* base) { return reinterpret_cast<uint32_t*>(base + kErrOff); }

__device__ __forceinline__ void report(const SymmArgs& a, uint32_t code) {
  __hip_atomic_store(err_ptr(a.base[a.rank]), code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (a.host_status) __hip_atomic_store(a.host_status, code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  if (a.dev_status) __hip_atomic_store(a.dev_status, (int32_t)code, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// a rank that timed out poisons every peer's error word (kPeerErr | 1 + its rank): the peers' next collective on the
// buffer fails at once instead of waiting for a rank that has left the protocol, so EVERY rank reaches the host-side
// agreement (comm/symmetric.py) before any of them switches to RCCL
constexpr uint32_t kPeerErr = 0x100u;

__device__ __forceinline__ void poison_peers(const SymmArgs& a) {
  for (int r = 0; r < a.world; ++r)
    if (r != a.rank)
      __hip_atomic_store(err_ptr(a.base[r]), kPeerErr | (1u + (uint32_t)a.rank), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ uint32_t* flag_ptr(char* base, int src, int blk) {
  return reinterpret_cast<uint32_t*>(base) + src * kMaxBlocks + blk;
}

__device__ __forceinline__ char* data_ptr(const SymmArgs& a, int r) {
  return a.base[r] + kDataOff + (int64_t)(a.epoch & 1u) * a.cap;
}

// publish this block's chunk (all threads' stores) to every peer, then wait for every peer's chunk
__device__ __forceinline__ void exchange(const SymmArgs& a) {
  __threadfence_system();
  __syncthreads();
  const int t = threadIdx.x, b = blockIdx.x;
  if (t < a.world && t != a.rank) {
    char* peer = nullptr;
#pragma unroll
    for (int r = 0; r < kMaxRanks; ++r)
      if (r == t) peer = a.base[r];
    __hip_atomic_store(flag_ptr(peer, a.rank, b), a.epoch, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    uint32_t* mine = flag_ptr(a.base[a.rank], t, b);
    // a failed (or poisoned) buffer does not wait: its result is invalid either way, and the sticky word is
    // re-reported below
    const bool failed = __hip_atomic_load(err_ptr(a.base[a.rank]), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
    bool ok = false;
    for (int it = 0; !failed && it < kSpinMax; ++it) {
      const uint32_t v = __hip_atomic_load(mine, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_SYSTEM);
      if ((int32_t)(v - a.epoch) >= 0) {
        ok = true;
        break;
      }
      __builtin_amdgcn_s_sleep(2);
    }
    if (!ok && !failed) {
      report(a, 1u + (uint32_t)t);
      poison_peers(a);
    }
  }
  if (t == 0) {  // a buffer that timed out before stays failed: re-report, so no later step trusts it
    const uint32_t prev = __hip_atomic_load(reinterpret_cast<uint32_t*>(a.base[a.rank] + kErrOff), __ATOMIC_RELAXED,
                                            __HIP_MEMORY_SCOPE_SYSTEM);
    if (prev != 0) report(a, prev);
  }
  __syncthreads();
  __threadfence_system();
}

// raw copy of one 8-element vector (16 B for 16-bit types, 32 B for fp32)
template <typename T>
__device__ __forceinline__ void copy8(T* dst, const T* src) {
#pragma unroll
  for (int j = 0; j < (int)(8 * sizeof(T) / 16); ++j)
    reinterpret_cast<u32x4*>(dst)[j] = reinterpret_cast<const u32x4*>(src)[j];
}

__device__ __forceinline__ void block_range(int64_t nvec, int64_t& lo, int64_t& hi) {
  const int64_t per = (nvec + gridDim.x - 1) / gridDim.x;
  lo = (int64_t)blockIdx.x * per;
  hi = lo + per < nvec ? lo + per : nvec;
}

// all-reduce (sum) of n elements (n % 8 == 0), accumulated in fp32, out may alias in
template <typename T>
__global__ __launch_bounds__(kThreads) void symm_allreduce_kernel(SymmArgs a) {
  int64_t lo, hi;
  block_range(a.n / 8, lo, hi);
  const T* in = reinterpret_cast<const T*>(a.in);
  T* mine = reinterpret_cast<T*>(data_ptr(a, a.rank));
  for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) copy8(mine + 8 * i, in + 8 * i);
  exchange(a);
  T* out = reinterpret_cast<T*>(a.out);
  for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    // fixed rank order: every rank computes the bit-identical sum
    for (int r = 0; r < a.world; ++r) {
      float v[8];
      Vec8<T>::load(reinterpret_cast<const T*>(data_ptr(a, r)) + 8 * i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
    Vec8<T>::store(out + 8 * i, acc);
  }
}

// all-gather of n bytes per rank (n % 16 == 0): out[r * n ...] = rank r's input
__global__ __launch_bounds__(kThreads) void symm_allgather_kernel(SymmArgs a) {
  int64_t lo, hi;
  block_range(a.n / 16, lo, hi);
  const u32x4* in = reinterpret_cast<const u32x4*>(a.in);
  u32x4* mine = reinterpret_cast<u32x4*>(data_ptr(a, a.rank));
  u32x4* out = reinterpret_cast<u32x4*>(a.out);
  const int64_t nv = a.n / 16;
  for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) {
    const u32x4 v = in[i];
    mine[i] = v;
    out[(int64_t)a.rank * nv + i] = v;
  }
  exchange(a);
  for (int d = 1; d < a.world; ++d) {
    const int r = (a.rank + d) % a.world;  // staggered source order spreads the first reads over the links
    const u32x4* src = reinterpret_cast<const u32x4*>(data_ptr(a, r));
    for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) out[(int64_t)r * nv + i] = src[i];
  }
}

// reduce-scatter (sum): input [world * n] elements, out[n] = sum over ranks of their input segment `rank`
template <typename T>
__global__ __launch_bounds__(kThreads) void symm_reduce_scatter_kernel(SymmArgs a) {
  int64_t lo, hi;
  block_range(a.n / 8, lo, hi);
  const T* in = reinterpret_cast<const T*>(a.in);
  T* mine = reinterpret_cast<T*>(data_ptr(a, a.rank));
  for (int s = 0; s < a.world; ++s)
    for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) {
      const int64_t e = (int64_t)s * a.n + 8 * i;
      copy8(mine + e, in + e);
    }
  exchange(a);
  T* out = reinterpret_cast<T*>(a.out);
  for (int64_t i = lo + threadIdx.x; i < hi; i += kThreads) {
    float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int r = 0; r < a.world; ++r) {
      float v[8];
      Vec8<T>::load(reinterpret_cast<const T*>(data_ptr(a, r)) + (int64_t)a.rank * a.n + 8 * i, v);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += v[j];
    }
    Vec8<T>::store(out + 8 * i, acc);
  }
}

int blocks_for(int64_t nvec) {
  int64_t nb = (nvec + 2 * kThreads - 1) / (2 * kThreads);
  return (int)(nb < 1 ? 1 : (nb > kMaxBlocks ? kMaxBlocks : nb));
}

bool make_args(SymmArgs& a, const int64_t* bases, int rank, int world, int64_t cap, uint32_t epoch, const void* in,
               void* out, int64_t n, void* host_status, void* dev_status) {
  a.host_status = static_cast<uint32_t*>(host_status);
  a.dev_status = static_cast<int32_t*>(dev_status);
  if (world < 1 || world > kMaxRanks || rank < 0 || rank >= world || !in || !out || epoch == 0) return false;
  for (int r = 0; r < kMaxRanks; ++r) a.base[r] = r < world ? reinterpret_cast<char*>(bases[r]) : nullptr;
  for (int r = 0; r < world; ++r)
    if (!a.base[r]) return false;
  a.rank = rank;
  a.world = world;
  a.cap = cap;
  a.epoch = epoch;
  a.in = in;
  a.out = out;
  a.n = n;
  return true;
}

}  // namespace

HDS_EXPORT int hds_symm_header_bytes() { return (int)kDataOff; }

// one uncached device buffer of kDataOff + 2 * cap bytes, zeroed, and its 64-byte IPC handle
HDS_EXPORT int hds_symm_alloc(int64_t cap, void** ptr, void* handle) {
  if (cap <= 0 || cap % 16) return hipErrorInvalidValue;
  const size_t bytes = (size_t)(kDataOff + 2 * cap);
  hipError_t e = hipExtMallocWithFlags(ptr, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return e;
  e = hipMemset(*ptr, 0, bytes);
  if (e != hipSuccess) return e;
  e = hipDeviceSynchronize();
  if (e != hipSuccess) return e;
  return hipIpcGetMemHandle(reinterpret_cast<hipIpcMemHandle_t*>(handle), *ptr);
}

HDS_EXPORT int hds_symm_open(const void* handle, void** ptr) {
  hipIpcMemHandle_t h;
  std::memcpy(&h, handle, sizeof(h));
  return hipIpcOpenMemHandle(ptr, h, hipIpcMemLazyEnablePeerAccess);
}

HDS_EXPORT int hds_symm_close(void* ptr) { return hipIpcCloseMemHandle(ptr); }

HDS_EXPORT int hds_symm_free(void* ptr) { return hipFree(ptr); }

// host-mapped, coherent pinned status word (device stores reach the host without a synchronize)
HDS_EXPORT int hds_symm_status_alloc(void** ptr) {
  hipError_t e = hipHostMalloc(ptr, 64, hipHostMallocMapped | hipHostMallocCoherent);
  if (e != hipSuccess) return e;
  std::memset(*ptr, 0, 64);
  return hipSuccess;
}

HDS_EXPORT int hds_symm_status_free(void* ptr) { return hipHostFree(ptr); }

// clear the sticky error word of this rank's buffer (after every rank abandoned the buffer's epochs)
HDS_EXPORT int hds_symm_clear_error(void* base) {
  return hipMemset(static_cast<char*>(base) + kErrOff, 0, 4);
}

// error word of this rank's buffer: 0, or 1 + the peer whose flag never arrived
HDS_EXPORT int hds_symm_error(void* base) {
  uint32_t v = 0;
  hipError_t e = hipMemcpy(&v, static_cast<char*>(base) + kErrOff, 4, hipMemcpyDeviceToHost);
  return e != hipSuccess ? -(int)e : (int)v;
}

// dtype: 0 fp32, 1 bf16, 2 fp16 (ops/native.py dt())
HDS_EXPORT int hds_symm_allreduce(const int64_t* bases, int rank, int world, int64_t cap, uint32_t epoch,
                                  const void* in, void* out, int64_t n, int dtype, void* host_status, void* dev_status,
                                  hipStream_t st) {
  SymmArgs a;
  const int64_t es = dtype == 0 ? 4 : 2;
  if (!make_args(a, bases, rank, world, cap, epoch, in, out, n, host_status, dev_status) || n % 8 || n * es > cap) return hipErrorInvalidValue;
  const dim3 grid(blocks_for(n / 8));
  switch (dtype) {
    case 0: hipLaunchKernelGGL(symm_allreduce_kernel<float>, grid, dim3(kThreads), 0, st, a); break;
    case 1: hipLaunchKernelGGL(symm_allreduce_kernel<bf16>, grid, dim3(kThreads), 0, st, a); break;
    case 2: hipLaunchKernelGGL(symm_allreduce_kernel<_Float16>, grid, dim3(kThreads), 0, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

HDS_EXPORT int hds_symm_allgather(const int64_t* bases, int rank, int world, int64_t cap, uint32_t epoch,
                                  const void* in, void* out, int64_t nbytes, void* host_status, void* dev_status,
                                  hipStream_t st) {
  SymmArgs a;
  if (!make_args(a, bases, rank, world, cap, epoch, in, out, nbytes, host_status, dev_status) || nbytes % 16 || nbytes > cap)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(symm_allgather_kernel, dim3(blocks_for(nbytes / 16)), dim3(kThreads), 0, st, a);
  return hipGetLastError();
}

HDS_EXPORT int hds_symm_reduce_scatter(const int64_t* bases, int rank, int world, int64_t cap, uint32_t epoch,
                                       const void* in, void* out, int64_t n, int dtype, void* host_status,
                                       void* dev_status, hipStream_t st) {
  SymmArgs a;
  const int64_t es = dtype == 0 ? 4 : 2;
  if (!make_args(a, bases, rank, world, cap, epoch, in, out, n, host_status, dev_status) || n % 8 || world * n * es > cap)
    return hipErrorInvalidValue;
  const dim3 grid(blocks_for(n / 8));
  switch (dtype) {
    case 0: hipLaunchKernelGGL(symm_reduce_scatter_kernel<float>, grid, dim3(kThreads), 0, st, a); break;
    case 1: hipLaunchKernelGGL(symm_reduce_scatter_kernel<bf16>, grid, dim3(kThreads), 0, st, a); break;
    case 2: hipLaunchKernelGGL(symm_reduce_scatter_kernel<_Float16>, grid, dim3(kThreads), 0, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}
