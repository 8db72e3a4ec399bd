// Pinned host memory tier: hipHostMalloc'd buffers and a slot ring drained by hipMemcpyAsync.
//
// Capability parity: reference inference/v2/ragged/csrc/fast_host_buffer.cu (`allocate_fast_host_buffer`,
// cudaHostAlloc portable|mapped|write-combined), the pinned bounce buffers of
// csrc/aio/py_lib/deepspeed_pin_tensor.cpp, and -- new -- the event-gated ring used by the training
// host activation cache (offload/activation_cache.py), ZeRO-Offload grad/param staging, async
// checkpointing and the HCache latent store.
//
// Ring protocol: a slot is (pinned bytes, one hipEvent). `acquire` returns the next slot after
// waiting for the event of its previous use (so a slot is never overwritten while a copy that
// reads or writes it is in flight); copies are issued on the caller's HIP stream and `record`ed
// on the slot; consumers `wait` (host) or make a stream wait on the slot event (device).
#include <hip/hip_runtime_api.h>

#include <atomic>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <vector>

#define HDS_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

struct Ring {
  char* base = nullptr;
  size_t slot_bytes = 0;
  int nslots = 0;
  std::vector<hipEvent_t> events;
  std::vector<int> used;
  int head = 0;
  std::mutex mu;
};

inline int check(hipError_t e) { return (int)e; }

}  // namespace

HDS_EXPORT void* hds_host_alloc(size_t bytes, int flags) {
  // flags bit0: portable, bit1: mapped, bit2: write-combined (reference fast host buffer)
  unsigned f = hipHostMallocDefault;
  if (flags & 1) f |= hipHostMallocPortable;
  if (flags & 2) f |= hipHostMallocMapped;
  if (flags & 4) f |= hipHostMallocWriteCombined;
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes, f) != hipSuccess) return nullptr;
  return p;
}

HDS_EXPORT int hds_host_free(void* p) { return check(hipHostFree(p)); }

HDS_EXPORT void* hds_ring_create(size_t slot_bytes, int nslots, int flags) {
  Ring* r = new Ring();
  r->slot_bytes = (slot_bytes + 4095) & ~size_t(4095);
  r->nslots = nslots;
  r->base = (char*)hds_host_alloc(r->slot_bytes * nslots, flags | 1);
  if (!r->base) {
    delete r;
    return nullptr;
  }
  r->events.resize(nslots);
  r->used.assign(nslots, 0);
  for (int i = 0; i < nslots; ++i) {
    if (hipEventCreateWithFlags(&r->events[i], hipEventDisableTiming) != hipSuccess) {
      delete r;
      return nullptr;
    }
  }
  return r;
}

HDS_EXPORT int hds_ring_destroy(void* h) {
  Ring* r = (Ring*)h;
  if (!r) return 0;
  for (auto& e : r->events) {
    hipEventSynchronize(e);
    hipEventDestroy(e);
  }
  if (r->base) hipHostFree(r->base);
  delete r;
  return 0;
}

HDS_EXPORT void* hds_ring_slot_ptr(void* h, int slot) {
  Ring* r = (Ring*)h;
  return r->base + (size_t)slot * r->slot_bytes;
}

HDS_EXPORT size_t hds_ring_slot_bytes(void* h) { return ((Ring*)h)->slot_bytes; }

// next slot in ring order, after its previous transfer has completed
HDS_EXPORT int hds_ring_acquire(void* h) {
  Ring* r = (Ring*)h;
  int s;
  {
    std::lock_guard<std::mutex> g(r->mu);
    s = r->head;
    r->head = (r->head + 1) % r->nslots;
  }
  if (r->used[s]) hipEventSynchronize(r->events[s]);
  r->used[s] = 0;
  return s;
}

// device -> slot (async on `stream`), event recorded after the copy
HDS_EXPORT int hds_ring_d2h(void* h, int slot, const void* dev, size_t bytes, size_t slot_offset, hipStream_t stream) {
  Ring* r = (Ring*)h;
  if (slot_offset + bytes > r->slot_bytes) return (int)hipErrorInvalidValue;
  hipError_t e = hipMemcpyAsync(r->base + (size_t)slot * r->slot_bytes + slot_offset, dev, bytes,
                                hipMemcpyDeviceToHost, stream);
  if (e != hipSuccess) return (int)e;
  r->used[slot] = 1;
  return check(hipEventRecord(r->events[slot], stream));
}

// slot -> device (async on `stream`)
HDS_EXPORT int hds_ring_h2d(void* h, int slot, void* dev, size_t bytes, size_t slot_offset, hipStream_t stream) {
  Ring* r = (Ring*)h;
  if (slot_offset + bytes > r->slot_bytes) return (int)hipErrorInvalidValue;
  hipError_t e = hipMemcpyAsync(dev, r->base + (size_t)slot * r->slot_bytes + slot_offset, bytes,
                                hipMemcpyHostToDevice, stream);
  if (e != hipSuccess) return (int)e;
  r->used[slot] = 1;
  return check(hipEventRecord(r->events[slot], stream));
}

HDS_EXPORT int hds_ring_record(void* h, int slot, hipStream_t stream) {
  Ring* r = (Ring*)h;
  r->used[slot] = 1;
  return check(hipEventRecord(r->events[slot], stream));
}

HDS_EXPORT int hds_ring_wait(void* h, int slot) {
  Ring* r = (Ring*)h;
  if (!r->used[slot]) return 0;
  return check(hipEventSynchronize(r->events[slot]));
}

HDS_EXPORT int hds_ring_stream_wait(void* h, int slot, hipStream_t stream) {
  Ring* r = (Ring*)h;
  if (!r->used[slot]) return 0;
  return check(hipStreamWaitEvent(stream, r->events[slot], 0));
}

HDS_EXPORT int hds_ring_query(void* h, int slot) {
  Ring* r = (Ring*)h;
  if (!r->used[slot]) return 1;
  return hipEventQuery(r->events[slot]) == hipSuccess ? 1 : 0;
}

// plain async copies between pinned host memory and device (used by offload paths)
HDS_EXPORT int hds_memcpy_async(void* dst, const void* src, size_t bytes, int kind, hipStream_t stream) {
  hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : (kind == 1 ? hipMemcpyDeviceToHost : hipMemcpyDefault);
  return check(hipMemcpyAsync(dst, src, bytes, k, stream));
}
