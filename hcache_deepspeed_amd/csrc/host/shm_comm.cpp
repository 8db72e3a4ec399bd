// Shared-memory all-reduce for CPU tensors of ranks on one host (the CPU / gloo configuration of the framework:
// CPU inference with AutoTP, plumbing tests).
//
// Capability parity: csrc/cpu/comm/shm.cpp + shm_interface.cpp (reference SURVEY §2.10 N21,
// ``torch.ops.deepspeed.inference_all_reduce_``): a low-latency all-reduce through a POSIX shared-memory segment
// instead of the gloo TCP ring.
//
// Segment layout: [control: 2 x world generation counters (64-byte padded)] [world input slots] [result slot].
// Protocol for generation g (one call):
//   1. copy my input into slot[rank]; publish arrive[rank] = g (release)
//   2. wait for arrive[*] == g (acquire)
//   3. reduce my 1/world share of the elements over all slots (fp32 accumulation) into the result slot;
//      publish reduced[rank] = g
//   4. wait for reduced[*] == g, copy the result back into my tensor.
// A rank cannot start writing slot[rank] of generation g+1 before it finished step 4 of g, and nobody reads slots
// of g+1 before every rank arrived at g+1, so no extra barrier is needed between calls.
#include <fcntl.h>
#include <sched.h>
#include <stdint.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <string>

#define HDS_HOST_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

struct alignas(64) Counter {
  std::atomic<int64_t> v;
  char pad[64 - sizeof(std::atomic<int64_t>)];
};

struct ShmComm {
  std::string name;
  int rank = 0, world = 1;
  size_t slot_bytes = 0, total = 0;
  char* base = nullptr;
  Counter* arrive = nullptr;
  Counter* reduced = nullptr;
  char* slots = nullptr;
  char* result = nullptr;
  int64_t gen = 0;
  bool owner = false;
};

inline void spin_until_all(Counter* c, int world, int64_t g) {
  for (int r = 0; r < world; ++r) {
    int spins = 0;
    while (c[r].v.load(std::memory_order_acquire) < g) {
      if (++spins > 1024) {
        sched_yield();
        spins = 0;
      }
    }
  }
}

inline float bf16_to_f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

inline uint16_t f_to_bf16(float f) {  // round to nearest even
  uint32_t u;
  memcpy(&u, &f, 4);
  if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x7FFFFFu)) return (uint16_t)((u >> 16) | 0x40);  // NaN
  u += 0x7FFFu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

}  // namespace

// dtype: 0 = fp32, 1 = bf16. create != 0: the first rank creates (and sizes) the segment.
HDS_HOST_EXPORT void* hds_shm_open(const char* name, int rank, int world, int64_t slot_bytes, int create) {
  auto* c = new ShmComm();
  c->name = name;
  c->rank = rank;
  c->world = world;
  c->slot_bytes = (size_t)((slot_bytes + 63) / 64 * 64);
  const size_t ctrl = 2 * (size_t)world * sizeof(Counter);
  c->total = ctrl + (size_t)(world + 1) * c->slot_bytes;
  int fd = shm_open(name, create ? (O_CREAT | O_RDWR) : O_RDWR, 0600);
  if (fd < 0) {
    delete c;
    return nullptr;
  }
  if (create && ftruncate(fd, (off_t)c->total) != 0) {
    close(fd);
    delete c;
    return nullptr;
  }
  void* p = mmap(nullptr, c->total, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  close(fd);
  if (p == MAP_FAILED) {
    delete c;
    return nullptr;
  }
  c->base = (char*)p;
  c->arrive = reinterpret_cast<Counter*>(c->base);
  c->reduced = c->arrive + world;
  c->slots = c->base + ctrl;
  c->result = c->slots + (size_t)world * c->slot_bytes;
  c->owner = create != 0;
  if (create) {
    for (int r = 0; r < 2 * world; ++r) c->arrive[r].v.store(0, std::memory_order_relaxed);
    std::atomic_thread_fence(std::memory_order_seq_cst);
  }
  return c;
}

HDS_HOST_EXPORT int hds_shm_close(void* h, int unlink) {
  auto* c = (ShmComm*)h;
  if (!c) return -1;
  munmap(c->base, c->total);
  if (unlink) shm_unlink(c->name.c_str());
  delete c;
  return 0;
}

HDS_HOST_EXPORT int64_t hds_shm_slot_bytes(void* h) { return h ? (int64_t)((ShmComm*)h)->slot_bytes : 0; }

// In-place SUM all-reduce of `n` elements at `buf` (n * elsize <= slot_bytes).
HDS_HOST_EXPORT int hds_shm_allreduce(void* h, void* buf, int64_t n, int dtype) {
  auto* c = (ShmComm*)h;
  const size_t es = dtype == 0 ? 4 : 2;
  if (!c || n < 0 || (size_t)n * es > c->slot_bytes || (dtype != 0 && dtype != 1)) return -1;
  const int64_t g = ++c->gen;
  const int W = c->world;
  memcpy(c->slots + (size_t)c->rank * c->slot_bytes, buf, (size_t)n * es);
  c->arrive[c->rank].v.store(g, std::memory_order_release);
  spin_until_all(c->arrive, W, g);
  const int64_t per = (n + W - 1) / W;
  const int64_t lo = per * c->rank, hi = lo + per < n ? lo + per : n;
  if (dtype == 0) {
    float* out = reinterpret_cast<float*>(c->result);
    for (int64_t i = lo; i < hi; ++i) {
      float s = 0.f;
      for (int r = 0; r < W; ++r) s += reinterpret_cast<const float*>(c->slots + (size_t)r * c->slot_bytes)[i];
      out[i] = s;
    }
  } else {
    uint16_t* out = reinterpret_cast<uint16_t*>(c->result);
    for (int64_t i = lo; i < hi; ++i) {
      float s = 0.f;
      for (int r = 0; r < W; ++r)
        s += bf16_to_f(reinterpret_cast<const uint16_t*>(c->slots + (size_t)r * c->slot_bytes)[i]);
      out[i] = f_to_bf16(s);
    }
  }
  c->reduced[c->rank].v.store(g, std::memory_order_release);
  spin_until_all(c->reduced, W, g);
  memcpy(buf, c->result, (size_t)n * es);
  return 0;
}
