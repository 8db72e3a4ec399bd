// Native RCCL communicator + stream-ordered collective executor (host C++).
//
// Reference parity: DeepCompile's native comm layer, csrc/compile/deepcompile.cpp:18,153 and z3.cpp:83,235 /
// z1.cpp:72 (a private ncclComm_t with ncclAllGather / ncclReduceScatter / ncclAllReduce on dedicated streams),
// SURVEY.md §2.10 N20 and §5.8 "Native path". Not a translation: this layer owns
//   * the RCCL communicator (one per process group, created from a unique id that python broadcasts once),
//   * ONE high-priority communication HIP stream per communicator, so collectives never queue behind compute
//     (created by torch's stream pool and passed in: torch never destroys pooled streams, so the caching
//     allocator's record_stream events on it stay valid after the communicator is gone),
//   * a ring of completion events: every collective first waits (on the GPU, hipStreamWaitEvent) for the caller's
//     stream, runs on the comm stream and records a completion event; the caller later makes ITS stream wait on
//     that event (or blocks the host), so nothing on the compute path synchronizes the device.
// librccl is dlopen'ed from the path python passes (torch's own librccl.so), so the process holds exactly one
// RCCL, the one torch.distributed uses; there is no link-time dependency and the library builds without a GPU.
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <atomic>
#include <mutex>
#include <vector>

#define HDS_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

typedef struct ncclComm* ncclComm_t;
typedef struct {
  char internal[128];
} ncclUniqueId;
typedef int ncclResult_t;

struct Rccl {
  void* h = nullptr;
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*AllGather)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*ReduceScatter)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Broadcast)(const void*, void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllToAll)(const void*, void*, size_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Send)(const void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, int, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
};

Rccl g;
std::mutex g_mu;

template <typename F>
bool sym(F& f, const char* name) {
  f = reinterpret_cast<F>(dlsym(g.h, name));
  return f != nullptr;
}

constexpr int kEvents = 64;  // completion events per communicator (ring)

struct Comm {
  ncclComm_t comm = nullptr;
  hipStream_t stream = nullptr;
  int rank = 0, nranks = 1;
  hipEvent_t ready[kEvents];  // caller-stream "inputs ready" events
  hipEvent_t done[kEvents];   // comm-stream completion events
  std::atomic<uint64_t> seq{0};
};

// 0 = issued, >0 = HIP error, <0 = -(RCCL error) - 1000
int rc_rccl(ncclResult_t r) { return r == 0 ? 0 : -(1000 + r); }

// Order the comm stream after the caller's stream, return the slot whose `done` event the op will record.
int begin(Comm* c, hipStream_t caller, int* slot) {
  const int s = (int)(c->seq.fetch_add(1) % kEvents);
  hipError_t e = hipEventRecord(c->ready[s], caller);
  if (e == hipSuccess) e = hipStreamWaitEvent(c->stream, c->ready[s], 0);
  *slot = s;
  return (int)e;
}

int end(Comm* c, int slot, int rc) {
  if (rc != 0) return rc;
  return (int)hipEventRecord(c->done[slot], c->stream);
}

}  // namespace

HDS_EXPORT int hds_rccl_load(const char* path) {
  std::lock_guard<std::mutex> lk(g_mu);
  if (g.h) return 0;
  void* h = dlopen(path, RTLD_NOW | RTLD_GLOBAL);
  if (!h) return 1;
  g.h = h;
  bool ok = sym(g.GetUniqueId, "ncclGetUniqueId") && sym(g.CommInitRank, "ncclCommInitRank") &&
            sym(g.CommDestroy, "ncclCommDestroy") && sym(g.AllGather, "ncclAllGather") &&
            sym(g.ReduceScatter, "ncclReduceScatter") && sym(g.AllReduce, "ncclAllReduce") &&
            sym(g.Broadcast, "ncclBroadcast") && sym(g.Send, "ncclSend") && sym(g.Recv, "ncclRecv") &&
            sym(g.GroupStart, "ncclGroupStart") && sym(g.GroupEnd, "ncclGroupEnd") &&
            sym(g.GetErrorString, "ncclGetErrorString");
  sym(g.AllToAll, "ncclAllToAll");  // RCCL extension (optional)
  if (!ok) {
    dlclose(h);
    g = Rccl();
    return 2;
  }
  return 0;
}

HDS_EXPORT const char* hds_rccl_error_string(int rc) {
  if (rc <= -1000 && g.GetErrorString) return g.GetErrorString(-rc - 1000);
  if (rc > 0) return hipGetErrorString((hipError_t)rc);
  return rc == 0 ? "success" : "unknown";
}

HDS_EXPORT int hds_rccl_unique_id(char* out128) {
  if (!g.h) return 3;
  ncclUniqueId id;
  int rc = rc_rccl(g.GetUniqueId(&id));
  if (rc == 0) memcpy(out128, id.internal, 128);
  return rc;
}

// Create the communicator on the CURRENT HIP device (python sets it), issuing on `stream` (a high-priority stream
// owned by the caller). Returns a handle or null (*err set).
HDS_EXPORT void* hds_rccl_init(const char* id128, int nranks, int rank, void* stream, int* err) {
  *err = 3;
  if (!g.h) return nullptr;
  Comm* c = new Comm();
  c->rank = rank;
  c->nranks = nranks;
  c->stream = (hipStream_t)stream;
  hipError_t e = hipSuccess;
  for (int i = 0; e == hipSuccess && i < kEvents; ++i) {
    e = hipEventCreateWithFlags(&c->ready[i], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&c->done[i], hipEventDisableTiming);
  }
  if (e != hipSuccess) {
    *err = (int)e;
    delete c;
    return nullptr;
  }
  ncclUniqueId id;
  memcpy(id.internal, id128, 128);
  *err = rc_rccl(g.CommInitRank(&c->comm, nranks, id, rank));
  if (*err != 0) {
    delete c;
    return nullptr;
  }
  return c;
}

HDS_EXPORT int hds_rccl_destroy(void* h) {
  Comm* c = (Comm*)h;
  if (!c) return 0;
  hipStreamSynchronize(c->stream);
  int rc = c->comm ? rc_rccl(g.CommDestroy(c->comm)) : 0;
  for (int i = 0; i < kEvents; ++i) {
    hipEventDestroy(c->ready[i]);
    hipEventDestroy(c->done[i]);
  }
  delete c;  // the stream belongs to the caller
  return rc;
}

HDS_EXPORT void* hds_rccl_stream(void* h) { return ((Comm*)h)->stream; }

// Every collective: (comm, buffers, count, nccl dtype, [op], caller stream, *slot out). The op is ordered after
// the work already queued on `caller`; its completion is `slot`'s event (hds_rccl_wait / hds_rccl_query).
HDS_EXPORT int hds_rccl_all_gather(void* h, const void* send, void* recv, size_t sendcount, int dtype, void* caller,
                                   int* slot) {
  Comm* c = (Comm*)h;
  int rc = begin(c, (hipStream_t)caller, slot);
  if (rc == 0) rc = rc_rccl(g.AllGather(send, recv, sendcount, dtype, c->comm, c->stream));
  return end(c, *slot, rc);
}

HDS_EXPORT int hds_rccl_reduce_scatter(void* h, const void* send, void* recv, size_t recvcount, int dtype, int op,
                                       void* caller, int* slot) {
  Comm* c = (Comm*)h;
  int rc = begin(c, (hipStream_t)caller, slot);
  if (rc == 0) rc = rc_rccl(g.ReduceScatter(send, recv, recvcount, dtype, op, c->comm, c->stream));
  return end(c, *slot, rc);
}

HDS_EXPORT int hds_rccl_all_reduce(void* h, const void* send, void* recv, size_t count, int dtype, int op,
                                   void* caller, int* slot) {
  Comm* c = (Comm*)h;
  int rc = begin(c, (hipStream_t)caller, slot);
  if (rc == 0) rc = rc_rccl(g.AllReduce(send, recv, count, dtype, op, c->comm, c->stream));
  return end(c, *slot, rc);
}

HDS_EXPORT int hds_rccl_broadcast(void* h, const void* send, void* recv, size_t count, int dtype, int root,
                                  void* caller, int* slot) {
  Comm* c = (Comm*)h;
  int rc = begin(c, (hipStream_t)caller, slot);
  if (rc == 0) rc = rc_rccl(g.Broadcast(send, recv, count, dtype, root, c->comm, c->stream));
  return end(c, *slot, rc);
}

// Equal-split all-to-all: `count` elements to every peer. Uses RCCL's ncclAllToAll when present, else a grouped
// send/recv over all peers (each GPU talks to all 7 xGMI peers at once).
HDS_EXPORT int hds_rccl_all_to_all(void* h, const void* send, void* recv, size_t count, int dtype, int elem_bytes,
                                   void* caller, int* slot) {
  Comm* c = (Comm*)h;
  int rc = begin(c, (hipStream_t)caller, slot);
  if (rc == 0) {
    if (g.AllToAll) {
      rc = rc_rccl(g.AllToAll(send, recv, count, dtype, c->comm, c->stream));
    } else {
      rc = rc_rccl(g.GroupStart());
      for (int p = 0; rc == 0 && p < c->nranks; ++p) {
        rc = rc_rccl(g.Send((const char*)send + (size_t)p * count * elem_bytes, count, dtype, p, c->comm, c->stream));
        if (rc == 0)
          rc = rc_rccl(g.Recv((char*)recv + (size_t)p * count * elem_bytes, count, dtype, p, c->comm, c->stream));
      }
      int rc2 = rc_rccl(g.GroupEnd());
      if (rc == 0) rc = rc2;
    }
  }
  return end(c, *slot, rc);
}

// Make `caller` wait (on the GPU) for the collective in `slot`.
HDS_EXPORT int hds_rccl_wait(void* h, int slot, void* caller) {
  Comm* c = (Comm*)h;
  return (int)hipStreamWaitEvent((hipStream_t)caller, c->done[slot], 0);
}

// 1 = complete, 0 = in flight, <0 error
HDS_EXPORT int hds_rccl_query(void* h, int slot) {
  Comm* c = (Comm*)h;
  hipError_t e = hipEventQuery(c->done[slot]);
  if (e == hipSuccess) return 1;
  if (e == hipErrorNotReady) return 0;
  return -(int)e;
}

HDS_EXPORT int hds_rccl_synchronize(void* h) { return (int)hipStreamSynchronize(((Comm*)h)->stream); }
