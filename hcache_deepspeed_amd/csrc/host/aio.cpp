// Asynchronous tensor file I/O for the NVMe offload tier (ZeRO-Infinity param/optimizer swapping).
//
// Capability parity: reference csrc/aio/** (`aio_handle(block_size, queue_depth, single_submit,
// overlap_events, intra_op_parallelism)` with read/write/pread/pwrite/sync_*/async_*/wait,
// py_lib/py_ds_aio.cpp:19-115, the libaio batched submission of common/deepspeed_aio_common.cpp:71-130;
// SURVEY §2.10 N6) and the GDS handle (N7, served on MI355X by the same bounce-buffer path).
//
// Two engines behind one request API:
//   * io_uring (default when the kernel allows it; raw syscalls, no liburing in the image): a request is cut
//     into block_size chunks, every chunk is one IORING_OP_READ / IORING_OP_WRITE SQE, up to queue_depth in
//     flight; a reaper thread harvests CQEs, resubmits short transfers, feeds the backlog and completes
//     requests. Files are opened O_DIRECT when buffer, size and offset are 4 KiB aligned (pinned
//     hipHostMalloc buffers are), buffered otherwise.
//   * a thread pool issuing positional pread/pwrite per chunk (fallback; HDS_AIO_ENGINE=threads forces it).
// Every submission returns a request id; hds_aio_wait_req(id) waits for exactly that request, so a pipeline
// (read chunk i+1 / compute chunk i / write chunk i-1) waits only on what it needs.
#include <fcntl.h>
#include <linux/io_uring.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cerrno>
#include <condition_variable>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <vector>

#define HDS_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

struct Request {
  int fd = -1;
  bool write = false;
  int64_t remaining = 0;  // chunks not finished (guarded by Engine::mu)
  int errors = 0;
  bool tracked = false;  // waited by id (otherwise by hds_aio_wait)
};

struct Chunk {
  std::shared_ptr<Request> req;
  char* buf;
  int64_t n, off, done;
};

bool aligned(const void* p, int64_t bytes, int64_t off) {
  return ((uintptr_t)p % 4096 == 0) && (bytes % 4096 == 0) && (off % 4096 == 0);
}

class Engine {
 public:
  virtual ~Engine() = default;
  int64_t block_size = 1 << 20;
  std::mutex mu;
  std::condition_variable done_cv;
  std::unordered_map<int64_t, std::shared_ptr<Request>> reqs;
  int64_t next_id = 1;
  int64_t untracked_done = 0;
  int untracked_errors = 0;

  int64_t submit(bool write, char* buf, int64_t bytes, const std::string& path, int64_t file_off, bool tracked) {
    const bool direct = aligned(buf, bytes, file_off);
    const int flags = write ? (O_WRONLY | O_CREAT) : O_RDONLY;
    int fd = open(path.c_str(), flags | (direct ? O_DIRECT : 0), 0644);
    if (fd < 0 && direct) fd = open(path.c_str(), flags, 0644);
    if (fd < 0) return -errno;
    auto r = std::make_shared<Request>();
    r->fd = fd;
    r->write = write;
    r->tracked = tracked;
    const int64_t bs = std::max<int64_t>(4096, block_size / 4096 * 4096);
    std::vector<Chunk*> chunks;
    for (int64_t o = 0; o < bytes; o += bs) chunks.push_back(new Chunk{r, buf + o, std::min(bs, bytes - o), file_off + o, 0});
    int64_t id;
    {
      std::lock_guard<std::mutex> l(mu);
      id = next_id++;
      r->remaining = (int64_t)chunks.size();
      reqs[id] = r;
    }
    if (chunks.empty()) {
      finish_chunk(nullptr, r);
      return id;
    }
    enqueue(chunks);
    return id;
  }

  int wait_req(int64_t id) {
    std::shared_ptr<Request> r;
    std::unique_lock<std::mutex> l(mu);
    auto it = reqs.find(id);
    if (it == reqs.end()) return -EINVAL;
    r = it->second;
    done_cv.wait(l, [&] { return r->remaining == 0; });
    reqs.erase(id);
    return r->errors ? -r->errors : 0;
  }

  // wait for every untracked request; returns how many completed since the last call (or -errors)
  int64_t wait_all() {
    std::unique_lock<std::mutex> l(mu);
    done_cv.wait(l, [&] {
      for (auto& kv : reqs)
        if (!kv.second->tracked && kv.second->remaining > 0) return false;
      return true;
    });
    for (auto it = reqs.begin(); it != reqs.end();) {
      if (!it->second->tracked) it = reqs.erase(it);
      else ++it;
    }
    const int64_t n = untracked_done;
    const int e = untracked_errors;
    untracked_done = 0;
    untracked_errors = 0;
    return e ? -(int64_t)e : n;
  }

  virtual int kind() const = 0;

 protected:
  virtual void enqueue(std::vector<Chunk*>& chunks) = 0;

  // one transfer step of a chunk finished with `res` bytes (or -errno); returns true when the chunk is done
  bool advance(Chunk* c, int64_t res) {
    if (res <= 0) {
      std::lock_guard<std::mutex> l(mu);
      c->req->errors++;
      return true;
    }
    c->done += res;
    return c->done >= c->n;
  }

  void finish_chunk(Chunk* c, std::shared_ptr<Request> r) {
    delete c;
    bool last = false;
    {
      std::lock_guard<std::mutex> l(mu);
      if (--r->remaining <= 0) {
        r->remaining = 0;
        last = true;
        if (!r->tracked) {
          untracked_done++;
          untracked_errors += r->errors;
        }
      }
    }
    if (last) {
      if (r->fd >= 0) close(r->fd);
      r->fd = -1;
      done_cv.notify_all();
    }
  }
};

// ------------------------------------------------------------------------------------------------
// thread-pool engine
// ------------------------------------------------------------------------------------------------
class ThreadEngine : public Engine {
 public:
  explicit ThreadEngine(int n) {
    for (int i = 0; i < std::max(1, n); ++i)
      workers.emplace_back([this] {
        for (;;) {
          Chunk* c;
          {
            std::unique_lock<std::mutex> l(qmu);
            qcv.wait(l, [this] { return stop || !q.empty(); });
            if (stop && q.empty()) return;
            c = q.front();
            q.pop_front();
          }
          for (;;) {
            const ssize_t r = c->req->write ? pwrite(c->req->fd, c->buf + c->done, c->n - c->done, c->off + c->done)
                                            : pread(c->req->fd, c->buf + c->done, c->n - c->done, c->off + c->done);
            if (advance(c, r <= 0 ? (r == 0 ? -EIO : -errno) : r)) break;
          }
          auto req = c->req;
          finish_chunk(c, req);
        }
      });
  }
  ~ThreadEngine() override {
    {
      std::lock_guard<std::mutex> l(qmu);
      stop = true;
    }
    qcv.notify_all();
    for (auto& t : workers) t.join();
  }
  int kind() const override { return 0; }

 protected:
  void enqueue(std::vector<Chunk*>& chunks) override {
    {
      std::lock_guard<std::mutex> l(qmu);
      for (auto* c : chunks) q.push_back(c);
    }
    qcv.notify_all();
  }

 private:
  std::vector<std::thread> workers;
  std::deque<Chunk*> q;
  std::mutex qmu;
  std::condition_variable qcv;
  bool stop = false;
};

// ------------------------------------------------------------------------------------------------
// io_uring engine (raw syscalls)
// ------------------------------------------------------------------------------------------------
class UringEngine : public Engine {
 public:
  static UringEngine* create(unsigned entries) {
    io_uring_params p;
    memset(&p, 0, sizeof p);
    const int fd = (int)syscall(__NR_io_uring_setup, entries, &p);
    if (fd < 0) return nullptr;
    auto* e = new UringEngine();
    e->ring_fd = fd;
    if (!e->map(p)) {
      delete e;
      return nullptr;
    }
    e->depth = p.sq_entries;
    e->reaper = std::thread([e] { e->reap_loop(); });
    return e;
  }
  ~UringEngine() override {
    if (reaper.joinable()) {
      {
        std::lock_guard<std::mutex> l(smu);
        stopping = true;
        push_sqe(nullptr, /*nop=*/true);  // wakes the reaper
        flush_locked();
      }
      reaper.join();
    }
    if (sqes) munmap(sqes, sqes_sz);
    if (cq_ptr && cq_ptr != sq_ptr) munmap(cq_ptr, cq_sz);
    if (sq_ptr) munmap(sq_ptr, sq_sz);
    if (ring_fd >= 0) close(ring_fd);
  }
  int kind() const override { return 1; }

 protected:
  void enqueue(std::vector<Chunk*>& chunks) override {
    std::lock_guard<std::mutex> l(smu);
    for (auto* c : chunks) backlog.push_back(c);
    pump_locked();
  }

 private:
  int ring_fd = -1;
  void *sq_ptr = nullptr, *cq_ptr = nullptr;
  io_uring_sqe* sqes = nullptr;
  size_t sq_sz = 0, cq_sz = 0, sqes_sz = 0;
  unsigned *sq_head, *sq_tail, *sq_mask, *sq_array, *cq_head, *cq_tail, *cq_mask;
  io_uring_cqe* cqes;
  unsigned depth = 0, inflight = 0, to_submit = 0;
  std::mutex smu;  // serialises the SQ ring, inflight accounting and the backlog
  std::deque<Chunk*> backlog;
  std::thread reaper;
  bool stopping = false;

  bool map(const io_uring_params& p) {
    sq_sz = p.sq_off.array + p.sq_entries * sizeof(unsigned);
    cq_sz = p.cq_off.cqes + p.cq_entries * sizeof(io_uring_cqe);
    const bool single = p.features & IORING_FEAT_SINGLE_MMAP;
    if (single) sq_sz = cq_sz = std::max(sq_sz, cq_sz);
    sq_ptr = mmap(nullptr, sq_sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, ring_fd, IORING_OFF_SQ_RING);
    if (sq_ptr == MAP_FAILED) return (sq_ptr = nullptr), false;
    cq_ptr = single ? sq_ptr
                    : mmap(nullptr, cq_sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, ring_fd, IORING_OFF_CQ_RING);
    if (cq_ptr == MAP_FAILED) return (cq_ptr = nullptr), false;
    sqes_sz = p.sq_entries * sizeof(io_uring_sqe);
    sqes = (io_uring_sqe*)mmap(nullptr, sqes_sz, PROT_READ | PROT_WRITE, MAP_SHARED | MAP_POPULATE, ring_fd,
                               IORING_OFF_SQES);
    if (sqes == MAP_FAILED) return (sqes = nullptr), false;
    char* s = (char*)sq_ptr;
    char* c = (char*)cq_ptr;
    sq_head = (unsigned*)(s + p.sq_off.head);
    sq_tail = (unsigned*)(s + p.sq_off.tail);
    sq_mask = (unsigned*)(s + p.sq_off.ring_mask);
    sq_array = (unsigned*)(s + p.sq_off.array);
    cq_head = (unsigned*)(c + p.cq_off.head);
    cq_tail = (unsigned*)(c + p.cq_off.tail);
    cq_mask = (unsigned*)(c + p.cq_off.ring_mask);
    cqes = (io_uring_cqe*)(c + p.cq_off.cqes);
    return true;
  }

  void push_sqe(Chunk* ch, bool nop = false) {
    const unsigned tail = *sq_tail;
    const unsigned idx = tail & *sq_mask;
    io_uring_sqe* e = &sqes[idx];
    memset(e, 0, sizeof *e);
    if (nop) {
      e->opcode = IORING_OP_NOP;
      e->user_data = 0;
    } else {
      e->opcode = ch->req->write ? IORING_OP_WRITE : IORING_OP_READ;
      e->fd = ch->req->fd;
      e->addr = (uint64_t)(ch->buf + ch->done);
      e->len = (uint32_t)(ch->n - ch->done);
      e->off = (uint64_t)(ch->off + ch->done);
      e->user_data = (uint64_t)ch;
      ++inflight;
    }
    sq_array[idx] = idx;
    __atomic_store_n(sq_tail, tail + 1, __ATOMIC_RELEASE);
    ++to_submit;
  }

  void flush_locked() {
    while (to_submit) {
      const int r = (int)syscall(__NR_io_uring_enter, ring_fd, to_submit, 0, 0, nullptr, 0);
      if (r < 0) {
        if (errno == EINTR || errno == EAGAIN || errno == EBUSY) continue;
        break;
      }
      to_submit -= (unsigned)r;
    }
  }

  // fill free SQ slots from the backlog (caller holds smu)
  void pump_locked() {
    while (!backlog.empty() && inflight < depth) {
      push_sqe(backlog.front());
      backlog.pop_front();
    }
    flush_locked();
  }

  void reap_loop() {
    for (;;) {
      unsigned head = __atomic_load_n(cq_head, __ATOMIC_RELAXED);
      const unsigned tail = __atomic_load_n(cq_tail, __ATOMIC_ACQUIRE);
      if (head == tail) {
        {
          std::lock_guard<std::mutex> l(smu);
          if (stopping && inflight == 0 && backlog.empty()) return;
        }
        syscall(__NR_io_uring_enter, ring_fd, 0, 1, IORING_ENTER_GETEVENTS, nullptr, 0);
        continue;
      }
      std::vector<std::pair<Chunk*, int64_t>> got;
      while (head != tail) {
        const io_uring_cqe& c = cqes[head & *cq_mask];
        got.emplace_back((Chunk*)c.user_data, (int64_t)c.res);
        ++head;
      }
      __atomic_store_n(cq_head, head, __ATOMIC_RELEASE);
      std::vector<Chunk*> again;
      for (auto& g : got) {
        Chunk* ch = g.first;
        if (ch == nullptr) continue;  // wake-up NOP
        {
          std::lock_guard<std::mutex> l(smu);
          --inflight;
        }
        if (advance(ch, g.second)) {
          auto req = ch->req;
          finish_chunk(ch, req);
        } else {
          again.push_back(ch);  // short transfer: resubmit the rest
        }
      }
      std::lock_guard<std::mutex> l(smu);
      for (auto* ch : again) backlog.push_front(ch);
      pump_locked();
    }
  }
};

}  // namespace

HDS_EXPORT void* hds_aio_create(int64_t block_size, int queue_depth, int single_submit, int overlap_events,
                                int intra_op_parallelism) {
  (void)single_submit;
  (void)overlap_events;
  Engine* e = nullptr;
  const char* forced = getenv("HDS_AIO_ENGINE");
  if (!(forced && strcmp(forced, "threads") == 0)) {
    unsigned entries = 1;
    while (entries < (unsigned)std::max(8, queue_depth)) entries <<= 1;
    e = UringEngine::create(std::min(entries, 4096u));
  }
  if (e == nullptr) e = new ThreadEngine(intra_op_parallelism > 0 ? intra_op_parallelism : 1);
  e->block_size = block_size > 0 ? block_size : (1 << 20);
  return e;
}

HDS_EXPORT int hds_aio_destroy(void* h) {
  delete (Engine*)h;
  return 0;
}

// 1 = io_uring, 0 = thread pool
HDS_EXPORT int hds_aio_engine(void* h) { return ((Engine*)h)->kind(); }

// returns a request id (> 0) to pass to hds_aio_wait_req, or -errno
HDS_EXPORT int64_t hds_aio_submit(void* h, int write, void* buf, int64_t bytes, const char* path, int64_t file_off) {
  return ((Engine*)h)->submit(write != 0, (char*)buf, bytes, path, file_off, true);
}

HDS_EXPORT int hds_aio_wait_req(void* h, int64_t id) { return ((Engine*)h)->wait_req(id); }

// async_op=0: blocks until this request completes; async_op=1: completes at the next hds_aio_wait
HDS_EXPORT int hds_aio_pread(void* h, void* buf, int64_t bytes, const char* path, int64_t file_off, int async_op) {
  Engine* e = (Engine*)h;
  const int64_t id = e->submit(false, (char*)buf, bytes, path, file_off, !async_op);
  if (id < 0) return -1;
  return async_op ? 0 : (e->wait_req(id) == 0 ? 0 : -1);
}

HDS_EXPORT int hds_aio_pwrite(void* h, const void* buf, int64_t bytes, const char* path, int64_t file_off,
                              int async_op) {
  Engine* e = (Engine*)h;
  const int64_t id = e->submit(true, (char*)buf, bytes, path, file_off, !async_op);
  if (id < 0) return -1;
  return async_op ? 0 : (e->wait_req(id) == 0 ? 0 : -1);
}

// wait for every outstanding async (untracked) request; returns the number completed since the last wait,
// or -errors if any chunk failed
HDS_EXPORT int64_t hds_aio_wait(void* h) { return ((Engine*)h)->wait_all(); }

HDS_EXPORT int64_t hds_aio_file_size(const char* path) {
  struct stat st;
  if (stat(path, &st) != 0) return -1;
  return st.st_size;
}
