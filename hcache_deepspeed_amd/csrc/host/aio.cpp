// Asynchronous tensor file I/O for the NVMe offload tier (ZeRO-Infinity param/optimizer swapping).
//
// Capability parity: reference csrc/aio/** (`aio_handle(block_size, queue_depth, single_submit,
// overlap_events, intra_op_parallelism)` with read/write/pread/pwrite/sync_*/async_*/wait,
// py_lib/py_ds_aio.cpp:19-115) and the GDS handle (N7, which on MI355X is served by
// the same bounce-buffer path). libaio is not part of this image, so the engine is a persistent
// thread pool issuing positional pread/pwrite; each request is split into `intra_op_parallelism`
// block-aligned chunks; files are opened O_DIRECT when buffer, size and offset are 4 KiB aligned
// (pinned hipHostMalloc buffers always are), buffered otherwise.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <memory>
#include <cstdint>
#include <cstring>
#include <deque>
#include <functional>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#define HDS_EXPORT extern "C" __attribute__((visibility("default")))

namespace {

struct Pool {
  std::vector<std::thread> workers;
  std::deque<std::function<void()>> q;
  std::mutex mu;
  std::condition_variable cv, done_cv;
  bool stop = false;
  int64_t pending = 0;       // chunks not yet finished
  int64_t completed_ops = 0;  // whole requests finished since last wait
  std::atomic<int> errors{0};
  int64_t block_size = 1 << 20;
  int parallel = 1;

  explicit Pool(int n) {
    for (int i = 0; i < n; ++i)
      workers.emplace_back([this] {
        for (;;) {
          std::function<void()> job;
          {
            std::unique_lock<std::mutex> l(mu);
            cv.wait(l, [this] { return stop || !q.empty(); });
            if (stop && q.empty()) return;
            job = std::move(q.front());
            q.pop_front();
          }
          job();
          {
            std::lock_guard<std::mutex> l(mu);
            --pending;
          }
          done_cv.notify_all();
        }
      });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> l(mu);
      stop = true;
    }
    cv.notify_all();
    for (auto& t : workers) t.join();
  }
  void submit(std::function<void()> f) {
    {
      std::lock_guard<std::mutex> l(mu);
      ++pending;
      q.push_back(std::move(f));
    }
    cv.notify_one();
  }
  void wait_all() {
    std::unique_lock<std::mutex> l(mu);
    done_cv.wait(l, [this] { return pending == 0; });
  }
};

bool aligned(const void* p, int64_t bytes, int64_t off) {
  return ((uintptr_t)p % 4096 == 0) && (bytes % 4096 == 0) && (off % 4096 == 0);
}

int do_io(bool write, void* buf, int64_t bytes, const std::string& path, int64_t file_off, Pool* pool) {
  const bool direct = aligned(buf, bytes, file_off);
  int flags = write ? (O_WRONLY | O_CREAT) : O_RDONLY;
  int fd = open(path.c_str(), flags | (direct ? O_DIRECT : 0), 0644);
  if (fd < 0 && direct) fd = open(path.c_str(), flags, 0644);
  if (fd < 0) return -1;
  const int64_t nchunks = pool->parallel;
  int64_t chunk = (bytes + nchunks - 1) / nchunks;
  chunk = (chunk + 4095) / 4096 * 4096;
  auto remaining = std::make_shared<std::atomic<int64_t>>(0);
  for (int64_t off = 0; off < bytes; off += chunk) remaining->fetch_add(1);
  for (int64_t off = 0; off < bytes; off += chunk) {
    const int64_t n = std::min(chunk, bytes - off);
    pool->submit([=] {
      int64_t done = 0;
      while (done < n) {
        ssize_t r = write ? pwrite(fd, (char*)buf + off + done, n - done, file_off + off + done)
                          : pread(fd, (char*)buf + off + done, n - done, file_off + off + done);
        if (r <= 0) {
          pool->errors++;
          break;
        }
        done += r;
      }
      if (remaining->fetch_sub(1) == 1) {
        close(fd);
        std::lock_guard<std::mutex> l(pool->mu);
        pool->completed_ops++;
      }
    });
  }
  return 0;
}

}  // namespace

HDS_EXPORT void* hds_aio_create(int64_t block_size, int queue_depth, int single_submit, int overlap_events,
                                int intra_op_parallelism) {
  int threads = intra_op_parallelism > 0 ? intra_op_parallelism : 1;
  Pool* p = new Pool(threads);
  p->block_size = block_size;
  p->parallel = threads;
  (void)queue_depth;
  (void)single_submit;
  (void)overlap_events;
  return p;
}

HDS_EXPORT int hds_aio_destroy(void* h) {
  delete (Pool*)h;
  return 0;
}

// async_op=0: blocks until this request completes
HDS_EXPORT int hds_aio_pread(void* h, void* buf, int64_t bytes, const char* path, int64_t file_off, int async_op) {
  Pool* p = (Pool*)h;
  int rc = do_io(false, buf, bytes, path, file_off, p);
  if (rc == 0 && !async_op) {
    p->wait_all();
    std::lock_guard<std::mutex> l(p->mu);
    p->completed_ops--;  // synchronous requests are not reported by wait()
  }
  return rc;
}

HDS_EXPORT int hds_aio_pwrite(void* h, const void* buf, int64_t bytes, const char* path, int64_t file_off,
                              int async_op) {
  Pool* p = (Pool*)h;
  int rc = do_io(true, (void*)buf, bytes, path, file_off, p);
  if (rc == 0 && !async_op) {
    p->wait_all();
    std::lock_guard<std::mutex> l(p->mu);
    p->completed_ops--;
  }
  return rc;
}

// wait for every outstanding request; returns the number of requests completed since the last wait,
// or -errors if any chunk failed
HDS_EXPORT int64_t hds_aio_wait(void* h) {
  Pool* p = (Pool*)h;
  p->wait_all();
  int64_t n;
  {
    std::lock_guard<std::mutex> l(p->mu);
    n = p->completed_ops;
    p->completed_ops = 0;
  }
  int e = p->errors.exchange(0);
  return e ? -(int64_t)e : n;
}

HDS_EXPORT int64_t hds_aio_file_size(const char* path) {
  struct stat st;
  if (stat(path, &st) != 0) return -1;
  return st.st_size;
}
