// Host-runtime self-test, built with AddressSanitizer + UndefinedBehaviorSanitizer (SURVEY.md §5.2 plan:
// "ASAN builds of the C++ host libraries (AIO, CPU Adam)"). Compiled straight from csrc/host/{cpu_optim,aio,
// shm_comm}.cpp by tests/test_host_sanitizers.py with g++ -fsanitize=address,undefined; exercises
//   * CPU Adam/AdamW (fp32 and bf16 grads, bf16 write-back) against a scalar double-precision reference,
//   * the async file I/O pool: chunked parallel pwrite + pread round trip of an odd-sized buffer,
//   * the shared-memory all-reduce with two ranks on two threads (generation-counter protocol, fp32 and bf16).
// Exit code 0 = all checks passed; any sanitizer report aborts with a non-zero code.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#include <string>
#include <thread>
#include <vector>

extern "C" {
int hds_cpu_adam(float* p, const void* g, int gdtype, float* m, float* v, uint16_t* out_bf16, int64_t n, float lr,
                 float b1, float b2, float eps, float wd, float bc1, float bc2, int adamw, float gscale);
void* hds_aio_create(int64_t block_size, int queue_depth, int single_submit, int overlap_events, int intra_op);
int hds_aio_destroy(void* h);
int hds_aio_pread(void* h, void* buf, int64_t bytes, const char* path, int64_t off, int async_op);
int hds_aio_pwrite(void* h, const void* buf, int64_t bytes, const char* path, int64_t off, int async_op);
int64_t hds_aio_wait(void* h);
int64_t hds_aio_submit(void* h, int write, void* buf, int64_t bytes, const char* path, int64_t off);
int hds_aio_wait_req(void* h, int64_t id);
int hds_aio_engine(void* h);
void* hds_shm_open(const char* name, int rank, int world, int64_t slot_bytes, int create);
int hds_shm_close(void* h, int unlink);
int hds_shm_allreduce(void* h, void* buf, int64_t n, int dtype);
}

static int fails = 0;
#define CHECK(c, ...)                    \
  do {                                   \
    if (!(c)) {                          \
      fprintf(stderr, "FAIL: " __VA_ARGS__); \
      fprintf(stderr, "\n");             \
      ++fails;                           \
    }                                    \
  } while (0)

static uint16_t f2bf(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  u += 0x7fff + ((u >> 16) & 1);
  return (uint16_t)(u >> 16);
}
static float bf2f(uint16_t h) {
  uint32_t u = (uint32_t)h << 16;
  float f;
  memcpy(&f, &u, 4);
  return f;
}

static void test_adam() {
  const int64_t n = 10007;  // not a multiple of the tile / vector width
  for (int gdt = 0; gdt < 2; ++gdt)
    for (int adamw = 0; adamw < 2; ++adamw) {
      std::vector<float> p(n), m(n, 0.f), v(n, 0.f), gf(n);
      std::vector<uint16_t> gh(n), out(n);
      std::vector<double> rp(n), rm(n, 0.0), rv(n, 0.0);
      srand(7);
      for (int64_t i = 0; i < n; ++i) {
        p[i] = rp[i] = (rand() / (float)RAND_MAX - 0.5f);
        gf[i] = (rand() / (float)RAND_MAX - 0.5f) * 0.1f;
        gh[i] = f2bf(gf[i]);
        if (gdt) gf[i] = bf2f(gh[i]);
      }
      const float lr = 1e-2f, b1 = 0.9f, b2 = 0.999f, eps = 1e-8f, wd = 0.01f;
      for (int step = 1; step <= 3; ++step) {
        const float bc1 = 1.f - powf(b1, step), bc2 = 1.f - powf(b2, step);
        hds_cpu_adam(p.data(), gdt ? (const void*)gh.data() : (const void*)gf.data(), gdt, m.data(), v.data(),
                     out.data(), n, lr, b1, b2, eps, wd, bc1, bc2, adamw, 1.f);
        for (int64_t i = 0; i < n; ++i) {
          double g = gf[i];
          if (!adamw) g += wd * rp[i];
          rm[i] = b1 * rm[i] + (1 - b1) * g;
          rv[i] = b2 * rv[i] + (1 - b2) * g * g;
          if (adamw) rp[i] -= lr * wd * rp[i];
          rp[i] -= (lr / bc1) * rm[i] / (sqrt(rv[i]) / sqrt(bc2) + eps);
        }
      }
      double err = 0, berr = 0;
      for (int64_t i = 0; i < n; ++i) {
        err = fmax(err, fabs(p[i] - rp[i]));
        berr = fmax(berr, fabs(bf2f(out[i]) - p[i]) / fmax(1e-3, fabs(p[i])));
      }
      CHECK(err < 1e-5, "adam gdt=%d adamw=%d max err %g", gdt, adamw, err);
      CHECK(berr < 1e-2, "adam bf16 write-back rel err %g", berr);
    }
}

static void test_aio_engine(const char* dir) {
  const int64_t bytes = (3 << 20) + 12345;
  std::vector<unsigned char> src(bytes), dst(bytes, 0);
  for (int64_t i = 0; i < bytes; ++i) src[i] = (unsigned char)(i * 131 + 7);
  std::string path = std::string(dir) + "/aio_selftest.bin";
  void* h = hds_aio_create(1 << 20, 8, 0, 1, 4);
  CHECK(h != nullptr, "aio create");
  CHECK(hds_aio_pwrite(h, src.data(), bytes, path.c_str(), 0, 1) == 0, "aio pwrite");
  CHECK(hds_aio_wait(h) >= 1, "aio wait write");
  CHECK(hds_aio_pread(h, dst.data(), bytes, path.c_str(), 0, 0) == 0, "aio pread");
  CHECK(memcmp(src.data(), dst.data(), bytes) == 0, "aio round trip mismatch");
  // many tracked requests in flight (more chunks than queue slots), waited out of order
  const int nreq = 12;
  const int64_t rb = (1 << 20) + 4096 * 3;
  std::vector<std::vector<unsigned char>> bufs(nreq, std::vector<unsigned char>(rb));
  std::vector<int64_t> ids;
  for (int r = 0; r < nreq; ++r) {
    for (int64_t i = 0; i < rb; ++i) bufs[r][i] = (unsigned char)(i * 7 + r);
    ids.push_back(hds_aio_submit(h, 1, bufs[r].data(), rb, path.c_str(), r * rb));
    CHECK(ids.back() > 0, "aio submit write");
  }
  for (int r = nreq - 1; r >= 0; --r) CHECK(hds_aio_wait_req(h, ids[r]) == 0, "aio wait_req write %d", r);
  std::vector<unsigned char> back(rb);
  for (int r = 0; r < nreq; ++r) {
    const int64_t id = hds_aio_submit(h, 0, back.data(), rb, path.c_str(), r * rb);
    CHECK(hds_aio_wait_req(h, id) == 0, "aio wait_req read");
    CHECK(memcmp(back.data(), bufs[r].data(), rb) == 0, "aio request %d mismatch", r);
  }
  CHECK(hds_aio_wait_req(h, 999999) != 0, "unknown request id must fail");
  hds_aio_destroy(h);
  unlink(path.c_str());
}

static void test_aio(const char* dir) {
  test_aio_engine(dir);  // io_uring when the kernel allows it
  setenv("HDS_AIO_ENGINE", "threads", 1);
  void* h = hds_aio_create(1 << 20, 8, 0, 1, 4);
  CHECK(hds_aio_engine(h) == 0, "HDS_AIO_ENGINE=threads must select the thread pool");
  hds_aio_destroy(h);
  test_aio_engine(dir);
  unsetenv("HDS_AIO_ENGINE");
}

static void test_shm() {
  const int64_t n = 4099;
  char name[64];
  snprintf(name, sizeof(name), "/hds_selftest_%d", (int)getpid());
  void* h0 = hds_shm_open(name, 0, 2, n * 4, 1);
  void* h1 = hds_shm_open(name, 1, 2, n * 4, 0);
  CHECK(h0 && h1, "shm open");
  if (!h0 || !h1) return;
  std::vector<float> a(n), b(n);
  std::vector<uint16_t> ha(n), hb(n);
  for (int64_t i = 0; i < n; ++i) {
    a[i] = (float)i;
    b[i] = 2.f * i;
    ha[i] = f2bf(1.5f);
    hb[i] = f2bf(0.25f);
  }
  for (int round = 0; round < 3; ++round) {  // repeated rounds exercise the generation counters
    std::vector<float> ca = a, cb = b;
    std::thread t0([&] { hds_shm_allreduce(h0, ca.data(), n, 0); });
    std::thread t1([&] { hds_shm_allreduce(h1, cb.data(), n, 0); });
    t0.join();
    t1.join();
    for (int64_t i = 0; i < n; ++i) {
      CHECK(ca[i] == 3.f * i && cb[i] == 3.f * i, "shm fp32 round %d at %ld", round, (long)i);
      if (ca[i] != 3.f * i) break;
    }
  }
  std::thread t0([&] { hds_shm_allreduce(h0, ha.data(), n, 1); });
  std::thread t1([&] { hds_shm_allreduce(h1, hb.data(), n, 1); });
  t0.join();
  t1.join();
  CHECK(bf2f(ha[0]) == 1.75f && bf2f(hb[n - 1]) == 1.75f, "shm bf16");
  hds_shm_close(h1, 0);
  hds_shm_close(h0, 1);
}

int main(int argc, char** argv) {
  const char* dir = argc > 1 ? argv[1] : "/tmp";
  test_adam();
  test_aio(dir);
  test_shm();
  if (fails) {
    fprintf(stderr, "%d check(s) failed\n", fails);
    return 1;
  }
  printf("host selftest ok\n");
  return 0;
}
