// CPU test of the host-buffer pipeline's protocol (mplib_amd/csrc/mpg_hostpipe.h)
// with a fake device: every "device" step runs on its own std::async thread
// after a random delay and reads its slot's input only then, so a slot that
// the feeder refilled too early gives wrong results.  Ragged sizes around the
// chunk boundaries, 1..3 slots, and failures injected in the feeder and the
// issuing thread (the run must return the status and not hang).
// Usage: hostpipe_test  -> prints "ok <cases>" or the first failure, exit 1.
#include <chrono>
#include <cstdio>
#include <future>
#include <random>
#include <vector>

#include "../../mplib_amd/csrc/mpg_hostpipe.h"

namespace {

constexpr int kRow = 7;

uint64_t mix(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

uint64_t row_hash(const double* r) {
  uint64_t h = 0;
  for (int k = 0; k < kRow; ++k) h = mix(h ^ (uint64_t)(r[k] * 1e6));
  return h;
}

// the "collide": flag ~ 1 in 5, mask row nonzero exactly when flagged
void ref_row(const double* r, int W, uint8_t& f, uint32_t* m) {
  const uint64_t h = row_hash(r);
  f = (h % 5) == 0;
  for (int k = 0; k < W; ++k) m[k] = f ? (uint32_t)mix(h + k) | (k == 0 ? 1u : 0u) : 0u;
}

struct FakeOps {
  const double* q;
  uint8_t* flags;
  uint32_t* masks;
  int W;
  int64_t chunk;
  int fail_h2d = -1, fail_issue = -1;
  std::mt19937 rng_feed{1}, rng_main{2};  // one per calling thread
  std::vector<std::vector<double>> in;
  std::vector<std::vector<uint8_t>> dfl;
  std::vector<std::vector<uint32_t>> dpk;
  std::vector<std::vector<uint32_t>> dbc;  // colliding configurations per kBlock block
  std::vector<std::future<void>> fut;
  mpg_hostpipe::Pool* pool = nullptr;
  static constexpr int64_t kBlock = 128;
  FakeOps(const double* q_, uint8_t* f_, uint32_t* m_, int W_, int64_t chunk_, int slots)
      : q(q_), flags(f_), masks(m_), W(W_), chunk(chunk_), in(slots), dfl(slots), dpk(slots), dbc(slots), fut(slots) {
    for (int j = 0; j < slots; ++j) {
      in[j].assign((size_t)chunk * kRow, 0.0);
      dfl[j].assign((size_t)chunk, 0);
      dpk[j].assign((size_t)chunk * W + 1, 0u);
      dbc[j].assign((size_t)(chunk + kBlock - 1) / kBlock, 0u);
    }
  }
  static void nap(std::mt19937& r) { std::this_thread::sleep_for(std::chrono::microseconds(r() % 60)); }
  int bind_thread() { return 0; }
  int h2d(int64_t k, int j, int64_t start, int64_t m) {
    if (k == fail_h2d) return 7;
    nap(rng_feed);
    std::copy(q + start * kRow, q + (start + m) * kRow, in[j].begin());
    return 0;
  }
  int issue(int64_t k, int j, int64_t, int64_t m) {
    if (k == fail_issue) return 9;
    const unsigned delay = rng_main() % 80;
    fut[j] = std::async(std::launch::async, [this, j, m, delay] {
      std::this_thread::sleep_for(std::chrono::microseconds(delay));
      int64_t pos = 0;
      std::vector<uint32_t> row(W);
      for (int64_t i = 0; i < m; ++i) {
        ref_row(&in[j][i * kRow], W, dfl[j][i], row.data());
        if (i % kBlock == 0) dbc[j][i / kBlock] = 0;
        dbc[j][i / kBlock] += dfl[j][i];
        if (dfl[j][i]) {
          std::copy(row.begin(), row.end(), dpk[j].begin() + pos * W);
          ++pos;
        }
      }
    });
    return 0;
  }
  int finish(int64_t, int j, int64_t start, int64_t m) {
    fut[j].get();
    mpg_hostpipe::unpack_chunk(pool, dfl[j].data(), dpk[j].data(), dbc[j].data(), kBlock, m, W, flags + start,
                               masks ? masks + start * W : nullptr);
    return 0;
  }
  void drain() {
    for (auto& f : fut)
      if (f.valid()) f.wait();
  }
};

int fails = 0;

void check(bool ok, const char* what, int64_t n, int64_t cmax, int ring) {
  if (!ok && fails++ < 10) std::printf("FAIL %s n=%lld chunk_max=%lld ring=%d\n", what, (long long)n, (long long)cmax, ring);
}

}  // namespace

int main() {
  std::mt19937_64 g(5);
  int cases = 0;
  mpg_hostpipe::Pool pool(3);
  for (int64_t n : {1ll, 63ll, 64ll, 65ll, 128ll, 129ll, 191ll, 1000ll, 4097ll, 9001ll}) {
    for (int64_t cmax : {64ll, 1000ll, 1ll << 18}) {
      for (int ring : {1, 2, 3}) {
        for (int W : {1, 5}) {
          const int64_t head = (W == 5) ? 64 : 0, tail = (ring == 3) ? 128 : 0;  // with and without small ends
          const mpg_hostpipe::Plan p = mpg_hostpipe::plan(n, cmax, 64, ring, head, tail);
          bool sizes_ok = p.chunk > 0 && p.chunk <= std::max<int64_t>(64, cmax) && p.start.front() == 0 &&
                          p.start.back() == n && (int64_t)p.start.size() == p.n_chunks + 1;
          for (int64_t k = 0; k < p.n_chunks; ++k) {
            const int64_t c = mpg_hostpipe::chunk_count(p, n, k);
            sizes_ok &= c > 0 && c <= p.chunk && (k == p.n_chunks - 1 || c % 64 == 0);
          }
          check(sizes_ok, "chunk sizes", n, cmax, ring);
          std::vector<double> q((size_t)n * kRow);
          for (auto& x : q) x = (double)(g() % 1000003) / 997.0;
          std::vector<uint8_t> f((size_t)n, 0xAB), fr((size_t)n);
          std::vector<uint32_t> m((size_t)n * W, 0xDEADBEEFu), mr((size_t)n * W);
          for (int64_t i = 0; i < n; ++i) ref_row(&q[i * kRow], W, fr[i], &mr[i * W]);
          FakeOps ops(q.data(), f.data(), m.data(), W, p.chunk, p.slots);
          if (ring != 2) ops.pool = &pool;  // the parallel unpack, and the serial one
          const int rc = mpg_hostpipe::run(p, n, ops);
          check(rc == 0 && f == fr && m == mr, "results", n, cmax, ring);
          ++cases;
          // flags only
          std::vector<uint8_t> f2((size_t)n, 0xCD);
          FakeOps ops2(q.data(), f2.data(), nullptr, W, p.chunk, p.slots);
          check(mpg_hostpipe::run(p, n, ops2) == 0 && f2 == fr, "flags only", n, cmax, ring);
          ++cases;
          // failures: the status comes back and nothing hangs
          if (p.n_chunks >= 2) {
            for (int at : {0, (int)(p.n_chunks / 2), (int)(p.n_chunks - 1)}) {
              FakeOps a(q.data(), f.data(), m.data(), W, p.chunk, p.slots);
              a.fail_h2d = at;
              check(mpg_hostpipe::run(p, n, a) == 7, "feeder failure status", n, cmax, ring);
              FakeOps b(q.data(), f.data(), m.data(), W, p.chunk, p.slots);
              b.fail_issue = at;
              check(mpg_hostpipe::run(p, n, b) == 9, "issue failure status", n, cmax, ring);
              cases += 2;
            }
          }
        }
      }
    }
  }
  // the plan's defaults for the sizes the library sees
  const auto p20 = mpg_hostpipe::plan(1ll << 20, 1ll << 18, 1ll << 15, 3);
  check(p20.chunk == (1ll << 18) && p20.n_chunks == 4 && p20.slots == 3, "plan 2^20", 1 << 20, 1 << 18, 3);
  const auto pht = mpg_hostpipe::plan(1ll << 20, 1ll << 18, 1ll << 15, 3, 1 << 16, 1 << 16);
  check(pht.n_chunks == 6 && mpg_hostpipe::chunk_count(pht, 0, 0) == (1 << 16) &&
            mpg_hostpipe::chunk_count(pht, 0, 5) == (1 << 16) && pht.chunk <= (1 << 18),
        "plan head/tail", 1 << 20, 1 << 18, 3);
  const auto p11 = mpg_hostpipe::plan(2000, 1ll << 18, 1ll << 15, 3);
  check(p11.chunk == 2000 && p11.n_chunks == 1 && p11.slots == 1, "plan 2000", 2000, 1 << 18, 3);
  const auto p24 = mpg_hostpipe::plan(1ll << 24, 1ll << 18, 1ll << 15, 3);
  check(p24.chunk == (1ll << 18) && p24.n_chunks == 64, "plan 2^24", 1 << 24, 1 << 18, 3);
  if (fails) {
    std::printf("%d failures\n", fails);
    return 1;
  }
  std::printf("ok %d\n", cases);
  return 0;
}
