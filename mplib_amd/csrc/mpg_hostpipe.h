// mpg_hostpipe.h -- host side of the host-buffer collide pipeline (no HIP).
//
// A caller that hands mpg_collide_batch host buffers (MPG_MEM_HOST: the
// route of PlanningWorld.collide_batch(numpy) and of a C++ binding of the
// reference's collide(), include/mpgpu.h) pays PCIe twice per configuration.
// The batch runs as chunks through a ring of `slots` device/pinned buffers:
//   feeder thread   h2d(k)     copy chunk k's rows to slot k % slots
//   issuer thread   issue(k)   queue chunk k's compute once its rows are there
//   caller          finish(k)  wait for chunk k's results, unpack them
// so the input of one chunk crosses PCIe while earlier ones compute and are
// unpacked.  Slot j is refilled (chunk k + slots) only after finish(k) has
// consumed it.  The protocol and the unpacking live here so the
// CPU tests can drive them with a fake device (tests/native/hostpipe_test.cpp).
#pragma once

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <functional>
#include <mutex>
#include <thread>
#include <vector>

namespace mpg_hostpipe {

struct Plan {
  int64_t chunk = 0;             // the largest chunk (a slot's capacity)
  int64_t n_chunks = 0;
  int slots = 0;
  std::vector<int64_t> start;    // chunk k = [start[k], start[k + 1])
};

inline int64_t round64(int64_t x) { return (x + 63) / 64 * 64; }

// Chunks of at most chunk_max configurations, at least four when that keeps
// them >= min_chunk (the pipeline needs chunks to overlap; below ~2^15
// configurations a chunk's launches dominate), multiples of 64 (a wave's
// tile) but for the last.  Optionally a smaller first chunk (`head`: the
// device starts once it has crossed PCIe) and last chunk (`tail`: the compute
// and unpacking left after the last input copy); the rest is split evenly.
inline Plan plan(int64_t n, int64_t chunk_max, int64_t min_chunk, int ring, int64_t head = 0, int64_t tail = 0) {
  Plan p;
  if (n <= 0) return p;
  int64_t c = round64((n + 3) / 4);
  c = std::max(c, min_chunk);
  c = std::min(c, std::max<int64_t>(64, chunk_max / 64 * 64));
  c = std::min(c, n);
  std::vector<int64_t> sz;
  int64_t rest = n;
  const int64_t h = round64(head), t = round64(tail);
  if (h > 0 && h < c && rest >= h + 2 * c) {
    sz.push_back(h);
    rest -= h;
  }
  const bool use_t = t > 0 && t < c && rest >= t + 2 * c;
  int64_t tlen = 0;
  if (use_t) {  // the tail also takes the ragged end, so every other chunk is a multiple of 64
    tlen = t + rest % 64;
    rest -= tlen;
  }
  const int64_t k = (rest + c - 1) / c;
  const int64_t e = std::min(c, round64((rest + k - 1) / k));
  for (int64_t left = rest; left > 0; left -= std::min(e, left)) sz.push_back(std::min(e, left));
  if (use_t) sz.push_back(tlen);
  p.start.assign(1, 0);
  for (int64_t x : sz) {
    p.start.push_back(p.start.back() + x);
    p.chunk = std::max(p.chunk, x);
  }
  p.n_chunks = (int64_t)sz.size();
  p.slots = (int)std::min<int64_t>(ring, p.n_chunks);
  return p;
}

inline int64_t chunk_start(const Plan& p, int64_t k) { return p.start[(size_t)k]; }
inline int64_t chunk_count(const Plan& p, int64_t, int64_t k) { return p.start[(size_t)k + 1] - p.start[(size_t)k]; }

// flags[i] != 0 exactly when configuration i has a mask bit; `packed` holds
// those rows in configuration order; out[i] = packed row or zeros
inline void unpack_masks(const uint8_t* fl, const uint32_t* packed, int64_t m, int W, uint32_t* out) {
  int64_t pos = 0;
  for (int64_t i = 0; i < m; ++i, out += W) {
    if (fl[i]) {
      const uint32_t* src = packed + pos * W;
      for (int k = 0; k < W; ++k) out[k] = src[k];
      ++pos;
    } else {
      for (int k = 0; k < W; ++k) out[k] = 0u;
    }
  }
}

// A few persistent helper threads for the host-side copies of a finished
// chunk: run(tasks, fn) calls fn(0..tasks-1) on the helpers and the caller
// and returns when all are done.  One run at a time (the caller holds the
// world's host_mu).
class Pool {
 public:
  explicit Pool(int helpers) {
    for (int i = 0; i < helpers; ++i) th_.emplace_back([this] { loop(); });
  }
  ~Pool() {
    {
      std::lock_guard<std::mutex> lk(mu_);
      quit_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  int threads() const { return (int)th_.size() + 1; }
  template <class F>
  void run(int tasks, const F& fn) {
    if (tasks <= 0) return;
    if (th_.empty() || tasks == 1) {
      for (int i = 0; i < tasks; ++i) fn(i);
      return;
    }
    std::function<void(int)> f(fn);
    {
      std::lock_guard<std::mutex> lk(mu_);
      fn_ = &f;
      n_ = tasks;
      next_ = 0;
      left_ = tasks;
      ++gen_;
    }
    cv_.notify_all();
    work();
    std::unique_lock<std::mutex> lk(mu_);
    done_cv_.wait(lk, [this] { return left_ == 0; });
    fn_ = nullptr;
  }

 private:
  void work() {
    for (;;) {
      int i;
      const std::function<void(int)>* f;
      {
        std::lock_guard<std::mutex> lk(mu_);
        if (!fn_ || next_ >= n_) return;
        i = next_++;
        f = fn_;
      }
      (*f)(i);
      std::lock_guard<std::mutex> lk(mu_);
      if (--left_ == 0) done_cv_.notify_all();
    }
  }
  void loop() {
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(mu_);
        cv_.wait(lk, [&] { return quit_ || gen_ != seen; });
        if (quit_) return;
        seen = gen_;
      }
      work();
    }
  }
  std::vector<std::thread> th_;
  std::mutex mu_;
  std::condition_variable cv_, done_cv_;
  const std::function<void(int)>* fn_ = nullptr;
  int n_ = 0, next_ = 0, left_ = 0;
  uint64_t gen_ = 0;
  bool quit_ = false;
};

// flags and masks of one finished chunk of m configurations into the
// caller's buffers, in parallel over ranges of whole pack blocks (`block`
// configurations each; bcnt[b] = colliding configurations of block b, so a
// range's first packed row is known without scanning the flags before it)
inline void unpack_chunk(Pool* pool, const uint8_t* fl, const uint32_t* packed, const uint32_t* bcnt, int64_t block,
                         int64_t m, int W, uint8_t* flags_out, uint32_t* masks_out) {
  const int64_t nb = (m + block - 1) / block;
  const int parts = (int)std::min<int64_t>(nb, pool ? pool->threads() : 1);
  auto part = [&](int t) {
    const int64_t b0 = nb * t / parts, b1 = nb * (t + 1) / parts;
    int64_t pos = 0;
    if (masks_out)
      for (int64_t b = 0; b < b0; ++b) pos += bcnt[b];
    const int64_t i0 = b0 * block, i1 = std::min(m, b1 * block);
    std::memcpy(flags_out + i0, fl + i0, (size_t)(i1 - i0));
    if (masks_out) unpack_masks(fl + i0, packed + pos * W, i1 - i0, W, masks_out + i0 * W);
  };
  if (pool) {
    pool->run(parts, part);
  } else {
    for (int t = 0; t < parts; ++t) part(t);
  }
}

inline void relax(int& spins) {
  if (++spins < 256) {
#if defined(__x86_64__)
    __builtin_ia32_pause();
#endif
  } else {
    std::this_thread::yield();
  }
}

// Ops: int bind_thread()                                      (each thread's start)
//      int h2d(int64_t k, int slot, int64_t start, int64_t count)    (feeder thread)
//      int issue(int64_t k, int slot, int64_t start, int64_t count)  (issuer thread)
//      int finish(int64_t k, int slot, int64_t start, int64_t count) (caller)
//      void drain()   after a failure: wait until no queued work uses a slot
// Three threads, so a blocking input copy, the launches of the next chunk and
// the unpacking of a finished one proceed at once.  Returns 0 or the first
// non-zero status (the caller's, else the feeder's, else the issuer's).
template <class Ops>
int run(const Plan& p, int64_t n, Ops& ops) {
  if (p.n_chunks == 0) return 0;
  const int S = p.slots;
  const int64_t K = p.n_chunks;
  std::atomic<int64_t> staged{0};         // chunks [0, staged) are in their slots
  std::atomic<int64_t> issued{0};         // chunks [0, issued) are queued on the device
  std::atomic<int64_t> freed{(int64_t)S};  // chunk k may be staged once k < freed
  std::atomic<bool> stop{false};
  auto wait_for = [&](std::atomic<int64_t>& c, int64_t want) {
    for (int spins = 0; c.load(std::memory_order_acquire) < want;) {
      if (stop.load(std::memory_order_acquire)) return c.load(std::memory_order_acquire) >= want;
      relax(spins);
    }
    return true;
  };
  int feed_rc = 0, issue_rc = 0;
  auto feed = [&] {
    feed_rc = ops.bind_thread();
    for (int64_t k = 0; k < K && !feed_rc; ++k) {
      if (!wait_for(freed, k + 1)) return;
      feed_rc = ops.h2d(k, (int)(k % S), chunk_start(p, k), chunk_count(p, n, k));
      if (!feed_rc) staged.store(k + 1, std::memory_order_release);
    }
    if (feed_rc) stop.store(true, std::memory_order_release);
  };
  auto iss = [&] {
    issue_rc = ops.bind_thread();
    for (int64_t k = 0; k < K && !issue_rc; ++k) {
      if (!wait_for(staged, k + 1)) return;
      issue_rc = ops.issue(k, (int)(k % S), chunk_start(p, k), chunk_count(p, n, k));
      if (!issue_rc) issued.store(k + 1, std::memory_order_release);
    }
    if (issue_rc) stop.store(true, std::memory_order_release);
  };
  std::thread feeder, issuer;
  if (K > 1) {
    feeder = std::thread(feed);
    issuer = std::thread(iss);
  } else {
    feed();
    if (!feed_rc) iss();
  }
  int rc = 0;
  for (int64_t k = 0; k < K && !rc; ++k) {
    if (!wait_for(issued, k + 1)) break;  // the feeder or the issuer failed
    rc = ops.finish(k, (int)(k % S), chunk_start(p, k), chunk_count(p, n, k));
    if (!rc) freed.store(k + 1 + S, std::memory_order_release);
  }
  if (rc) stop.store(true, std::memory_order_release);
  if (feeder.joinable()) feeder.join();
  if (issuer.joinable()) issuer.join();
  if (!rc) rc = feed_rc ? feed_rc : issue_rc;
  if (rc) ops.drain();
  return rc;
}

}  // namespace mpg_hostpipe
