// copy_pool.h -- the host copiers of the staging pipeline (no HIP: tests/cpp/copy_pool_test.cc builds it alone under
// ThreadSanitizer and AddressSanitizer).  Persistent threads copy pageable data into the pinned staging slots in
// parallel: one thread's memcpy (~10-25 GB/s) is below the PCIe Gen5 x16 rate the slots are drained at (~55 GB/s).
#pragma once
#include <pthread.h>
#include <sched.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <cstdint>
#include <cstring>
#include <mutex>
#include <thread>
#include <utility>
#include <vector>

namespace kvsep {

struct CopySeg {
  uint8_t* dst;
  const uint8_t* src;
  uint64_t n;
  uint8_t* dst2 = nullptr;  // optional second destination ("tee"): the bytes also land here, read from cache
};

class CopyPool {
 public:
  // cpus: the CPUs the workers run on (the staged device's NUMA node), or empty for the creator's affinity.
  explicit CopyPool(int nthreads, std::vector<int> cpus = {}) : cpus_(std::move(cpus)) {
    for (int i = 0; i < nthreads; ++i) th_.emplace_back([this] { worker(); });
  }
  ~CopyPool() {
    {
      std::lock_guard<std::mutex> g(m_);
      stop_ = true;
    }
    cv_.notify_all();
    for (auto& t : th_) t.join();
  }
  // Chunks of <= 1 MiB, grouped into units of >= 256 KiB of consecutive chunks, are claimed from one counter by the
  // workers and the caller alike.  A claim per unit, not per chunk: 16 K blocks of 4 KiB were 16 K claims on one
  // counter line per 64 MiB slot, and the gather ran at half the PCIe rate.
  void run(const CopySeg* segs, uint64_t nseg) {
    chunks_.clear();
    units_.clear();
    uint64_t acc = 0, first = 0;
    for (uint64_t i = 0; i < nseg; ++i)
      for (uint64_t o = 0; o < segs[i].n; o += kChunk) {
        const uint64_t n = std::min<uint64_t>(kChunk, segs[i].n - o);
        chunks_.push_back({segs[i].dst + o, segs[i].src + o, n, segs[i].dst2 ? segs[i].dst2 + o : nullptr});
        if ((acc += n) >= kUnit) {
          units_.push_back({first, chunks_.size()});
          first = chunks_.size();
          acc = 0;
        }
      }
    if (first < chunks_.size()) units_.push_back({first, chunks_.size()});
    if (units_.size() <= 2 || th_.empty()) {  // not worth waking anyone
      for (auto& c : chunks_) copy(c);
      return;
    }
    {
      std::lock_guard<std::mutex> g(m_);
      next_.store(0);
      active_ = int(th_.size());
      ++gen_;
    }
    cv_.notify_all();
    drain();
    std::unique_lock<std::mutex> lk(m_);
    done_cv_.wait(lk, [this] { return active_ == 0; });
  }

 private:
  static constexpr uint64_t kChunk = 1ull << 20;
  static constexpr uint64_t kUnit = 256ull << 10;
  static constexpr uint64_t kTee = 64ull << 10;  // a tee copies 64 KiB to dst, then the same 64 KiB (cached) to dst2
  static void copy(const CopySeg& c) {
    if (!c.dst2) {
      std::memcpy(c.dst, c.src, c.n);
      return;
    }
    for (uint64_t o = 0; o < c.n; o += kTee) {
      const uint64_t m = std::min(kTee, c.n - o);
      std::memcpy(c.dst + o, c.src + o, m);
      std::memcpy(c.dst2 + o, c.dst + o, m);
    }
  }
  void drain() {
    for (uint64_t k; (k = next_.fetch_add(1)) < units_.size();)
      for (uint64_t c = units_[k].first; c < units_[k].second; ++c) copy(chunks_[c]);
  }
  void worker() {
    pthread_setname_np(pthread_self(), "kvsep-copy");
    if (!cpus_.empty()) {
      cpu_set_t s;
      CPU_ZERO(&s);
      for (int c : cpus_)
        if (c >= 0 && c < CPU_SETSIZE) CPU_SET(c, &s);
      (void)sched_setaffinity(0, sizeof s, &s);
    }
    uint64_t seen = 0;
    for (;;) {
      {
        std::unique_lock<std::mutex> lk(m_);
        cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
        if (stop_) return;
        seen = gen_;
      }
      drain();
      std::lock_guard<std::mutex> g(m_);
      if (--active_ == 0) done_cv_.notify_one();
    }
  }
  const std::vector<int> cpus_;
  std::vector<std::thread> th_;
  std::vector<CopySeg> chunks_;
  std::vector<std::pair<uint64_t, uint64_t>> units_;  // [first, end) chunk ranges claimed as one
  std::atomic<uint64_t> next_{0};
  std::mutex m_;
  std::condition_variable cv_, done_cv_;
  uint64_t gen_ = 0;
  int active_ = 0;
  bool stop_ = false;
};

}  // namespace kvsep
