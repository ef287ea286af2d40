// ref_shim.cc -- TEST INFRASTRUCTURE ONLY.
// Exposes the *real* reference implementation (/root/reference/util/crc32c.cc, compiled
// from its own source file by oracle/Makefile) through a C ABI so tests/golden/make_golden.py
// can capture golden vectors with ctypes.  Nothing here is shipped or measured.
#include <cstddef>
#include <cstdint>

#include "util/crc32c.h"  // /root/reference/util/crc32c.h:17-38

extern "C" {
uint32_t ref_crc32c_extend(uint32_t init, const char* data, size_t n) {
  return leveldb::crc32c::Extend(init, data, n);  // util/crc32c.cc:276
}
uint32_t ref_crc32c_value(const char* data, size_t n) { return leveldb::crc32c::Value(data, n); }
uint32_t ref_crc32c_mask(uint32_t c) { return leveldb::crc32c::Mask(c); }
uint32_t ref_crc32c_unmask(uint32_t m) { return leveldb::crc32c::Unmask(m); }
}

// Batched driver over the reference Extend (same contract as oracle_crc32c_batch): blocks split over
// `nthreads` host threads by contiguous byte-balanced ranges.  Used as bench.py's cpu_baseline
// ("reference" kind) so the baseline is the reference's own code, compiled -O3.
#include <pthread.h>

namespace {
struct RefJob {
  const char* base; const uint64_t* off; const uint64_t* len; const uint32_t* init; uint32_t* out;
  size_t lo, hi;
};
void* ref_worker(void* p) {
  RefJob* j = static_cast<RefJob*>(p);
  for (size_t i = j->lo; i < j->hi; ++i)
    j->out[i] = leveldb::crc32c::Extend(j->init ? j->init[i] : 0u, j->base + j->off[i], j->len[i]);
  return nullptr;
}
}  // namespace

extern "C" int ref_crc32c_batch(const char* base, const uint64_t* off, const uint64_t* len, const uint32_t* init,
                                uint32_t* out, size_t count, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  uint64_t total = 0;
  for (size_t i = 0; i < count; ++i) total += len[i];
  pthread_t th[256];
  RefJob jobs[256];
  size_t start = 0;
  uint64_t acc = 0;
  int launched = 0;
  for (int t = 0; t < nthreads && start < count; ++t) {
    const uint64_t target = (total / uint64_t(nthreads)) * uint64_t(t + 1);
    size_t stop = start;
    if (t == nthreads - 1) stop = count;
    else
      while (stop < count && acc < target) acc += len[stop++];
    jobs[t] = RefJob{base, off, len, init, out, start, stop};
    if (pthread_create(&th[t], nullptr, ref_worker, &jobs[t]) != 0) return -1;
    ++launched;
    start = stop;
  }
  for (int t = 0; t < launched; ++t) pthread_join(th[t], nullptr);
  return 0;
}

// Full-size golden vectors (tests/golden/make_fullsize_golden.py): out[i] = reference Extend(0, block i) where block
// i is bytes [stream_base + off[i], + len[i]) of the repo's splitmix64 stream `seed` (kvsep/workloads.py), generated
// on the fly into a per-thread buffer at the block's own alignment mod 16, so whole BASELINE batches (64 GiB ..
// 512 GiB) are checksummed by the reference without holding them in memory.  Threads take contiguous,
// byte-balanced block ranges.
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {
inline uint64_t sm_word(uint64_t seed, uint64_t j) {
  uint64_t z = seed + (j + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
struct StreamJob {
  uint64_t seed, base;
  const uint64_t* off; const uint64_t* len; uint32_t* out;
  size_t lo, hi;
};
void* stream_worker(void* p) {
  StreamJob* j = static_cast<StreamJob*>(p);
  uint64_t maxlen = 0;
  for (size_t i = j->lo; i < j->hi; ++i) maxlen = j->len[i] > maxlen ? j->len[i] : maxlen;
  std::vector<uint64_t> words((maxlen + 32) / 8 + 2);
  std::vector<char> buf(maxlen + 32);
  for (size_t i = j->lo; i < j->hi; ++i) {
    const uint64_t g0 = j->base + j->off[i], n = j->len[i];
    const uint64_t nw = (n + (g0 & 7) + 7) / 8;
    for (uint64_t k = 0; k < nw; ++k) words[k] = sm_word(j->seed, (g0 >> 3) + k);  // little-endian host
    char* at = buf.data() + (j->off[i] & 15);
    std::memcpy(at, reinterpret_cast<const char*>(words.data()) + (g0 & 7), n);
    j->out[i] = leveldb::crc32c::Extend(0, at, n);
  }
  return nullptr;
}
}  // namespace

extern "C" int ref_crc32c_stream_batch(uint64_t seed, uint64_t stream_base, const uint64_t* off, const uint64_t* len,
                                       size_t count, uint32_t* out, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  uint64_t total = 0;
  for (size_t i = 0; i < count; ++i) total += len[i];
  pthread_t th[256];
  StreamJob jobs[256];
  size_t start = 0;
  uint64_t acc = 0;
  int launched = 0;
  for (int t = 0; t < nthreads && start < count; ++t) {
    const uint64_t target = (total / uint64_t(nthreads)) * uint64_t(t + 1);
    size_t stop = start;
    if (t == nthreads - 1) stop = count;
    else
      while (stop < count && acc < target) acc += len[stop++];
    jobs[t] = StreamJob{seed, stream_base, off, len, out, start, stop};
    if (pthread_create(&th[t], nullptr, stream_worker, &jobs[t]) != 0) return -1;
    ++launched;
    start = stop;
  }
  for (int t = 0; t < launched; ++t) pthread_join(th[t], nullptr);
  return 0;
}

// The CPU baseline of bench.py (cpu_baseline, kind "reference"): the reference Extend over a sample of blocks on
// `nthreads` host threads for about `seconds`, each thread pinned to cpus[t] (when given) and working on its OWN copy
// of its byte-balanced block range, made by itself before the clock starts -- first touch places those pages on the
// thread's NUMA node, so a 2-socket box is measured on local memory instead of on the one node the shared sample sits
// on.  Every thread passes over its range repeatedly until the common deadline; *bytes_out is the total checksummed,
// *secs_out the elapsed time from the common start to the last thread's end.  Returns 0, or -1 if a thread or a
// buffer could not be created.
#include <sched.h>

#include <atomic>
#include <chrono>

namespace {
struct LocalJob {
  const char* src; const uint64_t* off; const uint64_t* len;
  size_t lo, hi;
  int cpu;
  double seconds;
  std::atomic<int>* ready;   // threads done with their copy
  std::atomic<int>* abort;   // set when a thread could not be created: nobody waits for it
  int nthreads;
  std::atomic<double>* t0;
  uint64_t bytes = 0;
  double end = 0;
  uint32_t sink = 0;
  int err = 0;
};
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
void* local_worker(void* p) {
  LocalJob* j = static_cast<LocalJob*>(p);
  if (j->cpu >= 0) {
    cpu_set_t set;
    CPU_ZERO(&set);
    CPU_SET(j->cpu, &set);
    sched_setaffinity(0, sizeof set, &set);  // this thread; its later allocations follow it (first touch)
  }
  uint64_t total = 0;
  for (size_t i = j->lo; i < j->hi; ++i) total += j->len[i];
  char* mine = static_cast<char*>(std::malloc(total ? total : 1));
  std::vector<uint64_t> loff(j->hi - j->lo);
  if (!mine) j->err = 1;
  else {
    uint64_t pos = 0;
    for (size_t i = j->lo; i < j->hi; ++i) {  // the copy is this thread's first touch of its pages
      std::memcpy(mine + pos, j->src + j->off[i], j->len[i]);
      loff[i - j->lo] = pos;
      pos += j->len[i];
    }
  }
  j->ready->fetch_add(1);
  while (j->ready->load() < j->nthreads && !j->abort->load()) sched_yield();
  double expect = 0;
  if (j->t0->load() == 0) j->t0->compare_exchange_strong(expect, now_s());
  const double stop = j->t0->load() + j->seconds;
  uint32_t s = 0;
  if (mine) {
    do {
      for (size_t i = j->lo; i < j->hi; ++i) s ^= leveldb::crc32c::Extend(0, mine + loff[i - j->lo], j->len[i]);
      j->bytes += total;
    } while (now_s() < stop);
  }
  j->end = now_s();
  j->sink = s;
  std::free(mine);
  return nullptr;
}
}  // namespace

extern "C" int ref_crc32c_timed_local(const char* src, const uint64_t* off, const uint64_t* len, size_t count,
                                      int nthreads, const int* cpus, double seconds, uint64_t* bytes_out,
                                      double* secs_out) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 1024) nthreads = 1024;
  uint64_t total = 0;
  for (size_t i = 0; i < count; ++i) total += len[i];
  std::vector<LocalJob> jobs(nthreads);
  std::vector<pthread_t> th(nthreads);
  std::atomic<int> ready{0}, abort{0};
  std::atomic<double> t0{0};
  size_t start = 0;
  uint64_t acc = 0;
  int n = 0;
  for (int t = 0; t < nthreads && start < count; ++t, ++n) {
    const uint64_t target = (total / uint64_t(nthreads)) * uint64_t(t + 1);
    size_t stop = start;
    if (t == nthreads - 1) stop = count;
    else
      while (stop < count && acc < target) acc += len[stop++];
    if (stop == start && stop < count) acc += len[stop++];  // at least one block per thread
    jobs[t].src = src; jobs[t].off = off; jobs[t].len = len;
    jobs[t].lo = start; jobs[t].hi = stop;
    jobs[t].cpu = cpus ? cpus[t] : -1;
    jobs[t].seconds = seconds;
    jobs[t].t0 = &t0;
    start = stop;
  }
  int rc = 0, launched = 0;
  for (int t = 0; t < n; ++t) {
    jobs[t].ready = &ready;
    jobs[t].abort = &abort;
    jobs[t].nthreads = n;
    if (pthread_create(&th[t], nullptr, local_worker, &jobs[t]) != 0) {
      rc = -1;
      abort.store(1);  // the started threads stop waiting for the missing ones
      break;
    }
    ++launched;
  }
  double end = 0;
  uint64_t bytes = 0;
  for (int t = 0; t < launched; ++t) {
    pthread_join(th[t], nullptr);
    end = jobs[t].end > end ? jobs[t].end : end;
    bytes += jobs[t].bytes;
    if (jobs[t].err) rc = -1;
  }
  if (bytes_out) *bytes_out = bytes;
  if (secs_out) *secs_out = end - t0.load();
  return rc;
}
