// crc32c_host.cpp -- host half of libkvsep_crc32c: the scalar drop-in (Extend / Value / Mask /
// Unmask / AcceleratedCRC32C; its host legs are in host_crc.cpp), the host-memory batch entry points (pinned staging,
// H2D, kernel, D2H over two streams), and build info.
//
// Reference interfaces replaced (see include/kvsep_crc32c.h for the full list):
//   util/crc32c.h:17   leveldb::crc32c::Extend      -> kvsep_crc32c_extend
//   port/port_stdcxx.h:142 port::AcceleratedCRC32C  -> kvsep_accelerated_crc32c
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <thread>
#include <utility>
#include <vector>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>

#include "../../include/kvsep_crc32c.h"
#include "host_crc.h"
#include "kvsep_internal.h"
#include "numa.h"

namespace kvsep {

CopyPool* copy_pool_create(const std::vector<int>& cpus) {
  int n = 7;  // + the caller: 8 copiers
  if (const char* v = std::getenv("KVSEP_COPY_THREADS")) n = std::max(0, std::atoi(v) - 1);
  const int hw = cpus.empty() ? int(std::thread::hardware_concurrency()) : int(cpus.size());
  if (hw > 0) n = std::min(n, std::max(0, hw - 1));
  return new CopyPool(n, cpus);
}
void copy_pool_destroy(CopyPool* p) { delete p; }
void copy_pool_run(CopyPool* p, const CopySeg* segs, uint64_t nseg) { p->run(segs, nseg); }

void release_staging(HostStaging& s) {
  for (int i = 0; i < HostStaging::kSlots; ++i) {
    if (s.stream[i]) hipStreamSynchronize(s.stream[i]);
    hipHostFree(s.h_data[i]); hipHostFree(s.h_desc[i]); hipHostFree(s.h_init[i]); hipHostFree(s.h_out[i]);
    hipFree(s.d_data[i]); hipFree(s.d_desc[i]); hipFree(s.d_init[i]); hipFree(s.d_out[i]);
    if (s.done[i]) hipEventDestroy(s.done[i]);
    free_scratch(s.scratch[i]);
    if (s.stream[i]) hipStreamDestroy(s.stream[i]);
  }
  copy_pool_destroy(s.pool);
  s = HostStaging();
}

namespace {

std::atomic<uint64_t> g_offload_threshold{64ull << 20};
std::atomic<uint64_t> g_gpu_calls{0}, g_host_calls{0}, g_gpu_failures{0};

// ------------------------------------------------------------------ staging pipeline
constexpr uint64_t kSlotBytes = 64ull << 20;
constexpr uint64_t kSlotBlocks = 1ull << 16;

int hip_fail(const char* what, hipError_t e) {
  char buf[384];
  snprintf(buf, sizeof buf, "%s: %s (%d)", what, hipGetErrorString(e), int(e));
  set_last_error(buf);
  return KVSEP_EHIP;
}

#define KVSEP_HIPH(call)                              \
  do {                                                \
    hipError_t _e = (call);                           \
    if (_e != hipSuccess) return hip_fail(#call, _e); \
  } while (0)

int ensure_staging_once(HostStaging& s) {
  s.bytes = kSlotBytes;
  s.max_blocks = kSlotBlocks;
  for (int i = 0; i < HostStaging::kSlots; ++i) {
    KVSEP_HIPH(hipHostMalloc(reinterpret_cast<void**>(&s.h_data[i]), s.bytes, hipHostMallocDefault));
    KVSEP_HIPH(hipHostMalloc(reinterpret_cast<void**>(&s.h_desc[i]), 2 * s.max_blocks * 8, hipHostMallocDefault));
    KVSEP_HIPH(hipHostMalloc(reinterpret_cast<void**>(&s.h_init[i]), s.max_blocks * 4, hipHostMallocDefault));
    KVSEP_HIPH(hipHostMalloc(reinterpret_cast<void**>(&s.h_out[i]), s.max_blocks * 4, hipHostMallocDefault));
    KVSEP_HIPH(hipMalloc(&s.d_data[i], s.bytes));
    KVSEP_HIPH(hipMalloc(&s.d_desc[i], 2 * s.max_blocks * 8));
    KVSEP_HIPH(hipMalloc(&s.d_init[i], s.max_blocks * 4));
    KVSEP_HIPH(hipMalloc(&s.d_out[i], s.max_blocks * 4));
    KVSEP_HIPH(hipStreamCreateWithFlags(&s.stream[i], hipStreamNonBlocking));
    KVSEP_HIPH(hipEventCreateWithFlags(&s.done[i], hipEventDisableTiming));
  }
  return KVSEP_OK;
}

// Pinned slots, device slots, streams and events of the host entry points, created on first use.  A failure
// part-way frees what was created (nothing leaks into the next attempt).  It is retried after a backoff that doubles
// with each consecutive failure (10 ms .. 10 s): a transient shortage of pinned memory is not a permanent
// KVSEP_ENOMEM for the context, and meanwhile the framing writers' payload copies go straight to memcpy instead of
// retrying the allocation on every call.
int ensure_staging(kvsep_crc32c_ctx* c) {
  HostStaging& s = ctx_staging(c);
  if (s.ready) return KVSEP_OK;
  const int64_t now = std::chrono::duration_cast<std::chrono::nanoseconds>(
                          std::chrono::steady_clock::now().time_since_epoch()).count();
  if (s.failures && now < s.retry_at_ns) {
    set_last_error("host staging could not be allocated on this context (retried after a backoff)");
    return KVSEP_ENOMEM;
  }
  DeviceGuard dg(ctx_device(c));
  if (dg.err != hipSuccess) return hip_fail("hipSetDevice", dg.err);
  // On the device's NUMA node (round 5): this thread while it allocates the pinned slots (its preferred memory node),
  // then the copier threads that fill them -- the staged bytes never cross the socket link on their way to the GPU.
  numa::ScopedBind bind(ctx_host_node(c));
  const int rc = ensure_staging_once(s);
  if (rc != KVSEP_OK) {
    std::string msg = kvsep_last_error();
    release_staging(s);
    const int64_t backoff = std::min<int64_t>(10'000'000ll << std::min<uint32_t>(s.failures, 10), 10'000'000'000ll);
    ++s.failures;
    s.retry_at_ns = now + backoff;
    set_last_error(msg.c_str());
    return rc;
  }
  s.failures = 0;
  s.cpus = bind.cpus();
  s.pool = copy_pool_create(s.cpus);
  s.ready = true;
  return KVSEP_OK;
}

bool is_pinned(const void* p) {
  hipPointerAttribute_t attr;
  if (hipPointerGetAttributes(&attr, p) != hipSuccess) {
    (void)hipGetLastError();
    return false;
  }
  return attr.type == hipMemoryTypeHost;
}

// A submitted slot: which caller indices its h_out entries belong to.
struct SlotJob {
  bool busy = false;
  uint64_t first = 0, n = 0;  // caller indices [first, first+n) in order
};

// Collect results of a slot into the caller's out[], once its D2H has landed.
int retire(HostStaging& s, int slot, SlotJob& job, uint32_t* out) {
  if (!job.busy) return KVSEP_OK;
  KVSEP_HIPH(hipEventSynchronize(s.done[slot]));
  std::memcpy(out + job.first, s.h_out[slot], job.n * 4);
  job.busy = false;
  return KVSEP_OK;
}

// Submit the staged group in `slot`: the payload already sits in d_data (H2D queued) or h_data.
int submit(kvsep_crc32c_ctx* c, HostStaging& s, int slot, uint64_t nblk, uint64_t payload, uint64_t max_len,
           const uint8_t* pinned_src, bool have_init) {
  hipStream_t st = s.stream[slot];
  const uint8_t* src = pinned_src ? pinned_src : s.h_data[slot];
  KVSEP_HIPH(hipMemcpyAsync(s.d_data[slot], src, payload, hipMemcpyHostToDevice, st));
  KVSEP_HIPH(hipMemcpyAsync(s.d_desc[slot], s.h_desc[slot], nblk * 8, hipMemcpyHostToDevice, st));
  KVSEP_HIPH(hipMemcpyAsync(s.d_desc[slot] + s.max_blocks, s.h_desc[slot] + s.max_blocks, nblk * 8,
                            hipMemcpyHostToDevice, st));
  if (have_init) KVSEP_HIPH(hipMemcpyAsync(s.d_init[slot], s.h_init[slot], nblk * 4, hipMemcpyHostToDevice, st));
  int rc = device_batch_locked(c, s.scratch[slot], st, s.d_data[slot], s.d_desc[slot],
                               s.d_desc[slot] + s.max_blocks, have_init ? s.d_init[slot] : nullptr, s.d_out[slot],
                               nblk, payload, max_len);
  if (rc) return rc;
  KVSEP_HIPH(hipMemcpyAsync(s.h_out[slot], s.d_out[slot], nblk * 4, hipMemcpyDeviceToHost, st));
  KVSEP_HIPH(hipEventRecord(s.done[slot], st));
  return KVSEP_OK;
}

// One block longer than a slot: chain slot-sized segments, each seeded with the previous CRC.
int big_block(kvsep_crc32c_ctx* c, HostStaging& s, SlotJob* jobs, uint32_t* out, const uint8_t* p, uint64_t n,
              uint32_t init, bool pinned, uint32_t* result) {
  for (int i = 0; i < HostStaging::kSlots; ++i) {
    int rc = retire(s, i, jobs[i], out);
    if (rc) return rc;
  }
  uint32_t crc = init;
  int slot = 0;
  // Segments run on one stream; host data of segment k+1 is staged while segment k computes.
  for (uint64_t done = 0; done < n; done += s.bytes, slot ^= 1) {
    const uint64_t seg = std::min<uint64_t>(s.bytes, n - done);
    KVSEP_HIPH(hipEventSynchronize(s.done[slot]));  // previous use of this slot's buffers finished
    if (!pinned) {
      const CopySeg cs{s.h_data[slot], p + done, seg};
      copy_pool_run(s.pool, &cs, 1);
    }
    s.h_desc[slot][0] = 0;
    s.h_desc[slot][s.max_blocks] = seg;
    hipStream_t st = s.stream[0];
    KVSEP_HIPH(hipMemcpyAsync(s.d_data[slot], pinned ? p + done : s.h_data[slot], seg, hipMemcpyHostToDevice, st));
    KVSEP_HIPH(hipMemcpyAsync(s.d_desc[slot], s.h_desc[slot], 8, hipMemcpyHostToDevice, st));
    KVSEP_HIPH(hipMemcpyAsync(s.d_desc[slot] + s.max_blocks, s.h_desc[slot] + s.max_blocks, 8, hipMemcpyHostToDevice, st));
    if (done == 0) {
      s.h_init[slot][0] = crc;
      KVSEP_HIPH(hipMemcpyAsync(s.d_init[slot], s.h_init[slot], 4, hipMemcpyHostToDevice, st));
    } else {  // seed with the previous segment's CRC, straight from device memory
      KVSEP_HIPH(hipMemcpyAsync(s.d_init[slot], s.d_out[slot ^ 1], 4, hipMemcpyDeviceToDevice, st));
    }
    int rc = device_batch_locked(c, s.scratch[0], st, s.d_data[slot], s.d_desc[slot],
                                 s.d_desc[slot] + s.max_blocks, s.d_init[slot], s.d_out[slot], 1, seg, seg);
    if (rc) return rc;
    KVSEP_HIPH(hipEventRecord(s.done[slot], st));
  }
  slot ^= 1;  // slot of the last segment
  KVSEP_HIPH(hipMemcpyAsync(s.h_out[slot], s.d_out[slot], 4, hipMemcpyDeviceToHost, s.stream[0]));
  KVSEP_HIPH(hipStreamSynchronize(s.stream[0]));
  *result = s.h_out[slot][0];
  return KVSEP_OK;
}

// The drop-in's context: one per device, on the CALLER's current device (a rank bound to GPU N checksums on
// GPU N), created on first use.
constexpr int kMaxDevices = 64;
std::atomic<bool> g_dropin_busy[kMaxDevices];  // a caller holds that device's drop-in GPU leg
std::atomic<int> g_offload_wait{0};             // kvsep_set_offload_wait
kvsep_crc32c_ctx* default_ctx(int* dev_out) {
  static std::once_flag once[kMaxDevices];
  static kvsep_crc32c_ctx* ctx[kMaxDevices] = {};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    (void)hipGetLastError();
    return nullptr;
  }
  if (dev < 0 || dev >= kMaxDevices) return nullptr;
  *dev_out = dev;
  std::call_once(once[dev], [dev] {
    if (kvsep_crc32c_ctx_create(dev, &ctx[dev]) != KVSEP_OK) {
      std::fprintf(stderr, "kvsep_crc32c: GPU offload unavailable on device %d: %s\n", dev, kvsep_last_error());
      ctx[dev] = nullptr;
    }
  });
  return ctx[dev];
}

}  // namespace

// Parallel host copies for the framing writers (payloads into the framed image), on the context's copier
// pool; a serial memcpy when the pool cannot be set up.  Declared in framing.cpp.
int host_copy_parallel(kvsep_crc32c_ctx* c, char* const* dst, const char* const* src, const uint64_t* n,
                       uint64_t count) {
  std::vector<CopySeg> segs;
  segs.reserve(count);
  for (uint64_t i = 0; i < count; ++i)
    if (n[i]) segs.push_back({reinterpret_cast<uint8_t*>(dst[i]), reinterpret_cast<const uint8_t*>(src[i]), n[i]});
  std::lock_guard<std::mutex> g(ctx_mutex(c));
  if (ensure_staging(c) != KVSEP_OK || !ctx_staging(c).pool) {  // no staging: the copies run on this thread
    for (auto& sg : segs) std::memcpy(sg.dst, sg.src, sg.n);
    return KVSEP_OK;
  }
  copy_pool_run(ctx_staging(c).pool, segs.data(), segs.size());
  return KVSEP_OK;
}

// The pointer-per-block host form (kvsep_crc32c_batch_host), optionally with a tee: tee[i] != nullptr also receives
// record i's bytes, copied by the same gather that stages them for the GPU (one read of the source, two writes),
// so a framing writer needs no second pass over its payloads (kvsep_log_frame_host).
int batch_host_tee(kvsep_crc32c_ctx* c, const uint32_t* init, const char* const* ptr, const uint64_t* len,
                   uint32_t* out, uint64_t count, char* const* tee) {
  if (!c || (count && (!ptr || !len || !out))) {
    set_last_error("null argument");
    return KVSEP_EINVAL;
  }
  std::lock_guard<std::mutex> g(ctx_mutex(c));
  int rc = ensure_staging(c);
  if (rc) return rc;
  DeviceGuard dg(ctx_device(c));
  if (dg.err != hipSuccess) return hip_fail("hipSetDevice", dg.err);
  HostStaging& s = ctx_staging(c);
  SlotJob jobs[HostStaging::kSlots];
  int slot = 0;
  uint64_t i = 0;
  while (i < count) {
    if (len[i] > s.bytes) {
      uint32_t r = 0;
      rc = big_block(c, s, jobs, out, reinterpret_cast<const uint8_t*>(ptr[i]), len[i], init ? init[i] : 0u,
                     is_pinned(ptr[i]), &r);
      if (rc) return rc;
      out[i] = r;
      if (tee && tee[i]) {  // a record over the slot size is staged in pieces: its tee copy is one pass of its own
        const CopySeg cs{reinterpret_cast<uint8_t*>(tee[i]), reinterpret_cast<const uint8_t*>(ptr[i]), len[i]};
        copy_pool_run(s.pool, &cs, 1);
      }
      ++i;
      continue;
    }
    rc = retire(s, slot, jobs[slot], out);
    if (rc) return rc;
    uint64_t used = 0, j = i, max_len = 0;
    // gather: blocks packed back to back, each at a 16-B aligned staging offset (copied by the pool below)
    std::vector<CopySeg> segs;
    while (j < count && j - i < s.max_blocks && len[j] <= s.bytes) {
      const uint64_t at = (used + 15) & ~uint64_t(15);
      if (at + len[j] > s.bytes) break;
      if (len[j])
        segs.push_back({s.h_data[slot] + at, reinterpret_cast<const uint8_t*>(ptr[j]), len[j],
                        tee ? reinterpret_cast<uint8_t*>(tee[j]) : nullptr});
      s.h_desc[slot][j - i] = at;
      s.h_desc[slot][s.max_blocks + (j - i)] = len[j];
      if (init) s.h_init[slot][j - i] = init[j];
      max_len = std::max(max_len, len[j]);
      used = at + len[j];
      ++j;
    }
    copy_pool_run(s.pool, segs.data(), segs.size());
    rc = submit(c, s, slot, j - i, used, max_len, nullptr, init != nullptr);
    if (rc) return rc;
    jobs[slot].busy = true;
    jobs[slot].first = i;
    jobs[slot].n = j - i;
    slot ^= 1;
    i = j;
  }
  for (int k = 0; k < HostStaging::kSlots; ++k) {
    rc = retire(s, k, jobs[k], out);
    if (rc) return rc;
  }
  return KVSEP_OK;
}

}  // namespace kvsep

using namespace kvsep;

extern "C" {

uint32_t kvsep_crc32c_extend_host(uint32_t init_crc, const char* data, size_t n) {
  return host_crc(init_crc, reinterpret_cast<const uint8_t*>(data), n);
}

uint32_t kvsep_crc32c_extend(uint32_t init_crc, const char* data, size_t n) {
  if (n >= g_offload_threshold.load(std::memory_order_relaxed)) {
    int dev = 0;
    kvsep_crc32c_ctx* c = default_ctx(&dev);
    if (c) {
      // busy GPU leg and no waiting: this caller takes the host leg now (exact either way) instead of queueing
      // behind the staged copy of another caller on the same PCIe link
      const bool wait = g_offload_wait.load(std::memory_order_relaxed) != 0;
      bool idle = false;
      if (!wait && !g_dropin_busy[dev].compare_exchange_strong(idle, true, std::memory_order_acquire)) {
        g_host_calls.fetch_add(1, std::memory_order_relaxed);
        return host_crc(init_crc, reinterpret_cast<const uint8_t*>(data), n);
      }
      const uint64_t off = 0, len = n;
      uint32_t out = 0;
      const int rc = kvsep_crc32c_batch_host_span(c, data, n, &off, &len, &init_crc, &out, 1);
      if (!wait) g_dropin_busy[dev].store(false, std::memory_order_release);
      if (rc == KVSEP_OK) {
        g_gpu_calls.fetch_add(1, std::memory_order_relaxed);
        return out;
      }
      std::fprintf(stderr, "kvsep_crc32c: GPU offload failed: %s\n", kvsep_last_error());
    }
    // Extend is total (util/crc32c.h:17 has no error channel): a strict deployment aborts instead.
    if (std::getenv("KVSEP_STRICT_GPU")) std::abort();
    g_gpu_failures.fetch_add(1, std::memory_order_relaxed);
  }
  // below the threshold: no counter -- a shared atomic on every small call would be a cache line that every
  // writer, compaction, GC and reader thread bounces (the 4 KiB host leg takes ~60 ns)
  return host_crc(init_crc, reinterpret_cast<const uint8_t*>(data), n);
}

uint32_t kvsep_crc32c_value(const char* data, size_t n) { return kvsep_crc32c_extend(0, data, n); }

uint32_t kvsep_crc32c_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + 0xa282ead8u; }

uint32_t kvsep_crc32c_unmask(uint32_t masked_crc) {
  const uint32_t rot = masked_crc - 0xa282ead8u;
  return (rot >> 17) | (rot << 15);
}

uint32_t kvsep_accelerated_crc32c(uint32_t crc, const char* buf, size_t size) {
  return kvsep_crc32c_extend(crc, buf, size);
}

void kvsep_set_offload_threshold(uint64_t nbytes) { g_offload_threshold.store(nbytes); }

void kvsep_set_offload_wait(int wait) { g_offload_wait.store(wait != 0 ? 1 : 0); }

void kvsep_offload_stats(uint64_t* gpu_calls, uint64_t* host_calls, uint64_t* gpu_failures) {
  if (gpu_calls) *gpu_calls = g_gpu_calls.load();
  if (host_calls) *host_calls = g_host_calls.load();
  if (gpu_failures) *gpu_failures = g_gpu_failures.load();
}

int kvsep_crc32c_batch_host_span(kvsep_crc32c_ctx* c, const char* host_base, uint64_t span_bytes,
                                 const uint64_t* off, const uint64_t* len, const uint32_t* init, uint32_t* out,
                                 uint64_t count) {
  if (!c || (!host_base && span_bytes) || (count && (!off || !len || !out))) {
    set_last_error("null argument");
    return KVSEP_EINVAL;
  }
  for (uint64_t i = 0; i < count; ++i)
    if (off[i] > span_bytes || len[i] > span_bytes - off[i]) {
      set_last_error("block outside span");
      return KVSEP_EINVAL;
    }
  std::lock_guard<std::mutex> g(ctx_mutex(c));
  int rc = ensure_staging(c);
  if (rc) return rc;
  DeviceGuard dg(ctx_device(c));
  if (dg.err != hipSuccess) return hip_fail("hipSetDevice", dg.err);
  HostStaging& s = ctx_staging(c);
  const uint8_t* base = reinterpret_cast<const uint8_t*>(host_base);
  const bool pinned = span_bytes && is_pinned(host_base);
  SlotJob jobs[HostStaging::kSlots];
  int slot = 0;
  uint64_t i = 0;
  while (i < count) {
    if (len[i] > s.bytes) {  // long block: chained segments
      uint32_t r = 0;
      rc = big_block(c, s, jobs, out, base + off[i], len[i], init ? init[i] : 0u, pinned, &r);
      if (rc) return rc;
      out[i] = r;
      ++i;
      continue;
    }
    // group consecutive blocks whose covering range fits one slot
    uint64_t lo = off[i], hi = off[i] + len[i], j = i + 1, max_len = len[i];
    while (j < count && j - i < s.max_blocks && len[j] <= s.bytes) {
      const uint64_t nlo = std::min(lo, off[j]), nhi = std::max(hi, off[j] + len[j]);
      if (nhi - nlo > s.bytes) break;
      lo = nlo; hi = nhi; max_len = std::max(max_len, len[j]);
      ++j;
    }
    rc = retire(s, slot, jobs[slot], out);
    if (rc) return rc;
    const uint64_t nblk = j - i;
    for (uint64_t k = 0; k < nblk; ++k) {
      s.h_desc[slot][k] = off[i + k] - lo;
      s.h_desc[slot][s.max_blocks + k] = len[i + k];
      if (init) s.h_init[slot][k] = init[i + k];
    }
    if (!pinned) {
      const CopySeg cs{s.h_data[slot], base + lo, hi - lo};
      copy_pool_run(s.pool, &cs, 1);
    }
    rc = submit(c, s, slot, nblk, hi - lo, max_len, pinned ? base + lo : nullptr, init != nullptr);
    if (rc) return rc;
    jobs[slot].busy = true;
    jobs[slot].first = i;
    jobs[slot].n = nblk;
    slot ^= 1;
    i = j;
  }
  for (int k = 0; k < HostStaging::kSlots; ++k) {
    rc = retire(s, k, jobs[k], out);
    if (rc) return rc;
  }
  return KVSEP_OK;
}

int kvsep_crc32c_ctx_host_placement(kvsep_crc32c_ctx* c, int* device_node, int* staging_node, int* cpus, int cap) {
  if (!c) {
    set_last_error("null ctx");
    return KVSEP_EINVAL;
  }
  std::lock_guard<std::mutex> g(ctx_mutex(c));
  const HostStaging& s = ctx_staging(c);
  if (device_node) *device_node = ctx_host_node(c);
  if (staging_node) *staging_node = s.ready ? numa::page_node(s.h_data[0]) : -1;
  for (int i = 0; cpus && i < cap && i < int(s.cpus.size()); ++i) cpus[i] = s.cpus[i];
  return int(s.cpus.size());
}

int kvsep_crc32c_batch_host(kvsep_crc32c_ctx* c, const uint32_t* init, const char* const* ptr, const uint64_t* len,
                            uint32_t* out, uint64_t count) {
  return kvsep::batch_host_tee(c, init, ptr, len, out, count, nullptr);
}

void* kvsep_host_alloc_pinned(uint64_t bytes) {
  void* p = nullptr;
  if (hipHostMalloc(&p, bytes ? bytes : 1, hipHostMallocDefault) != hipSuccess) {
    (void)hipGetLastError();
    set_last_error("hipHostMalloc failed");
    return nullptr;
  }
  return p;
}

void kvsep_host_free_pinned(void* p) {
  if (p) (void)hipHostFree(p);
}

int kvsep_abi_version(void) { return KVSEP_ABI_VERSION; }

const char* kvsep_build_info(void) {
  return "kvsep_crc32c: gfx950 HIP kernels (LDS-replicated Z_1024 stride chains, v_perm addressing), "
         "host legs: VPCLMULQDQ fold / SSE4.2 crc32 / portable slicing-by-8, ABI 4";
}

const char* kvsep_crc32c_host_path(void) { return host_leg_name(host_leg()); }

}  // extern "C"
