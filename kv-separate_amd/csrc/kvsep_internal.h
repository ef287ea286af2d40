// kvsep_internal.h -- declarations shared by the device (.hip) and host (.cpp) halves of
// libkvsep_crc32c.  Not part of the public ABI (include/kvsep_crc32c.h is).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>
#include <vector>

#include "copy_pool.h"

struct kvsep_crc32c_ctx;

namespace kvsep {

// Device scratch of one in-flight batch: the piece plan (planned mode), the work counter, the verify
// defaults and the SST-verify arrays.  A scratch object is reused call after call; `last_use` orders a
// call on a different stream behind the previous user, so reuse across streams is race-free.  The host
// pipeline gives each staging slot its own Scratch so the two slots' batches overlap, and every graph capture takes a
// capture set's Scratch of its own (crc32c_device.hip, capture_scratch).
struct Scratch {
  uint64_t cap_count = 0, cap_pieces = 0;
  uint64_t* d_counts = nullptr;
  uint64_t* d_pstart = nullptr;
  uint32_t* d_pblk = nullptr;
  uint32_t* d_partial = nullptr;
  void* d_scan_tmp = nullptr;
  size_t scan_tmp_bytes = 0;
  uint32_t* d_counter = nullptr;
  unsigned long long* d_verify = nullptr;  // [first_bad, nbad] when the caller passes none, then the accumulator set
  bool vacc_dirty = false;                  // a failed eager call may have posted to the set: reset before its next use
  unsigned long long* d_vslot = nullptr;    // captured verify calls: one verdict slot (2 words) per publishing workgroup
  uint32_t cap_vslot = 0;
  uint64_t* d_sst_len1 = nullptr;           // SST verify: len + 1 ...
  uint32_t* d_sst_stored = nullptr;         // ... and the stored trailer words
  uint64_t cap_sst = 0;
  hipEvent_t last_use = nullptr;
  hipStream_t last_stream = nullptr;
  bool used = false;
};
void free_scratch(Scratch& sc);

// The persistent host copiers of the staging pipeline (copy_pool.h), bound to `cpus` when it is not empty.
CopyPool* copy_pool_create(const std::vector<int>& cpus);
void copy_pool_destroy(CopyPool* p);
void copy_pool_run(CopyPool* p, const CopySeg* segs, uint64_t nseg);  // returns when every byte is copied

// Double-buffered host<->device staging for the host-memory entry points.
struct HostStaging {
  static constexpr int kSlots = 2;
  uint64_t bytes = 0;        // payload bytes per slot
  uint64_t max_blocks = 0;   // descriptors per slot
  uint8_t* h_data[kSlots] = {nullptr, nullptr};   // pinned
  uint8_t* d_data[kSlots] = {nullptr, nullptr};
  uint64_t* h_desc[kSlots] = {nullptr, nullptr};  // pinned: off[max_blocks] | len[max_blocks]
  uint32_t* h_init[kSlots] = {nullptr, nullptr};  // pinned
  uint32_t* h_out[kSlots] = {nullptr, nullptr};   // pinned
  uint64_t* d_desc[kSlots] = {nullptr, nullptr};
  uint32_t* d_init[kSlots] = {nullptr, nullptr};
  uint32_t* d_out[kSlots] = {nullptr, nullptr};
  hipStream_t stream[kSlots] = {nullptr, nullptr};
  hipEvent_t done[kSlots] = {nullptr, nullptr};
  Scratch scratch[kSlots];
  CopyPool* pool = nullptr;
  std::vector<int> cpus;     // the CPUs the copiers (and the staging allocation) were bound to: the device's NUMA node
  bool ready = false;
  // allocation failed: retried only after a backoff (ensure_staging), so a transient failure is not permanent and
  // a persistent one does not cost an allocation attempt per call
  int64_t retry_at_ns = 0;
  uint32_t failures = 0;
};

void release_staging(HostStaging& s);

// Makes `dev` the calling thread's current HIP device for the scope and restores the caller's device on every
// exit path: the library never leaves a thread on another GPU than the one it came in with.
struct DeviceGuard {
  int prev = -1;
  hipError_t err = hipSuccess;
  explicit DeviceGuard(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) {
      (void)hipGetLastError();
      prev = -1;
    }
    if (prev != dev) err = hipSetDevice(dev);
  }
  ~DeviceGuard() {
    int now = -1;
    if (prev >= 0 && hipGetDevice(&now) == hipSuccess && now != prev) (void)hipSetDevice(prev);
  }
  DeviceGuard(const DeviceGuard&) = delete;
  DeviceGuard& operator=(const DeviceGuard&) = delete;
};

// Implemented in crc32c_device.hip; callers hold ctx_mutex.
int device_batch_locked(kvsep_crc32c_ctx* c, Scratch& sc, hipStream_t s, const void* base, const uint64_t* off,
                        const uint64_t* len, const uint32_t* init, uint32_t* out, uint64_t count,
                        uint64_t total_bytes, uint64_t max_len);
// kvsep_crc32c_batch_host with an optional tee: tee[i] (when tee and tee[i] are non-null) also receives record i's bytes
// from the gather that stages them (crc32c_host.cpp).  Takes the context's mutex.
int batch_host_tee(kvsep_crc32c_ctx* c, const uint32_t* init, const char* const* ptr, const uint64_t* len,
                   uint32_t* out, uint64_t count, char* const* tee);
HostStaging& ctx_staging(kvsep_crc32c_ctx* c);
std::mutex& ctx_mutex(kvsep_crc32c_ctx* c);
int ctx_device(kvsep_crc32c_ctx* c);
int ctx_host_node(kvsep_crc32c_ctx* c);  // NUMA node of the device (-1: unknown or binding off)
uint64_t ctx_piece_bytes(kvsep_crc32c_ctx* c);
void set_last_error(const char* msg);

}  // namespace kvsep
