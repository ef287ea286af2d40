// kvsep_internal.h -- declarations shared by the device (.hip) and host (.cpp) halves of
// libkvsep_crc32c.  Not part of the public ABI (include/kvsep_crc32c.h is).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <mutex>

struct kvsep_crc32c_ctx;

namespace kvsep {

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
  bool ready = false;
};

void release_staging(HostStaging& s);

// Implemented in crc32c_device.hip; callers hold ctx_mutex.
int device_batch_locked(kvsep_crc32c_ctx* c, hipStream_t s, const void* base, const uint64_t* off,
                        const uint64_t* len, const uint32_t* init, uint32_t* out, uint64_t count,
                        uint64_t total_bytes, uint64_t max_len);
HostStaging& ctx_staging(kvsep_crc32c_ctx* c);
std::mutex& ctx_mutex(kvsep_crc32c_ctx* c);
int ctx_device(kvsep_crc32c_ctx* c);
uint64_t ctx_piece_bytes(kvsep_crc32c_ctx* c);
void set_last_error(const char* msg);

}  // namespace kvsep
