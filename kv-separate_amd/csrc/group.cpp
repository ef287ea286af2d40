// group.cpp -- one process driving several GPUs: a batch of independent blocks is cut into
// contiguous block ranges balanced by bytes (a prefix sum of len), each range runs on its own device's context
// from its own host thread, and the u32 results land in ONE output array.  Payload bytes never cross between
// GPUs: host-resident data goes H2D over each GPU's own PCIe link, device-resident shards are read from their
// own HBM.  The verify forms reduce first_bad (min) and nbad (sum) over the shards.
//
// The consumer this is for is a single KVDB process scanning whole vlog files -- GC, db/db_impl.cc:880-951,
// over VlogReader::ReadPhysicalRecord (db/value_log_reader.cc:86-138) -- and recovery (db/db_impl.cc:485-571).
// Multi-process deployments (one rank per GPU) use kvsep_crc32c_partition the same way (bench.py).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/kvsep_crc32c.h"
#include "kvsep_internal.h"
#include "numa.h"

struct kvsep_crc32c_group {
  std::vector<int> devices;
  std::vector<kvsep_crc32c_ctx*> ctx;
  std::vector<hipStream_t> stream;  // device-resident form: one stream per member, on its device
  std::vector<uint64_t*> d_res;      // verify form: [first_bad, nbad] of each member's shard, on its device
  std::mutex mu;                     // device-resident calls share the streams and d_res: one at a time
  // each member's host node and its CPU list, read from sysfs once per node (not on every call)
  std::mutex node_mu;
  std::vector<int> node;
  std::vector<std::vector<int>> node_cpus;
};

namespace {

// Member i's host node and CPU list (cached; refreshed if the member's context was moved to another node).
const std::vector<int>* member_cpus(kvsep_crc32c_group* g, int i, int* node) {
  *node = kvsep::ctx_host_node(g->ctx[i]);
  std::lock_guard<std::mutex> lk(g->node_mu);
  if (g->node[i] != *node) {
    g->node[i] = *node;
    g->node_cpus[i] = kvsep::numa::node_cpus(*node);
  }
  return &g->node_cpus[i];
}

// Runs fn(i) for every member i on its own host thread (member 0 on the caller's); first error wins.  bind: the host
// forms, which fill pinned staging and drive the member's PCIe link -- each thread is bound for the call to the NUMA
// node of its member's device (round 5; the caller's own affinity and memory policy come back when member 0 is done).
// The device-resident forms touch no host memory of their own and run unbound.
template <typename Fn>
int fan_out(kvsep_crc32c_group* g, bool bind, Fn&& fn) {
  const int n = int(g->ctx.size());
  std::vector<int> rc(n, KVSEP_OK);
  std::vector<std::string> err(n);
  std::vector<std::thread> th;
  auto member = [&](int i) {
    int node = -1;
    const std::vector<int>* cpus = bind ? member_cpus(g, i, &node) : nullptr;
    kvsep::numa::ScopedBind sb(bind ? node : -1, cpus);
    rc[i] = fn(i);
    if (rc[i]) err[i] = kvsep_last_error();  // the error text is thread-local
  };
  for (int i = 1; i < n; ++i) th.emplace_back(member, i);
  member(0);
  for (auto& t : th) t.join();
  for (int i = 0; i < n; ++i)
    if (rc[i]) {
      kvsep::set_last_error(("group member " + std::to_string(i) + ": " + err[i]).c_str());
      return rc[i];
    }
  return KVSEP_OK;
}

}  // namespace

extern "C" {

int kvsep_crc32c_partition(const uint64_t* len, uint64_t count, int parts, uint64_t* bounds) {
  if (parts < 1 || !bounds || (count && !len)) {
    kvsep::set_last_error("partition: bad argument");
    return KVSEP_EINVAL;
  }
  unsigned __int128 total = 0;
  for (uint64_t i = 0; i < count; ++i) total += len[i];
  // bounds[p] = the block index whose prefix sum is closest to p/parts of the bytes; monotone by construction
  bounds[0] = 0;
  uint64_t b = 0;
  unsigned __int128 acc = 0;
  for (int p = 1; p < parts; ++p) {
    const unsigned __int128 target = total * unsigned(p) / unsigned(parts);
    while (b < count && acc + len[b] <= target) acc += len[b++];
    // one more block if that lands nearer the target (and keeps at least the ordering)
    if (b < count && (acc + len[b] - target) < (target - acc)) acc += len[b++];
    bounds[p] = b;
  }
  bounds[parts] = count;
  return KVSEP_OK;
}

int kvsep_crc32c_group_create(const int* devices, int ndev, kvsep_crc32c_group** out) {
  if (!devices || ndev < 1 || !out) {
    kvsep::set_last_error("group_create: bad argument");
    return KVSEP_EINVAL;
  }
  *out = nullptr;
  auto* g = new kvsep_crc32c_group();
  for (int i = 0; i < ndev; ++i) {
    kvsep_crc32c_ctx* c = nullptr;
    int rc = kvsep_crc32c_ctx_create(devices[i], &c);
    hipStream_t s = nullptr;
    uint64_t* res = nullptr;
    if (rc == KVSEP_OK) {
      kvsep::DeviceGuard dg(devices[i]);
      if (dg.err != hipSuccess || hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) {
        kvsep::set_last_error("group_create: stream creation failed");
        rc = KVSEP_EHIP;
      } else if (hipMalloc(&res, 16) != hipSuccess) {  // once here: a hipFree per call would synchronise the device
        kvsep::set_last_error("group_create: hipMalloc failed");
        rc = KVSEP_ENOMEM;
      }
    }
    if (rc != KVSEP_OK) {
      if (s) {
        kvsep::DeviceGuard dg(devices[i]);
        (void)hipStreamDestroy(s);
      }
      if (c) kvsep_crc32c_ctx_destroy(c);
      kvsep_crc32c_group_destroy(g);
      return rc;
    }
    g->devices.push_back(devices[i]);
    g->ctx.push_back(c);
    g->stream.push_back(s);
    g->d_res.push_back(res);
    g->node.push_back(-2);  // not read yet (member_cpus)
    g->node_cpus.emplace_back();
  }
  *out = g;
  return KVSEP_OK;
}

void kvsep_crc32c_group_destroy(kvsep_crc32c_group* g) {
  if (!g) return;
  for (size_t i = 0; i < g->ctx.size(); ++i) {
    if (g->stream[i]) {
      kvsep::DeviceGuard dg(g->devices[i]);
      (void)hipStreamSynchronize(g->stream[i]);
      (void)hipStreamDestroy(g->stream[i]);
      (void)hipFree(g->d_res[i]);
    }
    kvsep_crc32c_ctx_destroy(g->ctx[i]);
  }
  delete g;
}

int kvsep_crc32c_group_size(kvsep_crc32c_group* g) { return g ? int(g->ctx.size()) : 0; }

kvsep_crc32c_ctx* kvsep_crc32c_group_ctx(kvsep_crc32c_group* g, int i) {
  return g && i >= 0 && i < int(g->ctx.size()) ? g->ctx[i] : nullptr;
}

int kvsep_crc32c_group_batch_host_span(kvsep_crc32c_group* g, const char* host_base, uint64_t span_bytes,
                                       const uint64_t* off, const uint64_t* len, const uint32_t* init, uint32_t* out,
                                       uint64_t count) {
  if (!g || (count && (!off || !len || !out))) {
    kvsep::set_last_error("group_batch_host_span: bad argument");
    return KVSEP_EINVAL;
  }
  const int n = int(g->ctx.size());
  std::vector<uint64_t> bounds(n + 1);
  int rc = kvsep_crc32c_partition(len, count, n, bounds.data());
  if (rc) return rc;
  return fan_out(g, true, [&](int i) {
    const uint64_t b0 = bounds[i], b1 = bounds[i + 1];
    if (b0 == b1) return int(KVSEP_OK);
    return kvsep_crc32c_batch_host_span(g->ctx[i], host_base, span_bytes, off + b0, len + b0, init ? init + b0 : nullptr,
                                        out + b0, b1 - b0);
  });
}

int kvsep_crc32c_group_verify_host_span(kvsep_crc32c_group* g, const char* host_base, uint64_t span_bytes,
                                        const uint64_t* off, const uint64_t* len, const uint32_t* init,
                                        const uint32_t* expected_masked, uint32_t* out, uint64_t* first_bad,
                                        uint64_t* nbad, uint64_t count) {
  if (!expected_masked) {
    kvsep::set_last_error("group_verify_host_span: expected_masked is null");
    return KVSEP_EINVAL;
  }
  const int rc = kvsep_crc32c_group_batch_host_span(g, host_base, span_bytes, off, len, init, out, count);
  if (rc) return rc;
  uint64_t fb = UINT64_MAX, nb = 0;
  for (uint64_t i = 0; i < count; ++i)
    if (kvsep_crc32c_mask(out[i]) != expected_masked[i]) {
      fb = std::min(fb, i);
      ++nb;
    }
  if (first_bad) *first_bad = fb;
  if (nbad) *nbad = nb;
  return KVSEP_OK;
}

int kvsep_vlog_verify_host_group(kvsep_crc32c_group* g, const char* buf, uint64_t n, uint64_t* nrecords,
                                 uint64_t* ngood, uint64_t* good_bytes, uint64_t* drop_bytes) {
  if (!g || (!buf && n)) {
    kvsep::set_last_error("vlog_verify_host_group: bad argument");
    return KVSEP_EINVAL;
  }
  const uint64_t cnt = kvsep_vlog_walk(buf, n, nullptr, nullptr, nullptr, 0, nullptr);
  std::vector<uint64_t> off(cnt), len(cnt);
  std::vector<uint32_t> stored(cnt), crc(cnt);
  kvsep_vlog_walk(buf, n, off.data(), len.data(), stored.data(), cnt, nullptr);
  if (cnt) {
    const int rc = kvsep_crc32c_group_batch_host_span(g, buf, n, off.data(), len.data(), nullptr, crc.data(), cnt);
    if (rc) return rc;
  }
  uint64_t good = 0;
  while (good < cnt && kvsep_crc32c_mask(crc[good]) == stored[good]) ++good;  // db/value_log_reader.cc:109-122
  if (nrecords) *nrecords = cnt;
  if (ngood) *ngood = good;
  if (good_bytes) *good_bytes = good ? off[good - 1] + len[good - 1] : 0;
  if (drop_bytes) *drop_bytes = good < cnt ? len[good] : 0;
  return KVSEP_OK;
}

int kvsep_crc32c_group_batch_device(kvsep_crc32c_group* g, const void* const* base, const uint64_t* const* off,
                                    const uint64_t* const* len, const uint32_t* const* init, uint32_t* const* out,
                                    const uint64_t* count, const uint64_t* total_bytes, const uint64_t* max_len) {
  return kvsep_crc32c_group_verify_device(g, base, off, len, init, nullptr, out, nullptr, count, total_bytes, max_len,
                                          nullptr, nullptr);
}

int kvsep_crc32c_group_verify_device(kvsep_crc32c_group* g, const void* const* base, const uint64_t* const* off,
                                     const uint64_t* const* len, const uint32_t* const* init,
                                     const uint32_t* const* expected_masked, uint32_t* const* out,
                                     const uint64_t* index_base, const uint64_t* count, const uint64_t* total_bytes,
                                     const uint64_t* max_len, uint64_t* first_bad, uint64_t* nbad) {
  if (!g || !base || !off || !len || !out || !count || !total_bytes || !max_len ||
      (expected_masked && (!index_base || !first_bad || !nbad))) {
    kvsep::set_last_error("group_batch_device: bad argument");
    return KVSEP_EINVAL;
  }
  std::lock_guard<std::mutex> lk(g->mu);
  const int n = int(g->ctx.size());
  std::vector<uint64_t> fb(n, UINT64_MAX), nb(n, 0);
  const int rc = fan_out(g, false, [&](int i) {
    if (!count[i]) return int(KVSEP_OK);
    kvsep::DeviceGuard dg(g->devices[i]);
    if (dg.err != hipSuccess) {
      kvsep::set_last_error("hipSetDevice failed");
      return int(KVSEP_EHIP);
    }
    int r;
    uint64_t* d_res = expected_masked ? g->d_res[i] : nullptr;  // [first_bad, nbad] of this shard
    if (expected_masked) {
      r = kvsep_crc32c_verify_device(g->ctx[i], g->stream[i], base[i], off[i], len[i], init ? init[i] : nullptr,
                                     expected_masked[i], out[i], d_res, d_res + 1, count[i], total_bytes[i], max_len[i]);
    } else {
      r = kvsep_crc32c_batch_device(g->ctx[i], g->stream[i], base[i], off[i], len[i], init ? init[i] : nullptr, out[i],
                                    count[i], total_bytes[i], max_len[i]);
    }
    if (r == KVSEP_OK && hipStreamSynchronize(g->stream[i]) != hipSuccess) {
      kvsep::set_last_error("hipStreamSynchronize failed");
      r = KVSEP_EHIP;
    }
    if (r == KVSEP_OK && d_res) {
      uint64_t h[2];
      if (hipMemcpyAsync(h, d_res, 16, hipMemcpyDeviceToHost, g->stream[i]) != hipSuccess ||
          hipStreamSynchronize(g->stream[i]) != hipSuccess) {
        kvsep::set_last_error("hipMemcpy failed");
        r = KVSEP_EHIP;
      } else {
        fb[i] = h[0] == UINT64_MAX ? UINT64_MAX : index_base[i] + h[0];
        nb[i] = h[1];
      }
    }
    return r;
  });
  if (rc) return rc;
  if (expected_masked) {
    *first_bad = *std::min_element(fb.begin(), fb.end());
    uint64_t s = 0;
    for (uint64_t v : nb) s += v;
    *nbad = s;
  }
  return KVSEP_OK;
}

}  // extern "C"
