// host_leg_bench.cc -- the library's host leg (kvsep_crc32c_extend_host, the drop-in's path below the offload
// threshold) timed per block size, one thread: "hot" checksums one block over and over (in cache, as db_bench's
// crc32c benchmark does), "cold" walks a 1 GiB buffer block by block (DRAM-resident, as a vlog scan would).  Run it
// twice, with and without KVSEP_HOST_CRC=sse42, for the VPCLMULQDQ fold against the SSE4.2 crc32q loop.
// Prints one JSON line per (mode, size).  Build: make -C kv-separate_amd tools.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "kvsep_crc32c.h"

static double now() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

int main(int argc, char** argv) {
  const uint64_t cold_bytes = (argc > 1 ? strtoull(argv[1], nullptr, 10) : 1024) << 20;
  std::vector<uint8_t> buf(cold_bytes + 64);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (auto& b : buf) {
    x ^= x << 13, x ^= x >> 7, x ^= x << 17;
    b = uint8_t(x);
  }
  const char* mode = getenv("KVSEP_HOST_CRC") ? getenv("KVSEP_HOST_CRC") : "default";
  const uint64_t sizes[] = {64, 256, 1024, 4096, 16384, 65536, 1 << 20, 16 << 20};
  uint32_t sink = 0;
  for (uint64_t n : sizes) {
    // hot: the same block, ~0.25 s
    const char* p = reinterpret_cast<const char*>(buf.data());
    uint64_t reps = 0, done = 0;
    double t0 = now(), t = t0;
    while (t - t0 < 0.25) {
      for (int k = 0; k < 64; ++k) sink ^= kvsep_crc32c_extend_host(sink, p, n);
      reps += 64;
      t = now();
    }
    const double hot = double(reps * n) / (t - t0) / 1e9;
    // cold: consecutive blocks of the big buffer, one pass
    t0 = now();
    for (done = 0; done + n <= cold_bytes; done += n)
      sink ^= kvsep_crc32c_extend_host(0, reinterpret_cast<const char*>(buf.data()) + done, n);
    const double cold = double(done) / (now() - t0) / 1e9;
    printf("{\"mode\": \"%s\", \"bytes\": %llu, \"hot_GBps\": %.2f, \"cold_GBps\": %.2f}\n", mode,
           (unsigned long long)n, hot, cold);
  }
  fprintf(stderr, "sink %08x\n", sink);
  return 0;
}
