// The staging pipeline's host copiers (kv-separate_amd/csrc/copy_pool.h) on their own, no GPU: many random gathers --
// tiny segments (the 4 KiB SST blocks that are claimed in 256 KiB runs), segments over the 1 MiB chunk size, empty
// ones, a single segment (the caller copies alone), with and without a tee destination -- with several thread counts,
// every destination byte checked, and the pool reused call after call as the pipeline reuses it.  Built under ThreadSanitizer and under AddressSanitizer
// by tests/test_copy_pool_cpu.py.  Prints PASS.
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "copy_pool.h"

int main() {
  std::mt19937_64 rng(12345);
  std::vector<uint8_t> src(24 << 20), dst(24 << 20), tee(24 << 20);
  for (auto& b : src) b = uint8_t(rng());
  for (int threads : {0, 1, 3, 7}) {
    kvsep::CopyPool pool(threads);
    for (int round = 0; round < 40; ++round) {
      std::vector<kvsep::CopySeg> segs;
      std::vector<uint64_t> at, from, len;
      uint64_t used = 0;
      const int kind = round % 4;
      while (true) {
        uint64_t n = kind == 0 ? 4096 : kind == 1 ? rng() % 9000 : kind == 2 ? (rng() % (3u << 20)) : 0;
        if (kind == 3 && !segs.empty()) break;  // one segment: the caller copies alone
        if (kind == 3) n = rng() % (8u << 20);
        if (used + n > dst.size() || segs.size() > 20000) break;
        const uint64_t f = rng() % (src.size() - n + 1);
        // every other round also tees each segment into a second buffer (the framing writers' one-read gather)
        segs.push_back({dst.data() + used, src.data() + f, n, round % 2 ? tee.data() + used : nullptr});
        at.push_back(used);
        from.push_back(f);
        len.push_back(n);
        used += n;
      }
      std::memset(dst.data(), 0xA5, used);
      std::memset(tee.data(), 0x5A, used);
      pool.run(segs.data(), segs.size());
      for (size_t i = 0; i < segs.size(); ++i)
        if (std::memcmp(dst.data() + at[i], src.data() + from[i], len[i]) != 0 ||
            (round % 2 && std::memcmp(tee.data() + at[i], src.data() + from[i], len[i]) != 0)) {
          std::printf("FAILED threads %d round %d segment %zu\n", threads, round, i);
          return 1;
        }
    }
  }
  std::printf("PASS\n");
  return 0;
}
