// Host-sanitizer fuzz of the framing walkers (kv-separate_amd/csrc/framing.cpp), which parse untrusted
// file bytes.  Built by tests/test_sanitize_host.py with g++ -fsanitize=address,undefined against a
// stub batch backend (bitwise CRC-32C below), so no GPU or HIP runtime is involved.
#include <cstdint>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <random>
#include <vector>

#include "kvsep_crc32c.h"

static uint32_t bit_crc(uint32_t init, const uint8_t* p, uint64_t n) {
  uint32_t l = ~init;
  for (uint64_t i = 0; i < n; ++i) {
    l ^= p[i];
    for (int k = 0; k < 8; ++k) l = (l >> 1) ^ (0x82F63B78u & (0u - (l & 1u)));
  }
  return ~l;
}

extern "C" {
uint32_t kvsep_crc32c_mask(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }
uint32_t kvsep_crc32c_unmask(uint32_t m) {
  const uint32_t r = m - 0xa282ead8u;
  return (r >> 17) | (r << 15);
}
int kvsep_crc32c_batch_host_span(kvsep_crc32c_ctx*, const char* base, uint64_t span, const uint64_t* off,
                                 const uint64_t* len, const uint32_t* init, uint32_t* out, uint64_t count) {
  for (uint64_t i = 0; i < count; ++i) {
    if (off[i] > span || len[i] > span - off[i]) return KVSEP_EINVAL;
    out[i] = bit_crc(init ? init[i] : 0, reinterpret_cast<const uint8_t*>(base) + off[i], len[i]);
  }
  return KVSEP_OK;
}
uint32_t kvsep_crc32c_extend_host(uint32_t init, const char* data, size_t n) {
  return bit_crc(init, reinterpret_cast<const uint8_t*>(data), n);
}
int kvsep_crc32c_batch_host(kvsep_crc32c_ctx*, const uint32_t* init, const char* const* ptr, const uint64_t* len,
                            uint32_t* out, uint64_t count) {
  for (uint64_t i = 0; i < count; ++i)
    out[i] = bit_crc(init ? init[i] : 0, reinterpret_cast<const uint8_t*>(ptr[i]), len[i]);
  return KVSEP_OK;
}
}
namespace kvsep {
int host_copy_parallel(kvsep_crc32c_ctx*, char* const* dst, const char* const* src, const uint64_t* n,
                       uint64_t count) {
  for (uint64_t i = 0; i < count; ++i)
    if (n[i]) std::memcpy(dst[i], src[i], n[i]);
  return KVSEP_OK;
}
int batch_host_tee(kvsep_crc32c_ctx* c, const uint32_t* init, const char* const* ptr, const uint64_t* len,
                   uint32_t* out, uint64_t count, char* const* tee) {
  for (uint64_t i = 0; i < count; ++i)
    if (tee && tee[i] && len[i]) std::memcpy(tee[i], ptr[i], len[i]);
  return kvsep_crc32c_batch_host(c, init, ptr, len, out, count);
}
void set_last_error(const char*) {}
}  // namespace kvsep

int main() {
  std::mt19937_64 rng(7);
  auto* ctx = reinterpret_cast<kvsep_crc32c_ctx*>(0x1);  // the stubs never dereference it
  int failures = 0;
  for (int iter = 0; iter < 3000; ++iter) {
    // a valid vlog image from random payloads, then damaged and truncated at random
    std::vector<std::vector<char>> pl(rng() % 12);
    std::vector<const char*> ptr;
    std::vector<uint64_t> len;
    for (auto& p : pl) {
      p.resize(rng() % 300);
      for (auto& c : p) c = char(rng());
      ptr.push_back(p.data());
      len.push_back(p.size());
    }
    uint64_t need = 0;
    kvsep_vlog_frame_host(ctx, ptr.data(), len.data(), pl.size(), nullptr, 0, &need);
    std::vector<char> img(need);
    uint64_t w = 0;
    if (kvsep_vlog_frame_host(ctx, ptr.data(), len.data(), pl.size(), img.data(), img.size(), &w) != 0 || w != need)
      ++failures;
    uint64_t n = 0, good = 0, gb = 0;
    kvsep_vlog_verify_host(ctx, img.data(), img.size(), &n, &good, &gb, nullptr);
    if (n != pl.size() || good != n || gb != img.size()) ++failures;
    if (!img.empty()) {
      img[rng() % img.size()] ^= char(1 + rng() % 255);
      img.resize(rng() % (img.size() + 1));
    }
    std::vector<char> heap(img.begin(), img.end());  // exact-size heap buffer: ASan sees any over-read
    kvsep_vlog_verify_host(ctx, heap.data(), heap.size(), &n, &good, &gb, nullptr);
    if (good > n || gb > heap.size()) ++failures;
    // random bytes through the log/MANIFEST walker (32 KiB block framing)
    std::vector<char> junk(rng() % 70000);
    for (auto& c : junk) c = char(rng() % 4 == 0 ? 0 : rng());
    const uint64_t cnt = kvsep_log_walk(junk.data(), junk.size(), nullptr, nullptr, nullptr, nullptr, 0);
    std::vector<uint64_t> off(cnt), ln(cnt);
    std::vector<uint32_t> st(cnt);
    std::vector<uint8_t> ty(cnt), ok(cnt + 1);
    kvsep_log_walk(junk.data(), junk.size(), off.data(), ln.data(), st.data(), ty.data(), cnt);
    for (uint64_t i = 0; i < cnt; ++i)
      if (off[i] + ln[i] > junk.size()) ++failures;
    uint64_t nr = 0;
    kvsep_log_verify_host(ctx, junk.data(), junk.size(), ok.data(), ok.size(), &nr);
    if (nr != cnt) ++failures;
    std::vector<uint8_t> acc(cnt + 1);
    if (cnt && kvsep_log_accept(off.data(), ok.data(), cnt, junk.size(), acc.data()) > junk.size()) ++failures;
    // log/MANIFEST writer: random records appended at a random block offset, walked and verified back
    std::vector<std::vector<char>> recs(rng() % 6);
    std::vector<const char*> rp;
    std::vector<uint64_t> rl;
    for (auto& r : recs) {
      r.resize(rng() % 3 == 0 ? rng() % 80000 : rng() % 40);
      for (auto& c : r) c = char(rng());
      rp.push_back(r.data());
      rl.push_back(r.size());
    }
    const uint64_t dest = rng() % 32768;
    uint64_t lw = 0;
    kvsep_log_frame_host(ctx, rp.data(), rl.data(), recs.size(), dest, nullptr, 0, &lw);
    std::vector<char> logimg(dest + lw);  // zero prefix stands for the log's existing bytes
    if (kvsep_log_frame_host(ctx, rp.data(), rl.data(), recs.size(), dest, logimg.data() + dest, lw, &lw) != 0)
      ++failures;
    // every physical record from the first block boundary at or after dest on is framed by the writer
    const uint64_t b0 = (dest + 32767) / 32768 * 32768;
    std::vector<char> tail(logimg.begin() + long(std::min<uint64_t>(b0, logimg.size())), logimg.end());
    const uint64_t lc = kvsep_log_walk(tail.data(), tail.size(), nullptr, nullptr, nullptr, nullptr, 0);
    std::vector<uint8_t> lok(lc + 1);
    kvsep_log_verify_host(ctx, tail.data(), tail.size(), lok.data(), lok.size(), &nr);
    for (uint64_t i = 0; i < nr; ++i)
      if (!lok[i]) ++failures;
  }
  std::printf("%s (%d failures)\n", failures ? "FAIL" : "PASS", failures);
  return failures ? 1 : 0;
}
