// fold_variants_probe.cc -- A/B of the host leg's VPCLMULQDQ fold: 4 accumulators (256 B rounds, shipped in
// crc32c_host.cpp fold_bulk) against 8 (512 B rounds), hot, one thread; both checked equal.  Standalone: constants are
// recomputed from the polynomial as gf2.h does.  g++ -O3 -mavx512f -mvpclmulqdq -mpclmul -msse4.2
#include <immintrin.h>
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <vector>
static uint32_t mulmod(uint32_t a, uint32_t b) { uint32_t p = 0; for (int i = 31; i >= 0; --i) { if ((a >> i) & 1u) p ^= b; b = (b >> 1) ^ (0x82F63B78u & (0u - (b & 1u))); } return p; }
static uint32_t xpow(uint64_t e) { uint32_t sq[64]; sq[0] = 0x40000000u; for (int k = 1; k < 64; ++k) sq[k] = mulmod(sq[k-1], sq[k-1]); uint32_t r = 0x80000000u; for (int k = 0; e; ++k, e >>= 1) if (e & 1) r = mulmod(r, sq[k]); return r; }
static void K(uint64_t* k, uint64_t d) { k[0] = uint64_t(xpow(8*d+63)) << 32; k[1] = uint64_t(xpow(8*d-1)) << 32; }
static inline __m512i fold(__m512i x, __m512i k, __m512i d) { return _mm512_ternarylogic_epi64(_mm512_clmulepi64_epi128(x, k, 0), _mm512_clmulepi64_epi128(x, k, 0x11), d, 0x96); }
static inline __m128i f128(__m128i x, const uint64_t* k) { __m128i kk = _mm_loadu_si128((const __m128i*)k); return _mm_xor_si128(_mm_clmulepi64_si128(x, kk, 0), _mm_clmulepi64_si128(x, kk, 0x11)); }
uint64_t k512[2], k256[2], k64[2], k48[2], k32[2], k16[2];
static uint32_t tail(uint64_t l, const uint8_t* p, size_t n) { while (n >= 8) { uint64_t w; memcpy(&w, p, 8); l = _mm_crc32_u64(l, w); p += 8; n -= 8; } while (n) { l = _mm_crc32_u8(uint32_t(l), *p++); --n; } return ~uint32_t(l); }
static uint32_t reduce4(__m512i x0, __m512i x1, __m512i x2, __m512i x3) {
  __m512i kk = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i*)k64));
  x1 = fold(x0, kk, x1); x2 = fold(x1, kk, x2); x3 = fold(x2, kk, x3);
  __m128i r = _mm512_extracti32x4_epi32(x3, 3);
  r = _mm_xor_si128(r, f128(_mm512_extracti32x4_epi32(x3, 0), k48));
  r = _mm_xor_si128(r, f128(_mm512_extracti32x4_epi32(x3, 1), k32));
  r = _mm_xor_si128(r, f128(_mm512_extracti32x4_epi32(x3, 2), k16));
  uint64_t c = _mm_crc32_u64(0, uint64_t(_mm_cvtsi128_si64(r))); return uint32_t(_mm_crc32_u64(c, uint64_t(_mm_extract_epi64(r, 1))));
}
uint32_t crc4(uint32_t init, const uint8_t* p, size_t n) {
  uint64_t l = ~init;
  if (n >= 256) {
    __m512i k = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i*)k256));
    __m512i x0 = _mm512_loadu_si512(p), x1 = _mm512_loadu_si512(p+64), x2 = _mm512_loadu_si512(p+128), x3 = _mm512_loadu_si512(p+192);
    x0 = _mm512_xor_si512(x0, _mm512_zextsi128_si512(_mm_cvtsi32_si128(int(l)))); p += 256; n -= 256;
    while (n >= 256) { x0 = fold(x0, k, _mm512_loadu_si512(p)); x1 = fold(x1, k, _mm512_loadu_si512(p+64)); x2 = fold(x2, k, _mm512_loadu_si512(p+128)); x3 = fold(x3, k, _mm512_loadu_si512(p+192)); p += 256; n -= 256; }
    l = reduce4(x0, x1, x2, x3);
  }
  return tail(l, p, n);
}
uint32_t crc8(uint32_t init, const uint8_t* p, size_t n) {
  uint64_t l = ~init;
  if (n >= 512) {
    __m512i k = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i*)k512));
    __m512i x[8]; for (int i = 0; i < 8; ++i) x[i] = _mm512_loadu_si512(p + 64*i);
    x[0] = _mm512_xor_si512(x[0], _mm512_zextsi128_si512(_mm_cvtsi32_si128(int(l)))); p += 512; n -= 512;
    while (n >= 512) { for (int i = 0; i < 8; ++i) x[i] = fold(x[i], k, _mm512_loadu_si512(p + 64*i)); p += 512; n -= 512; }
    __m512i k2 = _mm512_broadcast_i32x4(_mm_loadu_si128((const __m128i*)k256));
    for (int i = 0; i < 4; ++i) x[i+4] = fold(x[i], k2, x[i+4]);
    l = reduce4(x[4], x[5], x[6], x[7]);
    // remaining >= 256 handled by crc4-style? keep simple: fall to tail
  }
  return tail(l, p, n);
}
static double now() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }
int main() {
  K(k512, 512); K(k256, 256); K(k64, 64); K(k48, 48); K(k32, 32); K(k16, 16);
  std::vector<uint8_t> b(1 << 20); uint64_t s = 1; for (auto& c : b) { s = s * 6364136223846793005ull + 1; c = uint8_t(s >> 56); }
  for (size_t n : {4096ul, 16384ul, 65536ul, 1ul << 20}) {
    if (crc4(7, b.data(), n) != crc8(7, b.data(), n)) { printf("MISMATCH %zu\n", n); return 1; }
    for (int v = 0; v < 2; ++v) {
      uint32_t sink = 0; uint64_t reps = 0; double t0 = now(), t = t0;
      while (t - t0 < 0.3) { for (int i = 0; i < 32; ++i) sink ^= (v ? crc8 : crc4)(sink, b.data(), n); reps += 32; t = now(); }
      printf("{\"variant\": %d, \"bytes\": %zu, \"GBps\": %.1f, \"sink\": %u}\n", v ? 8 : 4, n, reps * n / (t - t0) / 1e9, sink);
    }
  }
}
