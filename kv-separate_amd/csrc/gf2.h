// gf2.h -- host-side GF(2) algebra for reflected CRC-32C (Castagnoli, 0x82F63B78).
//
// Everything the kernels look up is one linear map: Z_d, "advance a CRC register over d zero
// bytes".  In the reflected, little-endian convention of util/crc32c.cc the register after
// consuming bytes up to position q is interchangeable with a 32-bit word XORed into bytes
// q..q+3 (that is why util/crc32c.cc:334 seeds stride 0 with `word ^ l`, and STEP4W at
// util/crc32c.cc:307-315 re-injects the stride words with `w ^= l`).  So:
//   * byte step         l' = Z_1(l ^ b)                          (util/crc32c.cc:287-292)
//   * 16-byte stride    c' = word ^ Z_16(c)                      (util/crc32c.cc:295-301)
//   * this engine's 1 KiB-strided lane chains   c' = word ^ Z_1024(c)
//   * lane / piece combine   R(A||B) = Z_|B|(R(A)) ^ R(B)
// A map is stored as 4 byte-tables: Z_d(w) = T0[w&255] ^ T1[(w>>8)&255] ^ T2[(w>>16)&255] ^ T3[w>>24].
#pragma once
#include <cstdint>
#include <cstring>

namespace kvsep {
namespace gf2 {

constexpr uint32_t kPolyReflected = 0x82F63B78u;

struct Mat32 {  // column i = image of basis bit i
  uint32_t col[32];
};

inline uint32_t apply(const Mat32& m, uint32_t v) {
  uint32_t r = 0;
  for (int i = 0; v; ++i, v >>= 1)
    if (v & 1u) r ^= m.col[i];
  return r;
}

inline Mat32 compose(const Mat32& a, const Mat32& b) {  // a after b
  Mat32 r;
  for (int i = 0; i < 32; ++i) r.col[i] = apply(a, b.col[i]);
  return r;
}

inline Mat32 identity() {
  Mat32 r;
  for (int i = 0; i < 32; ++i) r.col[i] = 1u << i;
  return r;
}

// One zero byte: l' = table[l & 255] ^ (l >> 8), table built bit by bit from the polynomial.
inline uint32_t byte_table_entry(uint32_t b) {
  uint32_t r = b;
  for (int k = 0; k < 8; ++k) r = (r >> 1) ^ (kPolyReflected & (0u - (r & 1u)));
  return r;
}

inline Mat32 zero_byte_map() {
  Mat32 m;
  for (int i = 0; i < 32; ++i) {
    uint32_t v = 1u << i;
    m.col[i] = byte_table_entry(v & 0xffu) ^ (v >> 8);
  }
  return m;
}

// Z_d for any d (square-and-multiply over Z_1).
inline Mat32 zero_bytes_map(uint64_t d) {
  Mat32 result = identity();
  Mat32 p = zero_byte_map();
  while (d) {
    if (d & 1u) result = compose(p, result);
    d >>= 1;
    if (d) p = compose(p, p);
  }
  return result;
}

// 4 x 256 byte-tables of a map: out[k*256 + b] = m(b << 8k).
inline void byte_tables(const Mat32& m, uint32_t* out) {
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) out[k * 256 + b] = apply(m, b << (8 * k));
}

// The same maps as polynomial products: in the reflected representation (bit 31 = x^0) the register is a
// polynomial R(x) and Z_n(R) = R * x^(8n) mod P.  mulmod is the carry-less product mod P, bit by bit.
inline uint32_t mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
  for (int i = 31; i >= 0; --i) {
    if ((a >> i) & 1u) p ^= b;
    b = (b >> 1) ^ (kPolyReflected & (0u - (b & 1u)));
  }
  return p;
}

// out[k] = x^(2^k) mod P, k < 64: Z_n of any n is a product of at most 64 of them (the device's gf2_shift).
inline void x2n_table(uint32_t* out) {
  out[0] = 0x40000000u;  // x^1
  for (int k = 1; k < 64; ++k) out[k] = mulmod(out[k - 1], out[k - 1]);
}

// x^-1 mod P: P has constant term 1, so x * (P - 1)/x = P - 1 = 1 mod P.  In the reflected representation (P - 1)/x
// is the constant without its x^0 bit (bit 31), every power moved down by one (bit 31 - i -> bit 32 - i: a left
// shift) and x^31 (bit 0) from P's x^32.
constexpr uint32_t kXInverse = (kPolyReflected << 1) | 1u;

// out[k] = x^(-8k) mod P, k < 16: Z_k^-1, the register rewound over k zero bytes (a register entering k zero bytes
// before position q that reaches R at q is Z_k^-1(R)).
inline void xinv_table(uint32_t* out) {
  uint32_t x8 = 0x80000000u;  // x^0
  for (int i = 0; i < 8; ++i) x8 = mulmod(x8, kXInverse);
  out[0] = 0x80000000u;
  for (int k = 1; k < 16; ++k) out[k] = mulmod(out[k - 1], x8);
}

}  // namespace gf2
}  // namespace kvsep
