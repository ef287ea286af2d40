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
