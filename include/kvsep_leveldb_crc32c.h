// kvsep_leveldb_crc32c.h -- source-compatible stand-in for the reference's util/crc32c.h
// (/root/reference/util/crc32c.h:11-41): same namespace, same signatures, same inline helpers,
// with Extend forwarded to libkvsep_crc32c (include/kvsep_crc32c.h).  A LevelDB/KVDB build that
// includes this instead of util/crc32c.h and drops util/crc32c.cc from its sources links against
// -lkvsep_crc32c and needs no other change at its call sites (db/value_log_writer.cc:57,
// db/value_log_reader.cc:110, db/log_writer.cc:19,98, db/log_reader.cc:248,
// table/table_builder.cc:223-224, table/format.cc:102).
#ifndef KVSEP_LEVELDB_CRC32C_H_
#define KVSEP_LEVELDB_CRC32C_H_

#include <cstddef>
#include <cstdint>

#include "kvsep_crc32c.h"

namespace leveldb {
namespace crc32c {

// util/crc32c.h:17 -- crc32c of concat(A, data[0,n-1]) where init_crc = crc32c(A).
inline uint32_t Extend(uint32_t init_crc, const char* data, size_t n) {
  return kvsep_crc32c_extend(init_crc, data, n);
}

// util/crc32c.h:20
inline uint32_t Value(const char* data, size_t n) { return Extend(0, data, n); }

// util/crc32c.h:22
static const uint32_t kMaskDelta = 0xa282ead8ul;

// util/crc32c.h:29-32: rotate right by 15 bits and add a constant.
inline uint32_t Mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + kMaskDelta; }

// util/crc32c.h:35-38
inline uint32_t Unmask(uint32_t masked_crc) {
  uint32_t rot = masked_crc - kMaskDelta;
  return ((rot >> 17) | (rot << 15));
}

}  // namespace crc32c
}  // namespace leveldb

#endif  // KVSEP_LEVELDB_CRC32C_H_
