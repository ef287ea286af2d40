// kvsep_leveldb_crc32c.h -- stand-in for the reference's util/crc32c.h (util/crc32c.h:11-41): same
// namespace, same declarations, same inline helpers.  Extend is declared, not defined, exactly as in
// util/crc32c.h:17: libkvsep_leveldb_abi.so exports the out-of-line definition (csrc/leveldb_abi.cpp), so a
// KVDB build can either keep its own util/crc32c.h or include this one -- both resolve
// leveldb::crc32c::Extend to the library at link time once util/crc32c.cc is dropped from the sources.
// Call sites: db/value_log_writer.cc:57, db/value_log_reader.cc:110, db/log_writer.cc:19,98,
// db/log_reader.cc:248, table/table_builder.cc:223-224, table/format.cc:102.
#ifndef KVSEP_LEVELDB_CRC32C_H_
#define KVSEP_LEVELDB_CRC32C_H_

#include <cstddef>
#include <cstdint>

#include "kvsep_crc32c.h"

namespace leveldb {
namespace crc32c {

// util/crc32c.h:17 -- crc32c of concat(A, data[0,n-1]) where init_crc = crc32c(A).  Defined in
// libkvsep_leveldb_abi.so (C++ linkage, = kvsep_crc32c_extend of libkvsep_crc32c.so).
uint32_t Extend(uint32_t init_crc, const char* data, size_t n);

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
