// leveldb_abi.cpp -- the link-level drop-in: libkvsep_leveldb_abi.so (a shim over libkvsep_crc32c.so, kept out of the
// engine library so that loading the engine never interposes a real LevelDB's Extend) exports the reference's own
// C++ symbol
//   uint32_t leveldb::crc32c::Extend(uint32_t init_crc, const char* data, size_t n)   (util/crc32c.h:17)
// (mangled _ZN7leveldb6crc32c6ExtendEjPKcm), defined out of line exactly as util/crc32c.cc:276 defines it.
// A KVDB build keeps its unchanged util/crc32c.h -- Value / Mask / Unmask / kMaskDelta stay header-inline there
// (util/crc32c.h:20-38) -- drops util/crc32c.cc from its sources and links this shim (and the engine) instead; every call
// site (db/value_log_writer.cc:57, db/value_log_reader.cc:110, db/log_writer.cc:19,98, db/log_reader.cc:248,
// table/table_builder.cc:223-224, table/format.cc:102) then resolves to the engine.  tests/test_refcallsites.py
// links the reference's own vlog writer/reader that way.
#include <cstddef>
#include <cstdint>

#include "../../include/kvsep_crc32c.h"

namespace leveldb {
namespace crc32c {

// Same contract as util/crc32c.cc:276-377: total, reentrant, any alignment, n == 0 returns init_crc.
__attribute__((visibility("default"))) uint32_t Extend(uint32_t init_crc, const char* data, size_t n) {
  return kvsep_crc32c_extend(init_crc, data, n);
}

}  // namespace crc32c
}  // namespace leveldb
