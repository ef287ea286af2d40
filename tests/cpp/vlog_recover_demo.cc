// End-to-end integration demo in C++ (what a KVDB maintainer would write around DBImpl::RecoverLogFile,
// db/db_impl.cc:448-571): frame a group of WriteBatch payloads into a vlog FILE on disk
// (db/value_log_writer.cc:46-76), read the file back into pinned memory, verify every record with one
// batched GPU checksum, corrupt one byte and check the reader's stop-at-first-bad semantics
// (db/value_log_reader.cc:109-123).  Prints PASS and exits 0 on success.  Usage: vlog_recover_demo <dir>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "kvsep_crc32c.h"

#define CHECK(c)                                              \
  do {                                                        \
    if (!(c)) {                                               \
      std::printf("FAILED line %d: %s (%s)\n", __LINE__, #c, kvsep_last_error()); \
      return 1;                                               \
    }                                                         \
  } while (0)

int main(int argc, char** argv) {
  const std::string path = std::string(argc > 1 ? argv[1] : "/tmp") + "/000001.vlog";
  kvsep_crc32c_ctx* ctx = nullptr;
  CHECK(kvsep_crc32c_ctx_create(0, &ctx) == KVSEP_OK);

  // 64 records of ~1 MiB (16-B key + 1 MiB value WriteBatch reps are 1,048,609 B)
  const int n = 64;
  std::vector<std::vector<char>> payload(n);
  std::vector<const char*> ptr(n);
  std::vector<uint64_t> len(n);
  uint64_t x = 0x9E3779B97F4A7C15ull;
  for (int i = 0; i < n; ++i) {
    payload[i].resize(1048609 + (i % 7) * 13);
    for (auto& c : payload[i]) {
      x ^= x << 13; x ^= x >> 7; x ^= x << 17;
      c = char(x);
    }
    ptr[i] = payload[i].data();
    len[i] = payload[i].size();
  }
  uint64_t need = 0;
  kvsep_vlog_frame_host(ctx, ptr.data(), len.data(), n, nullptr, 0, &need);
  std::vector<char> framed(need);
  uint64_t wrote = 0;
  CHECK(kvsep_vlog_frame_host(ctx, ptr.data(), len.data(), n, framed.data(), framed.size(), &wrote) == KVSEP_OK);
  FILE* f = std::fopen(path.c_str(), "wb");
  CHECK(f && std::fwrite(framed.data(), 1, wrote, f) == wrote);
  std::fclose(f);

  // recovery: file -> pinned buffer -> one batched verify
  char* img = static_cast<char*>(kvsep_host_alloc_pinned(wrote));
  CHECK(img);
  f = std::fopen(path.c_str(), "rb");
  CHECK(f && std::fread(img, 1, wrote, f) == wrote);
  std::fclose(f);
  uint64_t records = 0, good = 0, good_bytes = 0;
  CHECK(kvsep_vlog_verify_host(ctx, img, wrote, &records, &good, &good_bytes, nullptr) == KVSEP_OK);
  CHECK(records == uint64_t(n) && good == uint64_t(n) && good_bytes == wrote);

  // the host scalar drop-in agrees with every stored header (util/crc32c.h:17 semantics)
  for (uint64_t p = 0, i = 0; i < uint64_t(n); ++i) {
    uint32_t stored, l;
    std::memcpy(&stored, img + p, 4);
    std::memcpy(&l, img + p + 4, 4);
    CHECK(kvsep_crc32c_mask(kvsep_crc32c_value(img + p + 8, l)) == stored);
    p += 8 + l;
  }

  // corruption in record 40: the scan keeps records [0, 40)
  uint64_t off40 = 0;
  for (int i = 0; i < 40; ++i) off40 += 8 + len[i];
  img[off40 + 8 + 12345] ^= 0x80;
  CHECK(kvsep_vlog_verify_host(ctx, img, wrote, &records, &good, &good_bytes, nullptr) == KVSEP_OK);
  CHECK(records == uint64_t(n) && good == 40 && good_bytes == off40);

  kvsep_host_free_pinned(img);
  kvsep_crc32c_ctx_destroy(ctx);
  std::remove(path.c_str());
  std::printf("PASS\n");
  return 0;
}
