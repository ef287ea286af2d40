// Reference-side caller of the batched SST read check, in C++: what a KVDB maintainer would write for a whole-table
// verify pass -- RepairDB's ScanTable (db/repair.cc:220-260) and paranoid compaction inputs
// (db/version_set.cc:1462) read every block of a table with ReadOptions::verify_checksums, one ReadBlock
// (table/format.cc:73-108) per block.  Here the table file is read once into host memory, its footer and index block
// are decoded (table/format.cc:37-60, table/block.cc), and every block -- data blocks, the metaindex block and the index
// block -- is checked by ONE kvsep_sst_verify_host call.  Then one byte of data block k is flipped and the call must
// name exactly block k, as ReadBlock would fail exactly there.  Prints the handles it found, then PASS.
// Usage: sst_verify_demo <table.sst>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "kvsep_crc32c.h"

#define CHECK(c)                                                                  \
  do {                                                                            \
    if (!(c)) {                                                                   \
      std::printf("FAILED line %d: %s (%s)\n", __LINE__, #c, kvsep_last_error()); \
      return 1;                                                                   \
    }                                                                             \
  } while (0)

namespace {

constexpr uint64_t kTableMagic = 0xdb4775248b80fb57ull;  // table/format.h kTableMagicNumber
constexpr size_t kFooterLen = 48;                        // 2 * BlockHandle::kMaxEncodedLength + 8
constexpr size_t kTrailer = 5;                           // type byte + masked crc (table/format.h kBlockTrailerSize)

bool varint64(const uint8_t*& p, const uint8_t* end, uint64_t* v) {  // util/coding.cc GetVarint64Ptr
  uint64_t r = 0;
  for (int shift = 0; shift <= 63 && p < end; shift += 7) {
    const uint64_t b = *p++;
    r |= (b & 127) << shift;
    if (!(b & 128)) {
      *v = r;
      return true;
    }
  }
  return false;
}

uint32_t le32(const uint8_t* p) { return uint32_t(p[0]) | uint32_t(p[1]) << 8 | uint32_t(p[2]) << 16 | uint32_t(p[3]) << 24; }

// Block entries (table/block.cc DecodeEntry): shared, non_shared, value_length varint32s, key delta, value; the restart
// array (u32 each) and its count end the block.  The index block's values are the data blocks' BlockHandles.
bool index_handles(const uint8_t* blk, uint64_t n, std::vector<uint64_t>* off, std::vector<uint64_t>* len) {
  if (n < 4) return false;
  const uint32_t restarts = le32(blk + n - 4);
  if (uint64_t(restarts) * 4 + 4 > n) return false;
  const uint8_t* p = blk;
  const uint8_t* limit = blk + n - 4 - uint64_t(restarts) * 4;
  while (p < limit) {
    uint64_t shared, non_shared, vlen;
    if (!varint64(p, limit, &shared) || !varint64(p, limit, &non_shared) || !varint64(p, limit, &vlen)) return false;
    if (uint64_t(limit - p) < non_shared + vlen) return false;
    p += non_shared;  // the key delta (not needed here)
    const uint8_t* v = p;
    uint64_t o, s;
    if (!varint64(v, p + vlen, &o) || !varint64(v, p + vlen, &s)) return false;
    off->push_back(o);
    len->push_back(s);
    p += vlen;
  }
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  CHECK(argc > 1);
  FILE* f = std::fopen(argv[1], "rb");
  CHECK(f);
  std::fseek(f, 0, SEEK_END);
  const uint64_t size = uint64_t(std::ftell(f));
  std::fseek(f, 0, SEEK_SET);
  CHECK(size >= kFooterLen);
  char* img = static_cast<char*>(kvsep_host_alloc_pinned(size));
  CHECK(img);
  CHECK(std::fread(img, 1, size, f) == size);
  std::fclose(f);
  const uint8_t* u = reinterpret_cast<const uint8_t*>(img);

  // Footer (table/format.cc:37-60): metaindex handle, index handle, padding, magic
  const uint8_t* ft = u + size - kFooterLen;
  CHECK((uint64_t(le32(ft + 44)) << 32 | le32(ft + 40)) == kTableMagic);
  const uint8_t* p = ft;
  uint64_t meta_off, meta_len, index_off, index_len;
  CHECK(varint64(p, ft + 40, &meta_off) && varint64(p, ft + 40, &meta_len));
  CHECK(varint64(p, ft + 40, &index_off) && varint64(p, ft + 40, &index_len));
  CHECK(index_off + index_len + kTrailer <= size && meta_off + meta_len + kTrailer <= size);

  // the index block is itself checked before its handles are trusted (Table::Open reads it with ReadBlock)
  uint32_t crc;
  uint64_t first_bad = 0, nbad = 0;
  kvsep_crc32c_ctx* ctx = nullptr;
  CHECK(kvsep_crc32c_ctx_create(0, &ctx) == KVSEP_OK);
  CHECK(kvsep_sst_verify_host(ctx, img, size, &index_off, &index_len, &crc, &first_bad, &nbad, 1) == KVSEP_OK);
  CHECK(nbad == 0);

  std::vector<uint64_t> off, len;
  CHECK(index_handles(u + index_off, index_len, &off, &len));
  const size_t ndata = off.size();
  off.push_back(meta_off);
  len.push_back(meta_len);
  off.push_back(index_off);
  len.push_back(index_len);
  for (size_t i = 0; i < off.size(); ++i) std::printf("handle %zu %lu %lu\n", i, (unsigned long)off[i], (unsigned long)len[i]);

  // one batched read check over every block of the table
  std::vector<uint32_t> out(off.size());
  CHECK(kvsep_sst_verify_host(ctx, img, size, off.data(), len.data(), out.data(), &first_bad, &nbad, off.size()) ==
        KVSEP_OK);
  CHECK(nbad == 0 && first_bad == UINT64_MAX);
  // each word is the scalar drop-in's Value(block + type byte), i.e. Unmask of the stored trailer word
  for (size_t i = 0; i < off.size(); ++i) {
    CHECK(out[i] == kvsep_crc32c_value(img + off[i], len[i] + 1));
    CHECK(out[i] == kvsep_crc32c_unmask(le32(u + off[i] + len[i] + 1)));
  }

  // a flipped byte in data block k: the batch names exactly k, as the per-block ReadBlock loop would
  const size_t k = ndata / 2;
  img[off[k] + len[k] / 3] ^= 0x20;
  CHECK(kvsep_sst_verify_host(ctx, img, size, off.data(), len.data(), out.data(), &first_bad, &nbad, off.size()) ==
        KVSEP_OK);
  CHECK(first_bad == k && nbad == 1);
  std::printf("blocks %zu data %zu corrupted %zu -> first_bad %lu nbad %lu\n", off.size(), ndata, k,
              (unsigned long)first_bad, (unsigned long)nbad);

  kvsep_host_free_pinned(img);
  kvsep_crc32c_ctx_destroy(ctx);
  std::printf("PASS\n");
  return 0;
}
