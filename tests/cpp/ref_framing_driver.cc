// ref_framing_driver.cc -- TEST INFRASTRUCTURE ONLY (never shipped, never measured).
//
// Drives the reference's OWN framing code, compiled unchanged from /root/reference by oracle/Makefile:
//   db/value_log_writer.cc:33-76 / db/value_log_reader.cc:64-138   vlog records
//   db/log_writer.cc:23-115 / db/log_reader.cc:58-272              MANIFEST (log) records, 32 KiB blocks
//   table/table_builder.cc:83-232 / table/format.cc:73-155         SST blocks and their 5-byte trailers
// It is linked twice (oracle/Makefile `framing`):
//   oracle/_ref/ref_framing_golden   with the reference's util/crc32c.cc: writes the golden files and the readers'
//                                    verdicts on corrupted copies (tests/golden/make_framing_golden.py commits them);
//   oracle/_ref/ref_framing_kvsep    with util/crc32c.cc replaced by libkvsep_crc32c.so (its exported
//                                    leveldb::crc32c::Extend): the same call sites on this engine.  With "gpu"
//                                    every Extend -- down to InitTypeCrc's 1-byte ones -- goes through the GPU
//                                    (offload threshold 0) and the run checks that none fell back to the host.
// Both builds print the same JSON for the same inputs iff the engine is bit-exact at every call site.
//
// usage: <binary> <out_dir> [gpu]
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "db/log_reader.h"
#include "db/log_writer.h"
#include "db/value_log_reader.h"
#include "db/value_log_writer.h"
#include "leveldb/env.h"
#include "leveldb/options.h"
#include "leveldb/table_builder.h"
#include "table/format.h"
#include "util/crc32c.h"

#ifdef KVSEP_CALLSITE
#include "kvsep_crc32c.h"
#endif

using leveldb::Slice;
using leveldb::Status;

namespace {

// The repo's synthetic byte stream (kvsep/workloads.py): byte i = byte (i & 7) of splitmix64 word (i >> 3).
uint64_t splitmix_word(uint64_t seed, uint64_t j) {
  uint64_t z = seed + (j + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
std::string stream_bytes(uint64_t seed, uint64_t off, uint64_t n) {
  std::string s(n, '\0');
  for (uint64_t i = 0; i < n; ++i) s[i] = char(splitmix_word(seed, (off + i) >> 3) >> (8 * ((off + i) & 7)));
  return s;
}

uint64_t fnv64(const char* p, size_t n) {  // record identity in the JSON (independent of the CRC under test)
  uint64_t h = 0xcbf29ce484222325ull;
  for (size_t i = 0; i < n; ++i) h = (h ^ uint8_t(p[i])) * 0x100000001b3ull;
  return h;
}

class StringSink : public leveldb::WritableFile {
 public:
  std::string contents;
  std::vector<std::pair<uint64_t, uint64_t>> appends;  // (offset, size) of every Append
  Status Append(const Slice& d) override {
    appends.emplace_back(contents.size(), d.size());
    contents.append(d.data(), d.size());
    return Status::OK();
  }
  Status Close() override { return Status::OK(); }
  Status Flush() override { return Status::OK(); }
  Status Sync() override { return Status::OK(); }
  size_t GetSize() override { return contents.size(); }
};

class StringSource : public leveldb::SequentialFile {
 public:
  explicit StringSource(const std::string& s) : data_(s) {}
  Status Read(size_t n, Slice* result, char* scratch) override {
    const size_t k = std::min<size_t>(n, data_.size() - pos_);
    std::memcpy(scratch, data_.data() + pos_, k);
    pos_ += k;
    *result = Slice(scratch, k);
    return Status::OK();
  }
  Status Skip(uint64_t n) override {
    pos_ = std::min<size_t>(data_.size(), pos_ + n);
    return Status::OK();
  }

 private:
  const std::string& data_;
  size_t pos_ = 0;
};

class StringRandom : public leveldb::RandomAccessFile {
 public:
  explicit StringRandom(const std::string& s) : data_(s) {}
  Status Read(uint64_t offset, size_t n, Slice* result, char* scratch) const override {
    if (offset > data_.size()) return Status::IOError("offset past end");
    const size_t k = std::min<size_t>(n, data_.size() - offset);
    std::memcpy(scratch, data_.data() + offset, k);
    *result = Slice(scratch, k);
    return Status::OK();
  }

 private:
  const std::string& data_;
};

struct Drops {
  std::vector<std::pair<size_t, std::string>> v;
  std::string json() const {
    std::string s = "[";
    for (size_t i = 0; i < v.size(); ++i) {
      char b[64];
      std::snprintf(b, sizeof b, "%s[%zu,", i ? "," : "", v[i].first);
      s += b;
      s += "\"" + v[i].second + "\"]";
    }
    return s + "]";
  }
};

struct VlogReporter : leveldb::log::VlogReader::Reporter {
  Drops d;
  void Corruption(size_t bytes, const Status& st) override { d.v.emplace_back(bytes, st.ToString()); }
};

struct LogReporter : leveldb::log::Reader::Reporter {
  Drops d;
  void Corruption(size_t bytes, const Status& st) override { d.v.emplace_back(bytes, st.ToString()); }
};

bool write_file(const std::string& path, const std::string& s) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) return false;
  const bool ok = std::fwrite(s.data(), 1, s.size(), f) == s.size();
  return std::fclose(f) == 0 && ok;
}

std::string hex(const char* p, size_t n) {
  static const char* d = "0123456789abcdef";
  std::string s;
  for (size_t i = 0; i < n; ++i) {
    s += d[uint8_t(p[i]) >> 4];
    s += d[uint8_t(p[i]) & 15];
  }
  return s;
}

// ------------------------------------------------------------------ vlog
constexpr uint64_t kVlogSeed = 0x766c6f67;
const uint64_t kVlogLens[] = {0, 1, 7, 8, 15, 16, 100, 4095, 4096, 65539, 1048609, 1048609, 1048609, 300001, 33};
constexpr size_t kVlogN = sizeof(kVlogLens) / sizeof(kVlogLens[0]);

// Records VlogReader returns (header + payload each, db/value_log_reader.cc:101,126) and what it reported.
std::string vlog_read(const std::string& img) {
  StringSource src(img);
  VlogReporter rep;
  leveldb::log::VlogReader r(&src, &rep, true, 0);
  Slice rec;
  std::string scratch;
  std::string out = "[";
  int k = 0;
  while (r.ReadRecord(&rec, &scratch)) {
    char b[64];
    std::snprintf(b, sizeof b, "%s[%zu,\"%016llx\"]", k++ ? "," : "", rec.size(),
                  (unsigned long long)fnv64(rec.data(), rec.size()));
    out += b;
  }
  return "{\"records\":" + out + "],\"drops\":" + rep.d.json() + "}";
}

std::string vlog_section(const std::string& dir) {
  StringSink sink;
  leveldb::log::VlogWriter w(&sink);
  uint64_t pos = 0;
  std::string offs = "[";
  for (size_t i = 0; i < kVlogN; ++i) {
    const std::string p = stream_bytes(kVlogSeed, pos, kVlogLens[i]);
    pos += kVlogLens[i];
    uint64_t off = 0;
    if (!w.AddRecord(Slice(p), off).ok()) std::abort();
    offs += (i ? "," : "") + std::to_string(off);
  }
  offs += "]";
  const std::string& img = sink.contents;
  if (!dir.empty() && !write_file(dir + "/vlog.bin", img)) std::abort();
  std::string headers = "[";
  for (size_t i = 0, p = 0; i < kVlogN; p += 8 + kVlogLens[i], ++i) headers += (i ? ",\"" : "\"") + hex(&img[p], 8) + "\"";
  headers += "]";
  // corrupted copies: a payload byte of record 11, the stored CRC of record 3, the low length byte of record 9,
  // and a torn tail (the last record cut short)
  auto rec_at = [&](size_t k) {
    uint64_t p = 0;
    for (size_t i = 0; i < k; ++i) p += 8 + kVlogLens[i];
    return p;
  };
  struct Case {
    const char* name;
    uint64_t flip;  // byte XOR 0x80 at this offset, or
    uint64_t cut;   // truncate to this size (0 = no)
  };
  const Case cases[] = {{"payload_r11", rec_at(11) + 8 + 524288, 0},
                        {"crc_r3", rec_at(3) + 1, 0},
                        {"len_r9", rec_at(9) + 4, 0},
                        {"torn_tail", 0, img.size() - 5}};
  std::string cs = "[";
  for (size_t c = 0; c < sizeof(cases) / sizeof(cases[0]); ++c) {
    std::string bad = img;
    if (cases[c].cut) bad.resize(cases[c].cut);
    else bad[cases[c].flip] ^= char(0x80);
    char b[128];
    std::snprintf(b, sizeof b, "%s{\"name\":\"%s\",\"flip\":%llu,\"cut\":%llu,\"reader\":", c ? "," : "", cases[c].name,
                  (unsigned long long)cases[c].flip, (unsigned long long)cases[c].cut);
    cs += b + vlog_read(bad) + "}";
  }
  cs += "]";
  std::string lens = "[";
  for (size_t i = 0; i < kVlogN; ++i) lens += (i ? "," : "") + std::to_string(kVlogLens[i]);
  lens += "]";
  return "{\"seed\":" + std::to_string(kVlogSeed) + ",\"lens\":" + lens + ",\"offsets\":" + offs +
         ",\"size\":" + std::to_string(img.size()) + ",\"headers\":" + headers + ",\"intact\":" + vlog_read(img) +
         ",\"cases\":" + cs + "}";
}

// ------------------------------------------------------------------ log / MANIFEST
constexpr uint64_t kLogSeed = 0x6d616e69;
constexpr uint64_t kBlock = 32768, kHeader = 7;

std::string log_read(const std::string& img) {
  StringSource src(img);
  LogReporter rep;
  leveldb::log::Reader r(&src, &rep, true, 0);
  Slice rec;
  std::string scratch, out = "[";
  int k = 0;
  while (r.ReadRecord(&rec, &scratch)) {
    char b[64];
    std::snprintf(b, sizeof b, "%s[%zu,\"%016llx\"]", k++ ? "," : "", rec.size(),
                  (unsigned long long)fnv64(rec.data(), rec.size()));
    out += b;
  }
  return "{\"records\":" + out + "],\"drops\":" + rep.d.json() + "}";
}

std::string log_section(const std::string& dir) {
  // Lengths are chosen from the block offset so that every fragment type and every trailer case appears:
  // block trailers of 3 and 6 zero bytes, a record starting with exactly 7 bytes left in its block (a FIRST
  // fragment of 0 bytes, db/log_writer.cc:47-58), FIRST/MIDDLE/LAST chains, an empty record; then the log is
  // reopened with dest_length (the MANIFEST-reuse constructor, db/log_writer.cc:25-28) and appended to.
  StringSink sink;
  std::vector<uint64_t> lens;
  std::vector<int> writer_of;
  uint64_t pos = 0;
  auto boff = [&] { return sink.contents.size() % kBlock; };
  auto add = [&](leveldb::log::Writer& w, uint64_t n, int wi) {
    const std::string p = stream_bytes(kLogSeed, pos, n);
    pos += n;
    if (!w.AddRecord(Slice(p)).ok()) std::abort();
    lens.push_back(n);
    writer_of.push_back(wi);
  };
  auto leave = [&](uint64_t k) { return kBlock - boff() - kHeader - k; };  // record length leaving k bytes
  {
    leveldb::log::Writer w(&sink);
    add(w, 100, 0);
    add(w, leave(3), 0);   // 3-byte trailer
    add(w, 50000, 0);      // FIRST + LAST
    add(w, 0, 0);          // empty FULL record
    add(w, leave(6), 0);   // 6-byte trailer
    add(w, 100000, 0);     // FIRST + MIDDLE + MIDDLE + LAST
    add(w, leave(7), 0);   // exactly a header's room left ...
    add(w, 5000, 0);       // ... so this starts with a 0-byte FIRST fragment
  }
  const uint64_t reopen_at = sink.contents.size();
  {
    leveldb::log::Writer w(&sink, reopen_at);
    add(w, 1, 1);
    add(w, 70000, 1);
    add(w, leave(1), 1);   // 1-byte trailer
    add(w, 33, 1);
  }
  const std::string& img = sink.contents;
  if (!dir.empty() && !write_file(dir + "/manifest.log", img)) std::abort();
  // physical records (for picking corruption targets): walk as log_reader.cc does
  std::vector<uint64_t> phys;
  for (uint64_t b = 0; b < img.size(); b += kBlock) {
    uint64_t p = b;
    const uint64_t end = std::min<uint64_t>(b + kBlock, img.size());
    while (end - p >= kHeader) {
      const uint64_t l = uint8_t(img[p + 4]) | (uint64_t(uint8_t(img[p + 5])) << 8);
      if (img[p + 6] == 0 && l == 0) break;
      phys.push_back(p);
      p += kHeader + l;
    }
  }
  auto frag_len = [&](size_t k) { return uint8_t(img[phys[k] + 4]) | (uint64_t(uint8_t(img[phys[k] + 5])) << 8); };
  auto first_of_type = [&](int t, size_t from) {
    for (size_t k = from; k < phys.size(); ++k)
      if (img[phys[k] + 6] == t && frag_len(k) > 0) return k;
    std::abort();
  };
  const size_t full = first_of_type(1, 0), first = first_of_type(2, 0), middle = first_of_type(3, 0),
               last = first_of_type(4, middle);
  struct Case {
    const char* name;
    uint64_t flip;
  };
  const Case cases[] = {{"full_payload", phys[full] + kHeader + frag_len(full) / 2},
                        {"first_payload", phys[first] + kHeader + 17},
                        {"middle_payload", phys[middle] + kHeader + 1000},
                        {"last_payload", phys[last] + kHeader + frag_len(last) - 1},
                        {"type_byte", phys[middle] + 6},
                        {"length_field", phys[first_of_type(1, last)] + 5},
                        {"crc_after_reopen", phys[first_of_type(2, first_of_type(1, last))] + 2}};
  std::string cs = "[";
  for (size_t c = 0; c < sizeof(cases) / sizeof(cases[0]); ++c) {
    std::string bad = img;
    bad[cases[c].flip] ^= char(0x80);
    char b[128];
    std::snprintf(b, sizeof b, "%s{\"name\":\"%s\",\"flip\":%llu,\"reader\":", c ? "," : "", cases[c].name,
                  (unsigned long long)cases[c].flip);
    cs += b + log_read(bad) + "}";
  }
  cs += "]";
  std::string ls = "[", ws = "[";
  for (size_t i = 0; i < lens.size(); ++i) {
    ls += (i ? "," : "") + std::to_string(lens[i]);
    ws += (i ? "," : "") + std::to_string(writer_of[i]);
  }
  return "{\"seed\":" + std::to_string(kLogSeed) + ",\"lens\":" + ls + "],\"writer\":" + ws +
         "],\"reopen_at\":" + std::to_string(reopen_at) + ",\"size\":" + std::to_string(img.size()) +
         ",\"physical_records\":" + std::to_string(phys.size()) + ",\"intact\":" + log_read(img) + ",\"cases\":" + cs +
         "}";
}

// ------------------------------------------------------------------ SST
constexpr uint64_t kSstSeed = 0x73737462;

std::string sst_section(const std::string& dir) {
  leveldb::Options opt;  // block_size 4 KiB (include/leveldb/options.h:101); no snappy here -> raw blocks
  opt.compression = leveldb::kNoCompression;
  StringSink sink;
  {
    leveldb::TableBuilder tb(opt, &sink);
    for (int i = 0; i < 1500; ++i) {
      char key[32];
      std::snprintf(key, sizeof key, "key%08d", i * 7);
      const std::string v = stream_bytes(kSstSeed, uint64_t(i) * 100, 37 + (i * 13) % 200);
      tb.Add(Slice(key), Slice(v));
    }
    if (!tb.Finish().ok()) std::abort();
  }
  const std::string& img = sink.contents;
  if (!dir.empty() && !write_file(dir + "/table.sst", img)) std::abort();
  // WriteRawBlock appends the block, then its 5-byte trailer (table/table_builder.cc:217-227): every Append
  // followed by a 5-byte Append is a block.
  std::vector<std::pair<uint64_t, uint64_t>> blocks;
  for (size_t i = 0; i + 1 < sink.appends.size(); ++i)
    if (sink.appends[i + 1].second == leveldb::kBlockTrailerSize &&
        sink.appends[i + 1].first == sink.appends[i].first + sink.appends[i].second)
      blocks.push_back(sink.appends[i]);
  auto verdicts = [&](const std::string& f) {  // ReadBlock(verify_checksums) per block: 1 = ok
    StringRandom file(f);
    leveldb::ReadOptions ro;
    ro.verify_checksums = true;
    std::string s = "[";
    for (size_t k = 0; k < blocks.size(); ++k) {
      leveldb::BlockHandle h;
      h.set_offset(blocks[k].first);
      h.set_size(blocks[k].second);
      leveldb::BlockContents bc;
      const Status st = leveldb::ReadBlock(&file, ro, h, &bc);
      if (st.ok() && bc.heap_allocated) delete[] bc.data.data();
      s += std::string(k ? "," : "") + (st.ok() ? "1" : "0");
    }
    return s + "]";
  };
  std::string bl = "[";
  for (size_t k = 0; k < blocks.size(); ++k) {
    const uint64_t o = blocks[k].first, n = blocks[k].second;
    bl += (k ? ",[" : "[") + std::to_string(o) + "," + std::to_string(n) + "," + std::to_string(uint8_t(img[o + n])) +
          ",\"" + hex(&img[o + n + 1], 4) + "\"]";
  }
  bl += "]";
  const uint64_t b5 = blocks[5].first, b9 = blocks[9].first + blocks[9].second, b2 = blocks[2].first + blocks[2].second,
                 bi = blocks.back().first;
  const uint64_t flips[] = {b5 + 100, b9 + 3, b2, bi + 1};
  const char* names[] = {"data_block_5", "trailer_crc_9", "type_byte_2", "last_block"};
  std::string cs = "[";
  for (int c = 0; c < 4; ++c) {
    std::string bad = img;
    bad[flips[c]] ^= char(0x80);
    cs += std::string(c ? "," : "") + "{\"name\":\"" + names[c] + "\",\"flip\":" + std::to_string(flips[c]) +
          ",\"ok\":" + verdicts(bad) + "}";
  }
  cs += "]";
  return "{\"size\":" + std::to_string(img.size()) + ",\"blocks\":" + bl + ",\"intact_ok\":" + verdicts(img) +
         ",\"cases\":" + cs + "}";
}

}  // namespace

int main(int argc, char** argv) {
  const std::string dir = argc > 1 ? argv[1] : "";
  const bool gpu = argc > 2 && std::strcmp(argv[2], "gpu") == 0;
#ifdef KVSEP_CALLSITE
  if (gpu) {  // every Extend of the reference call sites on the GPU
    kvsep_set_offload_threshold(0);
    kvsep_set_offload_wait(1);
  }
#else
  if (gpu) {
    std::fprintf(stderr, "gpu mode needs the KVSEP_CALLSITE build\n");
    return 2;
  }
#endif
  const std::string j = "{\"vlog\":" + vlog_section(dir) + ",\"log\":" + log_section(dir) + ",\"sst\":" +
                        sst_section(dir) + "}";
#ifdef KVSEP_CALLSITE
  uint64_t g = 0, h = 0, f = 0;
  kvsep_offload_stats(&g, &h, &f);
  std::fprintf(stderr, "kvsep offload: %llu gpu calls, %llu host calls, %llu gpu failures\n", (unsigned long long)g,
               (unsigned long long)h, (unsigned long long)f);
  if (gpu && (g == 0 || h != 0 || f != 0)) return 3;  // every call must have run on the GPU
#endif
  std::printf("%s\n", j.c_str());
  return 0;
}
