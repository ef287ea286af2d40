/*
 * crc32c_oracle.c -- TEST INFRASTRUCTURE ONLY (the parity checker, never the product).
 *
 * A plain-C restatement of the reference's portable CRC-32C path
 *   /root/reference/util/crc32c.cc:276-377  (leveldb::crc32c::Extend)
 *   /root/reference/util/crc32c.h:17-38     (Value / Mask / Unmask / kMaskDelta)
 * used by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only.
 *
 * Parity pinning: the tables here are *generated* from the Castagnoli polynomial
 * (reflected 0x82F63B78) instead of copied, and the restatement is checked against
 *   (1) the RFC 3720 B.4 known answers of util/crc32c_test.cc:12-53, and
 *   (2) golden vectors produced by the real reference util/crc32c.cc, compiled
 *       from /root/reference by oracle/Makefile into oracle/_ref/ and captured by
 *       tests/golden/make_golden.py into tests/golden/crc32c_golden.json.
 *
 * Structure mirrors the reference loop so the two can be read side by side:
 *   - conditioning with ~0 on entry and exit            (util/crc32c.cc:284,376)
 *   - byte steps until the pointer is 4-byte aligned     (util/crc32c.cc:322-330)
 *   - four interleaved 4-byte strides over 16-byte swaths (util/crc32c.cc:332-348)
 *   - single-word rotation of the strides                 (util/crc32c.cc:350-359)
 *   - folding the four stride words back in byte by byte  (util/crc32c.cc:361-366)
 *   - byte tail                                           (util/crc32c.cc:369-371)
 */
#include <stdint.h>
#include <stddef.h>
#include <string.h>
#include <pthread.h>

#define ORACLE_POLY_REFLECTED 0x82F63B78u
#define ORACLE_MASK_DELTA 0xa282ead8u /* util/crc32c.h:22 */

/* byte_tab[b]      : register after one zero byte when the low register byte is b
 *                    (role of kByteExtensionTable, util/crc32c.cc:20)
 * swath_tab[k][b]  : contribution of byte b sitting in lane k (k = 0 is the lowest,
 *                    i.e. earliest, byte) of a 4-byte word that is carried 16 bytes
 *                    forward (role of kStrideExtensionTable3..0, util/crc32c.cc:65-245;
 *                    the reference indexes them in the opposite order). */
static uint32_t byte_tab[256];
static uint32_t swath_tab[4][256];
static pthread_once_t tab_once = PTHREAD_ONCE_INIT;

static uint32_t shift_zero_bytes(uint32_t reg, int nbytes) {
  for (int i = 0; i < nbytes; ++i) reg = byte_tab[reg & 0xffu] ^ (reg >> 8);
  return reg;
}

static void build_tables(void) {
  for (uint32_t b = 0; b < 256; ++b) {
    uint32_t r = b;
    for (int bit = 0; bit < 8; ++bit) r = (r >> 1) ^ (ORACLE_POLY_REFLECTED & (0u - (r & 1u)));
    byte_tab[b] = r;
  }
  for (int k = 0; k < 4; ++k)
    for (uint32_t b = 0; b < 256; ++b) swath_tab[k][b] = shift_zero_bytes(b << (8 * k), 16);
}

static inline uint32_t load_le32(const uint8_t* p) {
  /* util/coding.h:82 DecodeFixed32: little-endian regardless of host order */
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

static inline uint32_t carry_word16(uint32_t w) {
  return swath_tab[0][w & 0xffu] ^ swath_tab[1][(w >> 8) & 0xffu] ^
         swath_tab[2][(w >> 16) & 0xffu] ^ swath_tab[3][w >> 24];
}

uint32_t oracle_crc32c_extend(uint32_t init_crc, const uint8_t* data, size_t n) {
  pthread_once(&tab_once, build_tables);
  const uint8_t* p = data;
  const uint8_t* end = data + n;
  uint32_t reg = init_crc ^ 0xffffffffu;

  /* head: bytes until p is 4-byte aligned (only if the aligned point is inside) */
  const uint8_t* aligned = (const uint8_t*)(((uintptr_t)p + 3u) & ~(uintptr_t)3u);
  if (aligned <= end)
    while (p != aligned) reg = byte_tab[(reg ^ *p++) & 0xffu] ^ (reg >> 8);

  if (end - p >= 16) {
    uint32_t s[4];
    s[0] = load_le32(p) ^ reg;
    s[1] = load_le32(p + 4);
    s[2] = load_le32(p + 8);
    s[3] = load_le32(p + 12);
    p += 16;
    while (end - p >= 16) {
      for (int j = 0; j < 4; ++j) s[j] = load_le32(p + 4 * j) ^ carry_word16(s[j]);
      p += 16;
    }
    while (end - p >= 4) { /* advance one word, rotating the stride words */
      uint32_t nxt = load_le32(p) ^ carry_word16(s[0]);
      s[0] = s[1]; s[1] = s[2]; s[2] = s[3]; s[3] = nxt;
      p += 4;
    }
    reg = 0;
    for (int j = 0; j < 4; ++j) reg = shift_zero_bytes(s[j] ^ reg, 4);
  }
  while (p != end) reg = byte_tab[(reg ^ *p++) & 0xffu] ^ (reg >> 8);
  return reg ^ 0xffffffffu;
}

uint32_t oracle_crc32c_value(const uint8_t* data, size_t n) { return oracle_crc32c_extend(0, data, n); }

uint32_t oracle_crc32c_mask(uint32_t crc) { return ((crc >> 15) | (crc << 17)) + ORACLE_MASK_DELTA; }

uint32_t oracle_crc32c_unmask(uint32_t masked) {
  uint32_t rot = masked - ORACLE_MASK_DELTA;
  return (rot >> 17) | (rot << 15);
}

/* ---- synthetic-data generator shared with the device generator (kvsep_fill_splitmix64):
 * byte i of stream `seed` is byte (i & 7) (little-endian) of splitmix64 output number i>>3,
 * i.e. word j = mix(seed + (j + 1) * golden_gamma).  Counter-based so any range can be made
 * independently on host or device. */
static inline uint64_t splitmix_word(uint64_t seed, uint64_t j) {
  uint64_t z = seed + (j + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

void oracle_fill_splitmix64(uint8_t* dst, uint64_t nbytes, uint64_t seed, uint64_t stream_offset) {
  for (uint64_t i = 0; i < nbytes; ++i) {
    uint64_t g = stream_offset + i;
    dst[i] = (uint8_t)(splitmix_word(seed, g >> 3) >> (8 * (g & 7)));
  }
}

/* ---- batched form with the semantics of the device C-ABI (out[i] = Extend(init[i], base+off[i], len[i])),
 * optionally split over `nthreads` host threads by contiguous byte-balanced ranges. */
typedef struct {
  const uint8_t* base; const uint64_t* off; const uint64_t* len; const uint32_t* init;
  uint32_t* out; size_t lo, hi;
} batch_job;

static void* batch_worker(void* arg) {
  batch_job* j = (batch_job*)arg;
  for (size_t i = j->lo; i < j->hi; ++i)
    j->out[i] = oracle_crc32c_extend(j->init ? j->init[i] : 0u, j->base + j->off[i], (size_t)j->len[i]);
  return NULL;
}

int oracle_crc32c_batch(const uint8_t* base, const uint64_t* off, const uint64_t* len, const uint32_t* init,
                        uint32_t* out, size_t count, int nthreads) {
  pthread_once(&tab_once, build_tables);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  uint64_t total = 0;
  for (size_t i = 0; i < count; ++i) total += len[i];
  pthread_t th[256];
  batch_job jobs[256];
  size_t start = 0;
  uint64_t acc = 0;
  int launched = 0;
  for (int t = 0; t < nthreads && start < count; ++t) {
    uint64_t target = (total / (uint64_t)nthreads) * (uint64_t)(t + 1);
    size_t stop = start;
    if (t == nthreads - 1) stop = count;
    else
      while (stop < count && acc < target) acc += len[stop++];
    jobs[t] = (batch_job){base, off, len, init, out, start, stop};
    if (pthread_create(&th[t], NULL, batch_worker, &jobs[t]) != 0) return -1;
    ++launched;
    start = stop;
  }
  for (int t = 0; t < launched; ++t) pthread_join(th[t], NULL);
  return 0;
}
