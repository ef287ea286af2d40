// crc32c_device.hip -- CDNA4 (gfx950) kernels and the device-side C ABI of libkvsep_crc32c.
//
// Computes leveldb::crc32c::Extend (util/crc32c.cc:276-377) for batches of independent byte
// blocks resident in HBM.  Design:
//
//  * Work item = "piece": a block, or an end-aligned slice of at most `piece_bytes` of a long block
//    (pieces 1..k-1 are exactly piece_bytes long, piece 0 takes the remainder on top of a full piece, and the init CRC).
//  * One wavefront per piece.  The piece is cut at 16-byte-aligned addresses into
//      head  [ps, h0)   < 16 B, serial (word/byte steps),
//      body  [h0, a1)   16-B aligned, as rows of 1 KiB ending exactly at a1,
//      tail  [a1, pe)   < 16 B, serial.
//    In the body every lane loads one 16-B vector per row (global_load_dwordx4, one 1 KiB
//    coalesced wave-instruction per row) and owns four 32-bit "stride chains" -- the reference's
//    4-stride swath (util/crc32c.cc:332-348) widened to 256 strides, 1 KiB apart:
//        c' = word ^ Z_1024(c)
//    Z_1024 is evaluated as 4 byte-table lookups in LDS.  The four tables are replicated 32x so that
//    lane L always reads bank L%32: ds_read_b32 is conflict-free whatever the data.  The lookup
//    address (table pair, byte value, lane copy) is assembled by ONE v_perm_b32 per lookup.
//  * Chains are merged per lane with Z_4 (the STEP4W re-injection, util/crc32c.cc:307-315, 361-366),
//    then across the 64 lanes by a 6-level butterfly with Z_16 .. Z_512 (DPP/bpermute shuffles).
//  * Pieces of one block are merged by a tiny combine kernel: R(A||B) = Z_|B|(R(A)) ^ R(B).
//
// Every map Z_d ("advance the CRC register over d zero bytes") is generated on the host from the
// Castagnoli polynomial (gf2.h); no table is copied from the reference.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/kvsep_crc32c.h"
#include "gf2.h"
#include "kvsep_internal.h"

namespace kvsep {

// ------------------------------------------------------------------------------------------------
// LDS image of one CRC workgroup (bytes).  160,768 B of the 163,840 B a gfx950 workgroup may own.
constexpr int kWgThreads = 512;  // default CRC workgroup: 8 waves, 2 per SIMD (see launch_pieces_v)
// [0, 128 KiB): Z_1024, 4 byte-tables x 256 entries x 32 lane copies (see fold1024)
constexpr uint32_t kZ4Off = 131072;      // Z_4     (4 KiB)
constexpr uint32_t kTreeOff = 135168;    // Z_16, Z_32, Z_64, Z_128, Z_256, Z_512 (6 x 4 KiB)
constexpr uint32_t kByteOff = 159744;    // Z_1 low-byte table (1 KiB) = the STEP1 table
constexpr uint32_t kLdsBytes = 160768;
constexpr uint32_t kRowBytes = 1024;     // 64 lanes x 16 B

struct DevTables {
  uint32_t z1024[4][256];
  uint32_t z4[4][256];      // kZ4Off
  uint32_t ztree[6][4][256];// kTreeOff   (contiguous with z4 and byte1: copied to LDS as one run)
  uint32_t byte1[256];      // kByteOff
  uint32_t zpiece[4][256];  // Z_piece_bytes, used by the combine kernel
  uint32_t znarrow[4][256]; // Z_{16 kNarrowLanes}: the replicated table of the narrow kernel
  uint32_t zsmall[3][4][256];  // Z_16K, Z_32K, Z_64K: the automatic smaller pieces of small batches
  uint32_t x2n[64];         // x^(2^k) mod P (reflected): Z_n for ANY n by square-and-multiply (gf2_shift)
  uint32_t xinv[16];        // x^(-8k) mod P: Z_k^-1, a register rewound over k bytes (the padded-head variant)
};
static_assert(sizeof(DevTables) == 4096 * 13 + 1024 + 256 + 64, "table layout");
constexpr uint64_t kSmallPiece = 16 * 1024;  // zsmall[k] is Z_{kSmallPiece << k}

struct PiecesArgs {
  const uint8_t* base;
  const uint64_t* off;
  const uint64_t* len;
  const uint32_t* init;             // nullable -> 0
  uint32_t* out;
  uint64_t count;
  const uint64_t* pstart;           // planned mode: piece range of block b = [pstart[b], pstart[b+1]) (u64: an
                                    // understated total_bytes cannot wrap the scan, see the max_pieces fallback)
  const uint32_t* pblk;             // planned mode: block of piece g
  uint32_t* partial;                // planned mode: raw register of piece g
  uint32_t* work_counter;           // dynamic schedule
  uint64_t piece_bytes;             // of this batch (see piece_for)
  const uint32_t* zpiece;           // Z_piece_bytes as 4 byte tables (combine kernel)
  uint64_t max_pieces;              // capacity of pblk/partial
  uint32_t static_contig;           // static schedule: contiguous item ranges per wave (else round-robin)
  uint32_t guided_div;              // dynamic schedule: a grab takes remaining / (guided_div * nwaves) items;
                                    // 0: adaptive, clamp(total / (64 * nwaves), 4, 32)
  uint32_t guided_cap;              // dynamic schedule: at most this many items per grab (0: no cap)
  uint64_t hint;                    // narrow kernel: the caller's max_len hint; longer blocks are deferred (exact)
  // verify form (kVerify kernels): Mask(crc of block b) must equal expect[b] -- the check of
  // db/value_log_reader.cc:109-122 / table/format.cc:99-106.  The caller's result words first_bad (lowest mismatching
  // block, ~0 if none) and nbad are written once, by the last workgroup of the publishing kernel (verify_publish).
  const uint32_t* expect;
  unsigned long long* first_bad;
  unsigned long long* nbad;
  const DevTables* tabs;
  // The context's accumulator words, kept in their reset state between calls (layout at vacc_shard): mismatches post
  // there (atomicMin / atomicAdd); the last workgroup to arrive copies the verdict to first_bad / nbad and resets them,
  // so a verify call needs no init launch.
  unsigned long long* vacc;
};

// Descriptor reads through the constant address space: wave-uniform indices then lower to scalar
// s_load (lgkmcnt), so fetching the next item's descriptors never drains the vmcnt of in-flight
// payload loads.  Descriptors are read-only for the whole launch.
template <typename T>
__device__ __forceinline__ T ldc(const T* p, uint64_t i) {
  return reinterpret_cast<const __attribute__((address_space(4))) T*>(reinterpret_cast<uintptr_t>(p))[i];
}

__device__ __forceinline__ uint32_t lds_u32(const uint8_t* lds, uint32_t byte_off) {
  return *reinterpret_cast<const uint32_t*>(lds + byte_off);
}

// Three-input XOR as ONE instruction: CDNA4's v_bitop3_b32 with truth table 0x96 (a ^ b ^ c).  hipcc
// splits a^b^c^d of four LDS results into four v_xor_b32 (interleaved with partial lgkmcnt waits), and
// the folds are issue-bound for short blocks.
__device__ __forceinline__ uint32_t xor3(uint32_t a, uint32_t b, uint32_t c) {
  return __builtin_amdgcn_bitop3_b32(a, b, c, 0x96);
}

// Z_d through a plain (non-replicated) 4 KiB table set at byte offset t.
__device__ __forceinline__ uint32_t zmap(const uint8_t* lds, uint32_t t, uint32_t w) {
  return lds_u32(lds, t + ((w << 2) & 0x3fcu)) ^ lds_u32(lds, t + 1024u + ((w >> 6) & 0x3fcu)) ^
         lds_u32(lds, t + 2048u + ((w >> 14) & 0x3fcu)) ^ lds_u32(lds, t + 3072u + ((w >> 22) & 0x3fcu));
}

// Z_d(w) ^ x in two v_bitop3_b32.
__device__ __forceinline__ uint32_t zmap_x(const uint8_t* lds, uint32_t t, uint32_t w, uint32_t x) {
  return xor3(xor3(lds_u32(lds, t + ((w << 2) & 0x3fcu)), lds_u32(lds, t + 1024u + ((w >> 6) & 0x3fcu)), x),
              lds_u32(lds, t + 2048u + ((w >> 14) & 0x3fcu)), lds_u32(lds, t + 3072u + ((w >> 22) & 0x3fcu)));
}

// Z_1024 through the replicated tables.  Layout: byte addr = pair*64K + b*256 + half*128 + copy*4
// with table k = 2*pair + half.  v_perm_b32 picks {copy*4 | b<<8 | pair<<16} in one instruction:
//   sel byte0 = 0x00 -> lcX.byte0 (copy*4), byte1 = 0x04+k -> c.byte k, byte2 = 0x02 -> lcX.byte2 (pair),
//   byte3 = 0x0C -> 0.
__device__ __forceinline__ uint32_t fold1024(const uint8_t* lds, uint32_t c, uint32_t lc0, uint32_t lc1) {
  const uint32_t a0 = __builtin_amdgcn_perm(c, lc0, 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(c, lc0, 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(c, lc1, 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(c, lc1, 0x0C020700u);
  return lds_u32(lds, a0) ^ lds_u32(lds, a1 + 128u) ^ lds_u32(lds, a2) ^ lds_u32(lds, a3 + 128u);
}

// c' = w ^ Z(c) through the replicated table: two v_xor3_b32 for the five terms.
__device__ __forceinline__ uint32_t fold_step(const uint8_t* lds, uint32_t c, uint32_t w, uint32_t lc0, uint32_t lc1) {
  const uint32_t a0 = __builtin_amdgcn_perm(c, lc0, 0x0C020400u);
  const uint32_t a1 = __builtin_amdgcn_perm(c, lc0, 0x0C020500u);
  const uint32_t a2 = __builtin_amdgcn_perm(c, lc1, 0x0C020600u);
  const uint32_t a3 = __builtin_amdgcn_perm(c, lc1, 0x0C020700u);
  return xor3(xor3(lds_u32(lds, a0), lds_u32(lds, a1 + 128u), w), lds_u32(lds, a2), lds_u32(lds, a3 + 128u));
}

// DPP row_shr:N -- lane l receives lane l - N of its 16-lane row (a VALU op, no LDS round trip).
template <int N>
__device__ __forceinline__ uint32_t row_shr(uint32_t v) {
  return uint32_t(__builtin_amdgcn_update_dpp(0, int(v), 0x110 + N, 0xF, 0xF, false));
}

__device__ __forceinline__ uint4 uniform4(uint4 v) {
  return make_uint4(uint32_t(__builtin_amdgcn_readfirstlane(int(v.x))), uint32_t(__builtin_amdgcn_readfirstlane(int(v.y))),
                    uint32_t(__builtin_amdgcn_readfirstlane(int(v.z))), uint32_t(__builtin_amdgcn_readfirstlane(int(v.w))));
}

// Serial steps over bytes [q0, q1) of a 16-B aligned chunk (0 <= q0 <= q1 <= 16), wave-uniform.
// Aligned whole words take one Z_4 step (util/crc32c.cc STEP4W), the rest byte steps (STEP1).
// z4 / byte: where the LDS image keeps Z_4 and the STEP1 table (the compact narrow image reads the STEP1 table as
// Z_4's byte-3 table: Z_4(b << 24) = Z_1(b), see LdsCompact).
__device__ __forceinline__ uint32_t serial16(const uint8_t* lds, uint32_t reg, uint4 ch, int q0, int q1,
                                             uint32_t z4 = kZ4Off, uint32_t byte = kByteOff) {
  const uint32_t w[4] = {ch.x, ch.y, ch.z, ch.w};
#pragma unroll
  for (int k = 0; k < 4; ++k) {
    const int lo = 4 * k;
    if (q0 <= lo && lo + 4 <= q1) {
      reg = zmap(lds, z4, reg ^ w[k]);
    } else {
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const int pos = lo + i;
        if (pos >= q0 && pos < q1) {
          const uint32_t b = (reg ^ (w[k] >> (8 * i))) & 0xffu;
          reg = lds_u32(lds, byte + (b << 2)) ^ (reg >> 8);
        }
      }
    }
  }
  return reg;
}

// Global (not flat) address space: flat loads would tie the LDS counter to every data load.
// Streamed payload is read once: non-temporal loads (kNT) keep it from displacing anything useful and
// measured 6.2 -> 7.0 TB/s on this access pattern (kv-separate_amd/tools/hbm_probe.hip).
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef const __attribute__((address_space(1))) u32x4 gu32x4;
template <bool kNT = false>
__device__ __forceinline__ uint4 ld16(uintptr_t addr) {
  gu32x4* g = reinterpret_cast<gu32x4*>(addr);
  u32x4 v;
  if constexpr (kNT) v = __builtin_nontemporal_load(g);
  else v = *g;
  return make_uint4(v.x, v.y, v.z, v.w);
}

// A work item's loads, issued ahead of its compute so a wave can overlap the next item's HBM latency
// with the current item's serial lane merge.  All fields are wave-uniform except the vectors.
template <int kG>
struct Staged {
  uintptr_t ps, pe, hbase, h0, a1, seg;
  uint64_t K;     // body rows (0 = no body); the last row ends at ar (kAlign) or a1
  uint4 hc, tc;   // aligned 16 B around the head / the tail
  uint4 v;        // row 0; lanes with v_ok == false (front mask) use zeros instead
  uint4 A[kG];    // rows 1 .. kG (clamped to the last row)
  uint4 et;       // kAlign: the m full 16-B chunks [ar, a1) in lanes 8-m .. 7
  uint32_t m;     // kAlign: (a1 - ar) / 16, 0..7
  uintptr_t dummy;  // a valid, cache-resident device address for loads whose data is never used
  bool v_ok;
};

// Issues a FIXED set of 3 + kG loads whatever the geometry (unneeded ones read `dummy`, a valid
// device address), so the compiler can wait for exactly this item's loads with a counted vmcnt
// while the next item's loads stay in flight; masking is deferred to finish().
// kAlign: the rows end at ar = a1 rounded down to 128 B (never below h0), so every row is exactly eight 128-B
// lines and no line is requested by two rows; the m < 8 whole 16-B chunks between ar and a1 are one extra load
// (lanes 8-m .. 7) folded by a 3-level lane tree in finish().
// kPad (round 4, the shipped form): no serial head -- the body starts at the 16-B boundary at or below ps, the bytes
// before ps are zeroed in that first chunk, and the item's register enters there already rewound over them
// (x^-8k, fill_set).  A short item's head was a chain of up to 6 dependent LDS lookups ahead of its first fold.
template <int kG, bool kNT, bool kAlign = false, bool kPad = false>
__device__ __forceinline__ void stage(Staged<kG>& s, uintptr_t ps, uintptr_t pe, uint32_t lane, uintptr_t dummy,
                                      uint32_t vz) {
  s.ps = ps;
  s.pe = pe;
  s.dummy = dummy;
  s.hbase = ps & ~uintptr_t(15);
  s.h0 = kPad && ps < pe ? s.hbase : (ps + 15) & ~uintptr_t(15);
  if (s.h0 > pe) s.h0 = pe;
  s.a1 = pe & ~uintptr_t(15);
  if (s.a1 < s.h0) s.a1 = s.h0;
  uintptr_t ar = s.a1;
  if (kAlign) {
    ar = s.a1 & ~uintptr_t(127);
    if (ar < s.h0) ar = s.h0;
    s.m = uint32_t(s.a1 - ar) >> 4;
    const bool in = lane < 8 && lane + s.m >= 8;
    s.et = ld16((in ? s.a1 - 128 + uintptr_t(lane) * 16u : dummy) + vz);
  }
  s.K = ar > s.h0 ? (uint64_t(ar - s.h0) + kRowBytes - 1) / kRowBytes : 0;
  s.seg = ar - s.K * kRowBytes + uintptr_t(lane) * 16u;
  s.v_ok = s.K && s.seg >= s.h0;  // row 0 is front-masked: lanes before h0 hold zeros
  // Head and tail chunks are wave-uniform, but their addresses are offset by the opaque zero `vz` so the
  // compiler keeps them in VGPRs: a provably uniform load result is moved to SGPRs with readfirstlane
  // right here, which waits (vmcnt) for the NEXT item's first load inside the current item -- a full HBM
  // latency per item.  finish() reads them out after this item's own wait instead.
  s.hc = ld16((ps < s.h0 ? s.hbase : dummy) + vz);  // aligned 16 B holding the head (never crosses a page)
  s.tc = ld16((s.a1 < pe ? s.a1 : dummy) + vz);     // aligned 16 B holding the tail
  s.v = ld16<kNT>(s.v_ok ? s.seg : dummy);
  const uint64_t last = s.K > 1 ? s.K - 1 : 0;
#pragma unroll
  for (int i = 0; i < kG; ++i)
    s.A[i] = ld16<kNT>(last ? s.seg + (1 + i < last ? 1 + i : last) * kRowBytes : dummy);
}

// The 16-B chunk with its bytes [0, k) zeroed (k < 16).
__device__ __forceinline__ uint4 mask_low(uint4 c, uint32_t k) {
  auto m = [k](int d) -> uint32_t {
    const int lo = int(k) - 4 * d;
    return lo <= 0 ? ~0u : lo >= 4 ? 0u : (~0u << (8 * lo));
  };
  return make_uint4(c.x & m(0), c.y & m(1), c.z & m(2), c.w & m(3));
}

// The steps of the kernel templates below that the KVSEP_DIAG tools build replaces in its A/B forms and ablations
// (crc32c_diag.inc: other types with these members; the ablations give wrong results by design).  Those types exist only
// in that build: Exact is the only one the shipped library has, so no kernel it can instantiate computes anything but
// CRC-32C.
struct Exact {
  static constexpr bool kPad = true;        // the wide kernel's padded head (stage<kPad>, round 4)
  static constexpr bool kHeadTail = true;   // the wide kernel's serial head / tail bytes
  static constexpr bool kShortcut = false;  // short items run their whole chain (no short_item member needed)
  static constexpr bool kMerge = true;      // the lane merge (no unmerged member needed)
  static constexpr int kTreeLevels = 6;     // the wide kernel's lane tree: 64 lanes
  static constexpr bool kDrain = false;     // the sorted-window kernel drains nothing after a group
  // one stride-chain step c' = w ^ Z_row(c) through the LDS table: the wide kernel's Z_1024 (fold), the narrow kernels'
  // layout Lay (nfold)
  __device__ static __forceinline__ uint32_t fold(const uint8_t* lds, uint32_t c, uint32_t w, uint32_t lc0,
                                                  uint32_t lc1) {
    return fold_step(lds, c, w, lc0, lc1);
  }
  template <typename Lay>
  __device__ static __forceinline__ uint32_t nfold(const uint8_t* lds, uint32_t c, uint32_t w, uint32_t lc0,
                                                   uint32_t lc1) {
    return Lay::fold(lds, c, w, lc0, lc1);
  }
  // the sorted-window kernel's emit / join points (the round-3 bisection's compare variants live in the diag build)
  __device__ static __forceinline__ void sorted_emit(const PiecesArgs&, uint64_t, uint32_t) {}
  __device__ static __forceinline__ void sorted_join(const PiecesArgs&, bool, uint64_t, uint32_t, uint32_t, uint32_t) {}
};

// Raw CRC register after consuming the staged item [ps, pe) from register `reg` (no final inversion).
// kPad: the padded head of stage<kPad>: `reg` is the register at hbase (rewound), the first chunk's bytes before ps
// are zeroed here.
// Rows beyond the staged ones stream kG at a time, the next kG in flight during compute.
//
// `next()` stages the FOLLOWING work item's loads.  It is called once, as late as possible while still ahead
// of this item's last wait: after the last group's row loads are issued (or at once for an item with at most
// kG rows).  So (a) the main row loop runs without the next item's 28 staged VGPRs live -- that headroom
// lets the compiler keep all 16 LDS lookups of a row in flight instead of 2 -- and (b) the next item's
// loads are the most recent ones, so every wait of this item stays a counted vmcnt that leaves them in
// flight across the lane merge.
template <int kG, bool kNT, bool kAlign, bool kPad, typename Ext, typename Next>
__device__ __forceinline__ uint32_t finish(const uint8_t* lds, Staged<kG>& s, uint32_t reg, uint32_t lane,
                                           uint32_t lc0, uint32_t lc1, Next&& next) {
  if constexpr (Ext::kShortcut) {
    if (s.K <= uint64_t(kG)) return Ext::template short_item<kG>(s, reg, next);
  }
  if (s.K) {
    const uint64_t K = s.K, last = K - 1;
    if (Ext::kHeadTail && s.ps < s.h0) reg = serial16(lds, reg, uniform4(s.hc), int(s.ps - s.hbase), int(s.h0 - s.hbase));
    uint4 v = s.v_ok ? s.v : make_uint4(0, 0, 0, 0);
    if (s.seg == s.h0) {  // the head register enters as pending word at h0
      if (kPad) v = mask_low(v, uint32_t(s.ps - s.h0));
      v.x ^= reg;
    }
    uint32_t c0 = v.x, c1 = v.y, c2 = v.z, c3 = v.w;

#define KVSEP_ROW(V)                                  \
  do {                                                \
    c0 = Ext::fold(lds, c0, (V).x, lc0, lc1);         \
    c1 = Ext::fold(lds, c1, (V).y, lc0, lc1);         \
    c2 = Ext::fold(lds, c2, (V).z, lc0, lc1);         \
    c3 = Ext::fold(lds, c3, (V).w, lc0, lc1);         \
  } while (0)
// The group's loads go out before any of its compute: the scheduler would otherwise sink them below the
// first row's lookups and shorten the time they are in flight (the loop is HBM-latency bound).
#define KVSEP_LOADB(NR, CLAMP)                                                                   \
  do {                                                                                           \
    _Pragma("unroll") for (int i = 0; i < kG; ++i)                                               \
      B[i] = ld16<kNT>(s.seg + (!(CLAMP) || (NR) + i < last ? (NR) + i : last) * kRowBytes);     \
    __builtin_amdgcn_sched_barrier(0);                                                           \
  } while (0)

    uint64_t r = 1;
    for (; r + 2 * kG <= K; r += kG) {  // full group in A, another full group after it: no next item yet
      uint4 B[kG];
      KVSEP_LOADB(r + kG, false);  // rows r+kG .. r+2kG-1 <= K-1: no clamp
#pragma unroll
      for (int i = 0; i < kG; ++i) KVSEP_ROW(s.A[i]);
#pragma unroll
      for (int i = 0; i < kG; ++i) s.A[i] = B[i];
    }
    if (r + kG <= K) {  // the last full group: its successor rows load, then the next item stages
      uint4 B[kG];
      KVSEP_LOADB(r + kG, true);
      next();
#pragma unroll
      for (int i = 0; i < kG; ++i) KVSEP_ROW(s.A[i]);
#pragma unroll
      for (int i = 0; i < kG; ++i) s.A[i] = B[i];
      r += kG;
    } else {
      next();
    }
#pragma unroll
    for (int i = 0; i < kG; ++i)  // remainder rows r .. K-1, already in A
      if (r + i < K) KVSEP_ROW(s.A[i]);
#undef KVSEP_LOADB
#undef KVSEP_ROW
    if constexpr (!Ext::kMerge) return Ext::unmerged(c0, c1, c2, c3, lane);
    // lane merge: pending word at (16*lane + 12) of the last row
    uint32_t p = zmap_x(lds, kZ4Off, c0, c1);
    p = zmap_x(lds, kZ4Off, p, c2);
    p = zmap_x(lds, kZ4Off, p, c3);
    // reduction over lanes: at level j the lanes whose low j+1 bits are all ones (64 >> (j+1) of them)
    // pull the pending word of the segment 16*2^j bytes before theirs and carry it forward by 16*2^j.
    // Only those lanes touch LDS (exec-masked), which keeps the non-replicated tree tables' bank
    // conflicts small -- the tree is the LDS hot spot for short blocks.
    // The partner of an active lane l is l - 2^j: DPP row_shr for j < 4 (within a 16-lane row), lane
    // reads for j = 4, 5 -- no ds_bpermute round trips on this latency-bound chain.
#pragma unroll
    for (int j = 0; j < Ext::kTreeLevels; ++j) {
      uint32_t o;
      if (j == 0) {
        o = row_shr<1>(p);
      } else if (j == 1) {
        o = row_shr<2>(p);
      } else if (j == 2) {
        o = row_shr<4>(p);
      } else if (j == 3) {
        o = row_shr<8>(p);
      } else if (j == 4) {  // active lanes 31 and 63 need lanes 15 and 47
        const uint32_t lo = uint32_t(__builtin_amdgcn_readlane(int(p), 15));
        const uint32_t hi = uint32_t(__builtin_amdgcn_readlane(int(p), 47));
        o = lane < 32 ? lo : hi;
      } else {  // active lane 63 needs lane 31
        o = uint32_t(__builtin_amdgcn_readlane(int(p), 31));
      }
      const uint32_t m = (2u << j) - 1u;
      if ((lane & m) == m) p = zmap_x(lds, kTreeOff + 4096u * j, o, p);
    }
    p = uint32_t(__builtin_amdgcn_readlane(int(p), 63));  // pending word at the last row's end - 4 (uniform)
    reg = zmap(lds, kZ4Off, p);                              // register at ar (kAlign) or a1
  } else {
    next();
    if (Ext::kHeadTail && s.ps < s.h0) reg = serial16(lds, reg, uniform4(s.hc), int(s.ps - s.hbase), int(s.h0 - s.hbase));
  }
  if (kAlign && s.m) {
    // the chunks [ar, a1) right-aligned in lanes 8-m .. 7 (zeros before), the register entering at the first one;
    // per lane the STEP4W re-injection, then a 3-level tree over lanes 0..7 (Z_16, Z_32, Z_64): lane 7 ends with
    // the pending word at a1 - 4
    uint4 e = lane < 8 && lane + s.m >= 8 ? s.et : make_uint4(0, 0, 0, 0);
    if (lane + s.m == 8) {
      if (kPad && !s.K) e = mask_low(e, uint32_t(s.ps - s.h0));  // the first chunk (ar == h0)
      e.x ^= reg;
    }
    uint32_t p = zmap_x(lds, kZ4Off, e.x, e.y);
    p = zmap_x(lds, kZ4Off, p, e.z);
    p = zmap_x(lds, kZ4Off, p, e.w);
    {
      const uint32_t o = row_shr<1>(p);
      if ((lane & 1u) == 1u) p = zmap_x(lds, kTreeOff, o, p);
    }
    {
      const uint32_t o = row_shr<2>(p);
      if ((lane & 3u) == 3u) p = zmap_x(lds, kTreeOff + 4096u, o, p);
    }
    {
      const uint32_t o = row_shr<4>(p);
      if ((lane & 7u) == 7u) p = zmap_x(lds, kTreeOff + 8192u, o, p);
    }
    reg = zmap(lds, kZ4Off, uint32_t(__builtin_amdgcn_readlane(int(p), 7)));  // register at a1
  }
  if (Ext::kHeadTail && s.a1 < s.pe) {
    uint4 t = uniform4(s.tc);
    if (kPad && s.a1 == s.h0) t = mask_low(t, uint32_t(s.ps - s.h0));  // no body: the tail chunk is the first
    reg = serial16(lds, reg, t, 0, int(s.pe - s.a1));
  }
  return reg;
}

__device__ __forceinline__ uint32_t mask_crc(uint32_t c) { return ((c >> 15) | (c << 17)) + 0xa282ead8u; }

// a * b mod P in the reflected representation (bit 31 = x^0): carry-less multiply by VALU shifts, no tables.
__device__ __forceinline__ uint32_t gf2_mulmod(uint32_t a, uint32_t b) {
  uint32_t p = 0;
#pragma unroll 8
  for (int i = 31; i >= 0; --i) {
    p ^= (0u - ((a >> i) & 1u)) & b;
    b = (b >> 1) ^ (0x82F63B78u & (0u - (b & 1u)));
  }
  return p;
}

// Z_n(reg): the register advanced over n zero bytes, for any n, = reg * x^(8n) mod P (x2n[k] = x^(2^k) mod P).
// A few thousand VALU operations: only for the rare paths that need an arbitrary shift (gf2.h has the host side).
__device__ uint32_t gf2_shift(const DevTables* tabs, uint32_t reg, uint64_t n) {
  const uint64_t e = n << 3;
  uint32_t p = 0x80000000u;  // x^0
  for (int k = 0; k < 64; ++k)
    if ((e >> k) & 1u) p = gf2_mulmod(tabs->x2n[k], p);
  return gf2_mulmod(p, reg);
}

__device__ __forceinline__ void emit_block(const PiecesArgs& a, uint64_t b, uint32_t crc) { a.out[b] = crc; }

// The verify form's accumulators (PiecesArgs::vacc, u64 words, each group on a 128-B line of its own): [0] the lowest
// mismatching block (~0: none); [1] the final arrival word, (arrivals << 40) | mismatches: every mismatch count ends
// up there, so the count travels with the arrivals; and at [16 (s + 1)] the arrival word of shard s = blockIdx.x
// mod 8 (one shard per XCD: the dispatcher deals workgroups round-robin over the 8 XCDs), used by grids whose
// workgroups arrive together (verify_publish).
constexpr uint32_t kVaccShards = 8, kVaccStride = 16;  // 16 words = 128 B
constexpr unsigned long long kArrive = 1ull << 40, kCountMask = kArrive - 1;

// A workgroup that saw a mismatch waits until its lowest-block post is performed before it arrives (verify_publish);
// a clean workgroup arrives while its last result stores are still in flight.  Atomic against atomic, a completed post
// is all the order needs.  Not __threadfence(): on gfx950 that is an L2 writeback + invalidate (buffer_wbl2 /
// buffer_inv sc1), which at the end of every wave cost 130-170 us per launch (measured).
__device__ __forceinline__ void post_wait() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// The verify form's running verdict of one wave: its lowest mismatching block and its mismatch count, wave-uniform
// (scalar registers).  Round 5: a wave no longer posts each group's mismatches with global atomics as it goes (two
// atomics on one 128-B line per group, and a vmcnt(0) that drained the next group's staged rows): on an image where
// every block is bad that serialised ~16 K atomics on one line and ran 4x the clean call (217 vs 52 us, 65,536 blocks
// of 4 KiB).  The wave keeps its verdict here; the workgroup combines its waves' verdicts at the end and posts once
// (verify_publish / verify_post).
struct VAcc {
  uint64_t best = ~0ull;
  uint32_t cnt = 0;
};

// The verify form fused into the CRC kernels (db/value_log_reader.cc:109-122, table/format.cc:99-106).  Called by the
// whole wave (full EXEC) right after a group's emit: lanes with `mine` hold block b's crc and the stored word `ex`
// they loaded before the next group's staging (so waiting for it never drains those loads).  The compare itself is
// branch-free; the wave ballots the mismatches and only a mismatch enters a wave-uniform branch, which folds the
// lowest mismatching index and the count into the wave's verdict.  A per-lane branch on the compare nested inside the
// emit's divergent branch is what made the round-1 sorted-window kernel miscompute.  The lane's block
// is base + idx (base wave-uniform): one VGPR for the index, not a 64-bit pair.
__device__ __forceinline__ void verify_wave(VAcc& acc, bool mine, uint64_t base, uint32_t idx, uint32_t crc,
                                            uint32_t ex) {
  const uint64_t m = __builtin_amdgcn_ballot_w64(mine && mask_crc(crc) != ex);
  if (m) {  // wave-uniform
    uint32_t best = ~0u;
    for (uint64_t t = m; t; t &= t - 1) {
      const uint32_t il = uint32_t(__builtin_amdgcn_readlane(int(idx), __builtin_ctzll(t)));
      best = il < best ? il : best;
    }
    const uint64_t b = base + best;
    acc.best = b < acc.best ? b : acc.best;
    acc.cnt += uint32_t(__builtin_popcountll(m));
  }
}

// One block checked by a whole wave whose crc and stored word are wave-uniform (the wide kernel, the deferred walk).
__device__ __forceinline__ void verify_uniform(VAcc& acc, uint64_t b, uint32_t crc, uint32_t ex) {
  if (mask_crc(crc) != ex) {  // wave-uniform
    acc.best = b < acc.best ? b : acc.best;
    acc.cnt += 1;
  }
}

// The workgroup's verdict from its waves' (every wave calls it, full EXEC): each wave's lane 0 leaves its verdict in
// the workgroup's LDS slots, a barrier, then wave 0 reads them all.  Only wave 0's return value is the workgroup's.
template <uint32_t kWaves>
__device__ __forceinline__ VAcc verify_gather(const VAcc& acc, uint32_t wave, uint32_t lane) {
  __shared__ unsigned long long v_best[kWaves];
  __shared__ uint32_t v_cnt[kWaves];
  if (lane == 0) {
    v_best[wave] = acc.best;
    v_cnt[wave] = acc.cnt;
  }
  __syncthreads();  // every wave of the workgroup is done with its groups
  VAcc wg;
  if (wave == 0) {
#pragma unroll
    for (uint32_t w = 0; w < kWaves; ++w) {
      const unsigned long long b = v_best[w];
      wg.best = b < wg.best ? b : wg.best;
      wg.cnt += v_cnt[w];
    }
  }
  return wg;
}

// The lane, recomputed (v_mbcnt) rather than kept live from the kernel's start: at the 16-wave kernels' 128-VGPR cap
// one more long-lived VGPR spills.
__device__ __forceinline__ uint32_t lane_id() {
  uint32_t lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  return lane;
}

// One returning device-scope atomic add by lane 0, its old value broadcast (wave-uniform).
__device__ __forceinline__ unsigned long long arrive(unsigned long long* w, unsigned long long v, uint32_t lane) {
  unsigned long long old = 0;
  if (lane == 0) old = atomicAdd(w, v);
  return (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(old >> 32)), 0))) << 32) |
         uint32_t(__builtin_amdgcn_readlane(int(uint32_t(old)), 0));
}

// The end of a publishing verify kernel (the CRC kernel of an unsplit batch, the combine kernel of a split one), every
// workgroup: the workgroup's verdict (verify_gather); if it saw mismatches, wave 0 posts its lowest index (vacc[0],
// and waits for it), then arrives with its count added to the arrival: the last workgroup to arrive copies the verdict
// to the caller's first_bad / nbad and puts the accumulators back in their reset state (~0, 0) for the next call.  So
// a verify call needs no init launch, a clean batch costs its last workgroup one atomic round trip (vacc[0] is read,
// and reset, only when something mismatched), and a batch full of bad blocks one atomicMin per workgroup.
// kShards = 8: the workgroups arrive first on their shard's word and only each shard's last on the final word.  For a
// grid whose workgroups all arrive at once (the combine kernel): 256 arrivals on ONE word queue at ~11-13 ns each
// (MI355X_MICROARCH.md fanin: 3.2-4.5 us; measured +2.7 us on the combine kernel).  The CRC kernels' workgroups end
// over several us (issue-age staircase), so they take one level: one round trip less for the last one.
// `wave`: the wave's index in the workgroup (wave-uniform, an SGPR); the lane is recomputed here (v_mbcnt) rather than
// kept live from the kernel's start: at the 16-wave kernels' 128-VGPR cap one more long-lived VGPR spills.
template <uint32_t kWaves, uint32_t kShards = 1>
__device__ __forceinline__ void verify_publish(const PiecesArgs& a, uint32_t wave, const VAcc& acc) {
  const uint32_t lane = lane_id();
  const VAcc wg = verify_gather<kWaves>(acc, wave, lane);
  if (wave != 0) return;
  if (wg.cnt) {  // wave-uniform: the workgroup's lowest bad block lands before its arrival is counted
    if (lane == 0) atomicMin(a.vacc, (unsigned long long)wg.best);
    post_wait();
  }
  unsigned long long add = kArrive + wg.cnt;  // the count travels with the arrival
  uint32_t arrivals = gridDim.x;  // expected on the final word
  if (kShards > 1) {
    const uint32_t shard = blockIdx.x % kShards;
    unsigned long long* sw = a.vacc + kVaccStride * (1 + shard);
    const unsigned long long o1 = arrive(sw, add, lane);
    if ((o1 >> 40) + 1 != (gridDim.x - shard + kShards - 1) / kShards) return;  // not the shard's last
    if (lane == 0) atomicExch(sw, 0ull);  // the shard word back to its reset state
    add = kArrive + (o1 & kCountMask) + wg.cnt;  // the shard's count: its earlier workgroups' and this one's
    arrivals = gridDim.x < kShards ? gridDim.x : kShards;
  }
  const unsigned long long old = arrive(a.vacc + 1, add, lane);
  if ((old >> 40) + 1 != arrivals || lane != 0) return;  // the last workgroup of all, lane 0
  const unsigned long long nb = (old & kCountMask) + (add & kCountMask);
  atomicExch(a.vacc + 1, 0ull);  // first, so the wait for the swap's result below is a plain vmcnt(0)
  const unsigned long long fb = nb ? atomicExch(a.vacc, ~0ull) : ~0ull;
  *a.first_bad = fb;
  *a.nbad = nb;
}

// The end of a verify CRC kernel that does not publish (the wide kernel of a split batch: the combine kernel after it
// publishes): the workgroup's verdict goes to the accumulators directly -- its lowest bad block and its count on the
// final word, where the combine kernel's arrivals find them (the kernel boundary orders them).
template <uint32_t kWaves>
__device__ __forceinline__ void verify_post(const PiecesArgs& a, uint32_t wave, const VAcc& acc) {
  const uint32_t lane = lane_id();
  const VAcc wg = verify_gather<kWaves>(acc, wave, lane);
  if (wave == 0 && wg.cnt && lane == 0) {
    atomicMin(a.vacc, (unsigned long long)wg.best);
    atomicAdd(a.vacc + 1, (unsigned long long)wg.cnt);
  }
}

// A 32-bit global load (address space 1), for the stored words of the verify form.
__device__ __forceinline__ uint32_t ld32(const uint32_t* p) {
  return *reinterpret_cast<const __attribute__((address_space(1))) uint32_t*>(reinterpret_cast<uintptr_t>(p));
}

#include "crc32c_hooks.inc"  // diagnostic hook points: empty in the shipped library

// LDS image of a CRC workgroup: the replicated fold table `rep` (4 byte-tables) at [0, 128 KiB), then the
// small tables (Z_4, the tree tables, the byte table) as one contiguous run.
struct NoMid {
  __device__ void operator()() const {}
};

// `mid()` runs between the fill's global loads and its LDS stores (pinned there by sched barriers): loads it
// issues are younger than the table loads, so the stores wait for the tables only (a counted vmcnt).
// kNarrowSet: only the small tables the narrow kernel reads -- Z_4, Z_16, Z_32, Z_64 (one 16 KiB run from kZ4Off)
// and the byte table -- not Z_128 .. Z_512 (12 KiB less to load and store per workgroup).
constexpr uint32_t kSmallAll16 = (kLdsBytes - kZ4Off) / 16;                       // uint4 in the small-table run
constexpr uint32_t kSmallNarrow16 = (4 * 4096) / 16 + 1024 / 16;                  // Z_4..Z_64 + byte table
template <bool kNarrowSet>
__device__ __forceinline__ uint32_t small_index(uint32_t q) {  // uint4 index from kZ4Off (same in src and LDS)
  return !kNarrowSet || q < 1024 ? q : (kByteOff - kZ4Off) / 16 + (q - 1024);
}

template <int kThreads = kWgThreads, bool kNarrowSet = false, typename Mid = NoMid>
__device__ __forceinline__ void fill_lds(uint8_t* lds, const uint32_t* rep, const DevTables* tabs, uint32_t tid,
                                         Mid&& mid = Mid()) {
  // Every global load of the fill is issued before the first LDS store: one L2/HBM round trip per
  // workgroup instead of one per loop trip (the fill is a fixed cost of every launch; it dominates
  // small batches, e.g. 4 KiB-block batches of a few MiB).
  constexpr uint32_t kRep = (8192 + kThreads - 1) / kThreads;                           // uint4 stores
  constexpr uint32_t kN16 = kNarrowSet ? kSmallNarrow16 : kSmallAll16;
  constexpr uint32_t kSmall = (kN16 + kThreads - 1) / kThreads;                        // uint4 copies
  uint4* l128 = reinterpret_cast<uint4*>(lds);
  const uint4* src = reinterpret_cast<const uint4*>(&tabs->z4[0][0]);
  uint32_t v[kRep];
  uint4 w[kSmall];
#pragma unroll
  for (uint32_t i = 0; i < kRep; ++i) {
    const uint32_t q = tid + i * kThreads;  // uint4 index in the replicated image
    const uint32_t idx = q * 4, pair = idx >> 14, b = (idx >> 6) & 255u, half = (idx >> 5) & 1u;
    v[i] = q < 8192 ? rep[(2u * pair + half) * 256u + b] : 0u;
  }
#pragma unroll
  for (uint32_t i = 0; i < kSmall; ++i) {
    const uint32_t q = tid + i * kThreads;
    w[i] = q < kN16 ? src[small_index<kNarrowSet>(q)] : make_uint4(0, 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  mid();
  __builtin_amdgcn_sched_barrier(0);
  // 16-B stores: 4 consecutive dwords of the replicated image are 4 copies of one entry
#pragma unroll
  for (uint32_t i = 0; i < kRep; ++i) {
    const uint32_t q = tid + i * kThreads;
    if (q < 8192) l128[q] = make_uint4(v[i], v[i], v[i], v[i]);
  }
#pragma unroll
  for (uint32_t i = 0; i < kSmall; ++i) {
    const uint32_t q = tid + i * kThreads;
    if (q < kN16) l128[kZ4Off / 16 + small_index<kNarrowSet>(q)] = w[i];
  }
}

// LDS layouts of the narrow kernels (template parameter Lay of nfinish and the narrow kernel).
//   LdsFull: the pieces kernel's image (157 KiB; the narrow kernel fills only Z_128 replicated 32x and the small
//     tables it reads): every lookup conflict-free, one workgroup per CU.
//   LdsCompact: 80 KiB, so that two workgroups fit one CU: Z_128 replicated 16x at byte b<<8 | k<<6 | copy<<2
//     (table k, copy = lane % 16), then Z_4 and Z_16 / Z_32 / Z_64; the STEP1 table is read as Z_4's byte-3 table
//     (Z_4(b << 24) = Z_1(b): three of the four zero bytes only shift b down).  Lanes l and l + 16 of a 32-lane
//     LDS group share a copy, so a lookup is a 2-way bank conflict (4 LDS-array cycles per wave-instruction, not 2).
struct LdsFull {
  static constexpr uint32_t kBytes = kLdsBytes, kZ4 = kZ4Off, kTree = kTreeOff, kByte = kByteOff;
  static constexpr bool kCompact = false;
  static __device__ __forceinline__ uint32_t lc0(uint32_t lane) { return (lane & 31u) << 2; }
  static __device__ __forceinline__ uint32_t lc1(uint32_t lane) { return ((lane & 31u) << 2) | 0x10000u; }
  static __device__ __forceinline__ uint32_t fold(const uint8_t* lds, uint32_t c, uint32_t w, uint32_t lc0,
                                                  uint32_t lc1) {
    return fold_step(lds, c, w, lc0, lc1);
  }
};
struct LdsCompact {
  static constexpr uint32_t kBytes = 81920, kZ4 = 65536, kTree = 65536 + 4096, kByte = 65536 + 3072;
  static constexpr bool kCompact = true;
  static __device__ __forceinline__ uint32_t lc0(uint32_t lane) { return (lane & 15u) << 2; }
  static __device__ __forceinline__ uint32_t lc1(uint32_t) { return 0; }
  static __device__ __forceinline__ uint32_t fold(const uint8_t* lds, uint32_t c, uint32_t w, uint32_t lc0,
                                                  uint32_t) {
    // v_perm_b32: byte0 = lc0.byte0 (copy*4), byte1 = c.byte k, bytes 2-3 zero; table k by the immediate offset
    const uint32_t a0 = __builtin_amdgcn_perm(c, lc0, 0x0C0C0400u);
    const uint32_t a1 = __builtin_amdgcn_perm(c, lc0, 0x0C0C0500u);
    const uint32_t a2 = __builtin_amdgcn_perm(c, lc0, 0x0C0C0600u);
    const uint32_t a3 = __builtin_amdgcn_perm(c, lc0, 0x0C0C0700u);
    return xor3(xor3(lds_u32(lds, a0), lds_u32(lds, a1 + 64u), w), lds_u32(lds, a2 + 128u), lds_u32(lds, a3 + 192u));
  }
};
static_assert(LdsCompact::kTree + 3 * 4096 == LdsCompact::kBytes, "compact narrow image");

// The compact image's fill (LdsCompact): 4096 16-B stores of the replicated Z_128 and the 16 KiB run Z_4, Z_16,
// Z_32, Z_64 (contiguous in DevTables from z4).  All loads before the first store, `mid()` between (see fill_lds).
template <int kThreads, typename Mid = NoMid>
__device__ __forceinline__ void fill_lds_compact(uint8_t* lds, const uint32_t* rep, const DevTables* tabs,
                                                 uint32_t tid, Mid&& mid = Mid()) {
  constexpr uint32_t kRep = (4096 + kThreads - 1) / kThreads;
  constexpr uint32_t kN16 = 4 * 4096 / 16;
  constexpr uint32_t kSmall = (kN16 + kThreads - 1) / kThreads;
  uint4* l128 = reinterpret_cast<uint4*>(lds);
  const uint4* src = reinterpret_cast<const uint4*>(&tabs->z4[0][0]);
  uint32_t v[kRep];
  uint4 w[kSmall];
#pragma unroll
  for (uint32_t i = 0; i < kRep; ++i) {
    const uint32_t q = tid + i * kThreads;  // bytes 16q .. 16q+15 = b<<8 | k<<6 | 4 copies
    v[i] = q < 4096 ? rep[((q >> 2) & 3u) * 256u + (q >> 4)] : 0u;
  }
#pragma unroll
  for (uint32_t i = 0; i < kSmall; ++i) {
    const uint32_t q = tid + i * kThreads;
    w[i] = q < kN16 ? src[q] : make_uint4(0, 0, 0, 0);
  }
  __builtin_amdgcn_sched_barrier(0);
  mid();
  __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (uint32_t i = 0; i < kRep; ++i) {
    const uint32_t q = tid + i * kThreads;
    if (q < 4096) l128[q] = make_uint4(v[i], v[i], v[i], v[i]);
  }
#pragma unroll
  for (uint32_t i = 0; i < kSmall; ++i) {
    const uint32_t q = tid + i * kThreads;
    if (q < kN16) l128[LdsCompact::kZ4 / 16 + q] = w[i];
  }
}

// kThreads: 512 (8 waves, 2 per SIMD, <= 256 VGPRs; the default), 768, 1024 or 256 for A/B (launch_pieces_v).
// One workgroup per CU in every case (the LDS image is 157 KiB).
// kVerify: the verify form -- each whole block this kernel emits is checked against a.expect (verify_uniform); the
// pieces of split blocks are checked by the combine kernel, which produces their CRC.
// Ext: Exact (the shipped steps; the KVSEP_DIAG build's other types, crc32c_diag.inc, are its A/B forms and ablations).
template <bool kPlanned, bool kDynamic, int kG, bool kNT, bool kAhead, int kThreads = kWgThreads, bool kAlign = true,
          bool kVerify = false, typename Ext = Exact>
__global__ void __launch_bounds__(kThreads) crc32c_pieces_kernel(PiecesArgs a) {
  constexpr uint32_t kWavesPerWg = kThreads / 64;
  // the padded head (stage<kPad>); diag variant 26 keeps the serial head of rounds 1-3 for A/B: measured 3a -0.8 /
  // -1.8 %, config 4 -0.1 / -0.2 %, 3b and config 4's short blocks equal, in one process on two boxes
  // (profiles/round4/pad_variant/)
  constexpr bool kPad = Ext::kPad;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  const uint32_t tid = threadIdx.x;
  KVSEP_WSTAMP_ENTRY();  // stamp hooks (crc32c_hooks.inc): empty in the shipped library
  const uint32_t lane = tid & 63u;
  uint32_t vz;  // 0, opaque to the uniformity analysis (see stage())
  asm volatile("v_mov_b32 %0, 0" : "=v"(vz));
  const uint32_t lc0 = (lane & 31u) << 2;
  const uint32_t lc1 = lc0 | 0x10000u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t nwaves = uint64_t(gridDim.x) * kWavesPerWg;

  uint64_t total = a.count;
  bool planned = kPlanned;
  if (kPlanned) {
    total = ldc(a.pstart, a.count);
    // More pieces than scratch (the caller under-stated total_bytes): do not split at all -- one work
    // item per block is slower for long blocks but exact; the combine kernel then skips every block.
    if (total > a.max_pieces) {
      planned = false;
      total = a.count;
    }
  }

  // Work distribution.  Static: wave w owns the run [w*per, (w+1)*per) (or round-robin single items).
  // Dynamic ("guided"): a wave grabs a run of max(1, remaining / (d * nwaves)) consecutive items with
  // ONE atomic, so early runs are long and the tail is single items -- far below the ~88 dequeues/us a
  // single counter serves.  d = clamp(total / (64 * nwaves), 4, 32): the first runs are one 64-item descriptor
  // window.  Measured in one process (diag variants 14-21): d = 4 is best for 128 KiB pieces of 1 MiB blocks
  // (3a, 3b: d = 8 -1.4 %, 16 -2 %, 32 -4 %; d = 1 or 2 -4 to -8 %), while the Zipf batch (2.1 M items, a third
  // of them tiny) gains 1.8-2.2 % at d = 16 over d = 4: its item counts say little about bytes, and shorter
  // runs keep the tail balanced.  The adaptive d is 4 for 3a/3b and 16 for config 4.  Prefetching the next
  // window's descriptors and the next run's grab a run ahead (so the item stream never drains at a boundary)
  // was 3.6-8 % SLOWER: the boundaries are not where the time goes, the spread of the waves over the batch is.
  uint64_t lo = ~uint64_t(0), hi = 0;
  uint64_t seen = 0;  // dynamic: counter value this wave last observed
  uint64_t gdiv = a.guided_div;
  if (!gdiv) {
    gdiv = total / (64 * nwaves);
    gdiv = gdiv < 4 ? 4 : gdiv > 32 ? 32 : gdiv;
  }
  auto grab = [&]() -> bool {
    if (kDynamic) {
      const uint64_t rem = total > seen ? total - seen : 0;
      uint64_t c = rem / (gdiv * nwaves);
      if (a.guided_cap && c > a.guided_cap) c = a.guided_cap;
      if (c < 1) c = 1;
      if (c > 0xffffffffull) c = 0xffffffffull;
      uint32_t t = 0;
      if (lane == 0) t = atomicAdd(a.work_counter, uint32_t(c));
      lo = uint32_t(__builtin_amdgcn_readfirstlane(t));
      hi = lo + c < total ? lo + c : total;
      seen = lo + c;
    } else if (a.static_contig) {
      if (lo != ~uint64_t(0)) return false;
      const uint64_t per = (total + nwaves - 1) / nwaves;
      lo = (uint64_t(wave) * gridDim.x + blockIdx.x) * per;  // wave-major: see the narrow kernel
      hi = lo + per < total ? lo + per : total;
    } else {
      lo = (lo == ~uint64_t(0)) ? uint64_t(wave) * gridDim.x + blockIdx.x : lo + nwaves;
      hi = lo + 1;
    }
    return lo < total;
  };

  // Descriptor window: lane i resolves item w0 + i (block, byte range, initial register) with vector
  // loads issued once per 64 items; items are then taken out with readlane.  Keeps dependent
  // first-touch descriptor loads out of the per-item critical path (short blocks).
  uint64_t w0 = 0, wn = 0;        // window [w0, w0 + wn) of the current run
  uintptr_t w_ps = 0, w_pe = 0;   // per lane
  uint32_t w_b = 0, w_reg0 = 0, w_only = 0, w_exp = 0;
  auto fill_set = [&](uint64_t start, uint64_t n, uintptr_t& w_ps, uintptr_t& w_pe, uint32_t& w_b, uint32_t& w_reg0,
                      uint32_t& w_only, uint32_t& w_exp) {
    const uint64_t g = start + lane;
    w_ps = w_pe = 0;
    w_b = w_reg0 = w_only = w_exp = 0;
    if (g < start + n) {
      uint64_t b, rs, re;
      bool first, only;
      if (planned) {
        b = a.pblk[g];
        const uint64_t s0 = a.pstart[b], k = a.pstart[b + 1] - s0, j = g - s0;
        const uint64_t n = a.len[b];
        re = n - (k - 1 - j) * a.piece_bytes;
        rs = j ? n - (k - j) * a.piece_bytes : 0;
        first = (j == 0);
        only = (k == 1);
      } else {
        b = g;
        rs = 0;
        re = a.len[b];
        first = true;
        only = true;
      }
      const uintptr_t blk = reinterpret_cast<uintptr_t>(a.base) + a.off[b];
      w_ps = blk + rs;
      w_pe = blk + re;
      w_b = uint32_t(b);
      w_reg0 = first ? ~(a.init ? a.init[b] : 0u) : 0u;
      if (kPad && w_ps < w_pe && (w_ps & 15u) && w_reg0)  // padded head: the register rewound to hbase
        w_reg0 = gf2_mulmod(a.tabs->xinv[w_ps & 15u], w_reg0);
      w_only = only ? 1u : 0u;
      if (kVerify) w_exp = only ? a.expect[b] : 0u;  // travels with the descriptors, a window ahead of its use
    }
  };
  auto fill = [&](uint64_t start, uint64_t stop) {
    w0 = start;
    const uint64_t left = stop - start;
    wn = left < 64 ? left : 64;
    fill_set(w0, wn, w_ps, w_pe, w_b, w_reg0, w_only, w_exp);
  };
  struct Item {
    uint64_t g, b;
    uint32_t reg0, exp;
    bool only;
  };
  auto take = [&](uint64_t g, Item& it, Staged<kG>& st) {  // item g of the window -> stage its loads
    const uint32_t i = uint32_t(g - w0);
    // readlane returns int: go through uint32_t so nothing is sign-extended into the upper half
    auto rl = [i](uint32_t v) -> uint32_t { return uint32_t(__builtin_amdgcn_readlane(int(v), int(i))); };
    it.g = g;
    it.b = rl(w_b);
    it.reg0 = rl(w_reg0);
    it.only = rl(w_only) != 0;
    it.exp = kVerify ? rl(w_exp) : 0u;
    const uintptr_t ps = (uintptr_t(rl(uint32_t(w_ps >> 32))) << 32) | uintptr_t(rl(uint32_t(w_ps)));
    const uintptr_t pe = (uintptr_t(rl(uint32_t(w_pe >> 32))) << 32) | uintptr_t(rl(uint32_t(w_pe)));
    stage<kG, kNT, kAlign, kPad>(st, ps, pe, lane, reinterpret_cast<uintptr_t>(a.tabs), vz);
  };
  VAcc vacc;  // the verify form's verdict of this wave
  auto emit = [&](const Item& it, uint32_t reg) {
    if (lane == 0) {
      if (it.only) emit_block(a, it.b, ~reg);
      else a.partial[it.g] = reg;
    }
    // lane 0 holds the register: its readlane makes the compare, and the branch on it, wave-uniform
    if (kVerify && it.only) verify_uniform(vacc, it.b, ~uint32_t(__builtin_amdgcn_readlane(int(reg), 0)), it.exp);
  };

  // One item: finish item g (staged in A) while item g+1 is staged into B.  The loop below alternates the
  // roles of the two buffers (ping-pong) instead of copying B into A after each item: such a copy must wait
  // for ALL of B's loads (vmcnt(0)) and would put a full HBM latency back on every item.
  auto step = [&](uint64_t g, uint64_t end, Item& ia, Staged<kG>& A, Item& ib, Staged<kG>& B) {
    const bool hn = g + 1 < end;
    KVSEP_WSTAMP_ITEM_BEGIN();
    // The next item's HBM loads overlap the end of this item's compute (finish() stages them late, see
    // there).  The take is unconditional (the last item re-stages itself): on a path without it, this item's loads would be the most recent ones and the
    // compiler's counted wait (which merges both paths) would drain everything, vmcnt(0), on every item.
    emit(ia, finish<kG, kNT, kAlign, kPad, Ext>(lds, A, ia.reg0, lane, lc0, lc1, [&]() {
           if (kAhead) take(hn ? g + 1 : g, ib, B);
         }));
    KVSEP_WSTAMP_ITEM_END(ia);
    if (!kAhead && hn) take(g + 1, ib, B);
    return hn;
  };

  Item cur, nxt;
  Staged<kG> S, T;
  fill_lds<kThreads>(lds, &a.tabs->z1024[0][0], a.tabs, tid);
  __syncthreads();
  KVSEP_WSTAMP_FILLED();
  while (grab()) {
    for (uint64_t ws = lo; ws < hi; ws += 64) {
      fill(ws, hi);
      const uint64_t end = w0 + wn;
      take(w0, cur, S);
      for (uint64_t g = w0;; g += 2) {
        if (!step(g, end, cur, S, nxt, T)) break;
        if (!step(g + 1, end, nxt, T, cur, S)) break;
      }
    }
  }
  KVSEP_WSTAMP_EXIT();
  if (kVerify && !kPlanned) verify_publish<kWavesPerWg>(a, wave, vacc);
  if (kVerify && kPlanned) verify_post<kWavesPerWg>(a, wave, vacc);  // the combine kernel publishes a split batch's
}

// ------------------------------------------------------------------------------------------------
// Narrow kernel for batches of many short blocks (use_narrow): a wavefront runs 8 blocks at once,
// kNarrowLanes = 8 lanes ("a slot") per block and rows of 128 B on the 128-B address grid (see nstage).  The wide
// kernel pays a fixed cost per block (lane merge, 6-level lane tree, staging: ~230 of its ~313 VALU
// instructions for a 4 KiB block, PMC SQ_INSTS_VALU); here the merge is a 3-level tree inside the slot and
// staging is shared by the 8 blocks, so the cost per block is mostly the fold itself.  The chain fold uses
// the same replicated-table lookup as the wide kernel, with Z_128 (16 B per lane x 8 lanes) in place of
// Z_1024.  All geometry is per lane (divergent across slots); every load instruction still reads whole
// 128-B lines, one per slot.
constexpr int kNarrowLanes = 8;
constexpr uint32_t kNarrowRow = 16u * kNarrowLanes;
constexpr uint64_t kNarrowMax = 32 * 1024;  // longest block the narrow kernel is ever chosen for (use_narrow)

template <int kG>
struct NStaged {
  uintptr_t ps, seg;  // this lane's slot item [ps, ps + len); its 16-B chunk of row 0
  uint32_t len;       // < 2^31: <= the hint (<= 64 KiB) on the main path, <= 1 GiB parts on the deferred one
  uint32_t K;         // body rows of the slot item
  uint4 hc, tc, v;
  uint4 A[kG];            // rows 1 .. kG (clamped to the last row)
};

// kAlign: a slot's rows end at ar = a1 rounded down to 128 B (never below h0), so every slot row is one whole
// 128-B line; the m < 8 whole chunks [ar, a1) come in with the tail load: lane j loads a1 - 112 + 16 j, i.e.
// lanes 7-m .. 6 hold those chunks and lane 7 the partial tail chunk at a1 (the old tc) -- no extra load, no
// extra registers.  Without it a block at a 16-B but not 128-B aligned address reads two half lines per row
// (SST blocks in a file image: 20 % slower).
// The slot geometry in 32-bit offsets from the 128-B line holding ps (len < 2^31, so nothing wraps): P = ps's
// offset in that line, E = the end, h0 / a1 = the first / last 16-B boundary inside [P, E] (clamped), ar = where
// the rows end.  64-bit address arithmetic only for the loads.
struct NGeo {
  uint32_t P, E, h0, a1, ar;
};
template <bool kAlign, int kL = kNarrowLanes>
__device__ __forceinline__ NGeo ngeo(uintptr_t ps, uint32_t len) {
  constexpr uint32_t kRow = 16u * kL;
  NGeo g;
  g.P = uint32_t(ps) & (kRow - 1);
  g.E = g.P + len;
  g.h0 = (g.P + 15u) & ~15u;
  if (g.h0 > g.E) g.h0 = g.E;
  g.a1 = g.E & ~15u;
  if (g.a1 < g.h0) g.a1 = g.h0;
  g.ar = g.a1;
  if (kAlign) {
    g.ar = g.a1 & ~(kRow - 1);
    if (g.ar < g.h0) g.ar = g.h0;
  }
  return g;
}

template <int kG, bool kNT, bool kAlign = true, int kL = kNarrowLanes>
__device__ __forceinline__ void nstage(NStaged<kG>& s, uintptr_t ps, uint32_t len, uint32_t j, uintptr_t dummy) {
  constexpr uint32_t kRow = 16u * kL;
  s.ps = ps;
  s.len = len;
  const NGeo g = ngeo<kAlign, kL>(ps, len);
  const uintptr_t line = ps - g.P;
  s.K = (g.ar - g.h0 + kRow - 1) / kRow;
  const int32_t rel0 = int32_t(g.ar - s.K * kRow + j * 16u);  // row 0's chunk, may start before the line
  s.seg = line + intptr_t(rel0);
  const bool v_ok = s.K && rel0 >= int32_t(g.h0);
  s.hc = ld16(g.P < g.h0 ? line + (g.P & ~15u) : dummy);
  if (kAlign) {
    const uint32_t m = (g.a1 - g.ar) >> 4;
    s.tc = ld16((j == kL - 1 ? g.a1 < g.E : j + m >= kL - 1) ? line + (g.a1 - (kRow - 16u) + j * 16u) : dummy);
  } else {
    s.tc = ld16(g.a1 < g.E ? line + g.a1 : dummy);
  }
  s.v = ld16<kNT>(v_ok ? s.seg : dummy);
  const uint32_t last = s.K > 1 ? s.K - 1 : 0;
#pragma unroll
  for (int i = 0; i < kG; ++i)
    s.A[i] = ld16<kNT>(last ? s.seg + uintptr_t(1 + i < int(last) ? 1 + i : last) * kRow : dummy);
}

// Raw register after the slot item, valid in the slot's last lane (j == 7).  kmin / kmax: wave min / max of K.
// `next()` stages the following group, after this group's last row loads (see the wide kernel's finish()).
// kL: lanes per slot, 8 (Z_128 rows, a 3-level slot tree) or 16 (diag: Z_256 rows, 4 levels; LdsFull only).
template <int kG, bool kNT, bool kAlign = true, typename Lay = LdsFull, int kL = kNarrowLanes, typename Ext = Exact,
          typename Next>
__device__ __forceinline__ uint32_t nfinish(const uint8_t* lds, NStaged<kG>& s, uint32_t reg, uint32_t j,
                                            uint32_t lc0, uint32_t lc1, uint32_t kmin, uint32_t kmax,
                                            uintptr_t dummy, Next&& next) {
  static_assert(kL == 8 || (kL == 16 && !Lay::kCompact), "slots of 8 lanes, or 16 on the full LDS image");
  constexpr uint32_t kRow = 16u * kL;
  const NGeo g = ngeo<kAlign, kL>(s.ps, s.len);
  // what the end needs, packed in one 32-bit value computed here, live across the row loop (at 16 waves the kernel
  // sits at 128 VGPRs): bits 0-3 the bytes after a1, bits 4-6 (kAlign) m, the whole chunks [ar, a1)
  const uint32_t endg = (g.E - g.a1) | (g.a1 - g.ar);
  const int32_t rel0 = int32_t(uint32_t(s.seg) - uint32_t(s.ps) + g.P);  // row 0's chunk from the line (as staged)
  if (!kmax) next();
  if (g.P < g.h0) reg = serial16(lds, reg, s.hc, int(g.P & 15u), int(g.h0 - (g.P & ~15u)), Lay::kZ4, Lay::kByte);
  if (kmax) {
    const uint32_t K = s.K, last = K > 1 ? K - 1 : 0;
    uint4 v = (K && rel0 >= int32_t(g.h0)) ? s.v : make_uint4(0, 0, 0, 0);
    if (K && rel0 == int32_t(g.h0)) v.x ^= reg;  // the head register enters as pending word at h0
    uint32_t c0 = v.x, c1 = v.y, c2 = v.z, c3 = v.w;
    KVSEP_NSTAMP_FIRST_DATA(c0);  // stamp hook (crc32c_hooks.inc): empty in the shipped library
#define KVSEP_NROW(V)                                                 \
  do {                                                                \
    c0 = Ext::template nfold<Lay>(lds, c0, (V).x, lc0, lc1);          \
    c1 = Ext::template nfold<Lay>(lds, c1, (V).y, lc0, lc1);          \
    c2 = Ext::template nfold<Lay>(lds, c2, (V).z, lc0, lc1);          \
    c3 = Ext::template nfold<Lay>(lds, c3, (V).w, lc0, lc1);          \
  } while (0)
    uint32_t r = 1;
    for (; r + 2 * kG <= kmin; r += kG) {  // every slot has rows r .. r+2kG-1: no guards, no clamps
      uint4 B[kG];
#pragma unroll
      for (int i = 0; i < kG; ++i) B[i] = ld16<kNT>(s.seg + uintptr_t(r + kG + i) * kRow);
      __builtin_amdgcn_sched_barrier(0);  // loads go out before the group's compute
#pragma unroll
      for (int i = 0; i < kG; ++i) KVSEP_NROW(s.A[i]);
#pragma unroll
      for (int i = 0; i < kG; ++i) s.A[i] = B[i];
    }
    for (; r + kG <= kmax; r += kG) {  // ragged end: per-lane clamps and guards
      uint4 B[kG];
      const uint32_t nr = r + kG;
#pragma unroll
      for (int i = 0; i < kG; ++i)
        B[i] = ld16<kNT>(last ? s.seg + uintptr_t(nr + i < last ? nr + i : last) * kRow : dummy);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int i = 0; i < kG; ++i)
        if (r + i < K) KVSEP_NROW(s.A[i]);
#pragma unroll
      for (int i = 0; i < kG; ++i) s.A[i] = B[i];
    }
    next();
#pragma unroll
    for (int i = 0; i < kG; ++i)
      if (r + i < K) KVSEP_NROW(s.A[i]);
#undef KVSEP_NROW
    uint32_t p = zmap_x(lds, Lay::kZ4, c0, c1);
    p = zmap_x(lds, Lay::kZ4, p, c2);
    p = zmap_x(lds, Lay::kZ4, p, c3);
    // 3-level tree inside the slot (lanes 8k .. 8k+7 of one DPP row): Z_16, Z_32, Z_64
    {
      const uint32_t o = row_shr<1>(p);
      if ((j & 1u) == 1u) p = zmap_x(lds, Lay::kTree, o, p);
    }
    {
      const uint32_t o = row_shr<2>(p);
      if ((j & 3u) == 3u) p = zmap_x(lds, Lay::kTree + 4096u, o, p);
    }
    {
      const uint32_t o = row_shr<4>(p);
      if ((j & 7u) == 7u) p = zmap_x(lds, Lay::kTree + 8192u, o, p);
    }
    if (kL == 16) {  // a 16-lane slot is one DPP row: the 4th level (Z_128)
      const uint32_t o = row_shr<8>(p);
      if ((j & 15u) == 15u) p = zmap_x(lds, Lay::kTree + 12288u, o, p);
    }
    if (K) reg = zmap(lds, Lay::kZ4, p);  // lane 7 of the slot: pending word at the rows' end - 4 -> register there
  }
  if (kAlign) {
    const uint32_t m = endg >> 4;
    if (__builtin_amdgcn_ballot_w64(m != 0)) {  // whole chunks [ar, a1) in lanes 7-m .. 6 of the tail load
      // their raw register from 0: per lane the STEP4W re-injection, moved up one lane (chunks in lanes 8-m .. 7),
      // the slot's 3-level tree; then R = Z_16m(register at ar) ^ that (Z_16m from the tree tables by the bits of m)
      const uint4 e = j < kL - 1 && j + m >= kL - 1 ? s.tc : make_uint4(0, 0, 0, 0);
      uint32_t p = zmap_x(lds, Lay::kZ4, e.x, e.y);
      p = zmap_x(lds, Lay::kZ4, p, e.z);
      p = zmap_x(lds, Lay::kZ4, p, e.w);
      p = row_shr<1>(p);  // lane 8k + 7 holds no chunk (its e is zero, so p is zero): slot k+1's lane 0 gets 0
      {
        const uint32_t o = row_shr<1>(p);
        if ((j & 1u) == 1u) p = zmap_x(lds, Lay::kTree, o, p);
      }
      {
        const uint32_t o = row_shr<2>(p);
        if ((j & 3u) == 3u) p = zmap_x(lds, Lay::kTree + 4096u, o, p);
      }
      {
        const uint32_t o = row_shr<4>(p);
        if ((j & 7u) == 7u) p = zmap_x(lds, Lay::kTree + 8192u, o, p);
      }
      if (kL == 16) {
        const uint32_t o = row_shr<8>(p);
        if ((j & 15u) == 15u) p = zmap_x(lds, Lay::kTree + 12288u, o, p);
      }
      if (m & 1u) reg = zmap(lds, Lay::kTree, reg);
      if (m & 2u) reg = zmap(lds, Lay::kTree + 4096u, reg);
      if (m & 4u) reg = zmap(lds, Lay::kTree + 8192u, reg);
      if (kL == 16 && (m & 8u)) reg = zmap(lds, Lay::kTree + 12288u, reg);
      reg ^= zmap(lds, Lay::kZ4, p);  // lane 7: register at a1
    }
  }
  if (endg & 15u) reg = serial16(lds, reg, s.tc, 0, int(endg & 15u), Lay::kZ4, Lay::kByte);  // lane 7's tail load is the chunk at a1
  return reg;
}

// Blocks longer than the narrow kernel's hint (a.hint), skipped by the main pass: the wave walks its run
// [lo, hi) again and checksums those blocks one at a time, each cut into parts of <= 1 GiB, 8 at a time (one per
// slot; the slot geometry is 32-bit), merged with R(A||B) = Z_|B|(R(A)) ^ R(B) through gf2_shift.  Slower than the
// main path (long blocks are not what the narrow kernels are for) but exact for any 64-bit length.
template <int kG, bool kNT, bool kAlignN, typename Lay = LdsFull, bool kVerify = false, int kL = kNarrowLanes>
__device__ __forceinline__ void narrow_deferred(const PiecesArgs& a, const uint8_t* lds, uint64_t lo, uint64_t hi,
                                                uintptr_t dummy, VAcc& vacc) {
  constexpr uint32_t kPerGroup = 64 / kL;
  // The lane constants are recomputed here (volatile, so not merged with the kernel's own): values kept live across
  // the main group loop for this rarely taken walk would cost registers at the 16-wave kernels' 128-VGPR cap.
  uint32_t lane;
  asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(lane));
  const uint32_t lc0 = Lay::lc0(lane), lc1 = Lay::lc1(lane);
  const uint32_t j = lane & (kL - 1);
  const uint32_t slot = lane / kL;
  const uint32_t hint32 = uint32_t(a.hint);
  struct Desc {
    uint64_t off;
    uint32_t len, lenhi, init;
  };
  auto load_desc = [&](uint64_t g, Desc& d) {
    const uint64_t b = g + slot;
    const uint64_t bb = b < hi ? b : hi - 1;
    d.off = a.off[bb];
    const uint2 l = *reinterpret_cast<const uint2*>(a.len + bb);
    d.len = l.x;
    d.lenhi = l.y;
    d.init = *(a.init ? a.init + bb : &a.tabs->z4[0][0]);
  };
  {
    for (uint64_t g = lo; g < hi; g += kPerGroup) {
      Desc d;
      load_desc(g, d);
      uint64_t over = __builtin_amdgcn_ballot_w64(g + slot < hi && (d.lenhi != 0 || d.len > hint32));
      while (over) {
        const uint32_t k = uint32_t(__builtin_ctzll(over)) / kL;  // slot of the next deferred block
        over &= ~(((1ull << kL) - 1) << (k * kL));
        const uint32_t src = k * kL;
        const uint64_t boff = (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(uint32_t(d.off >> 32)), int(src)))) << 32) |
                              uint32_t(__builtin_amdgcn_readlane(int(uint32_t(d.off)), int(src)));
        const uint64_t L = (uint64_t(uint32_t(__builtin_amdgcn_readlane(int(d.lenhi), int(src)))) << 32) |
                           uint32_t(__builtin_amdgcn_readlane(int(d.len), int(src)));
        const uint32_t binit = uint32_t(__builtin_amdgcn_readlane(int(d.init), int(src)));
        // parts of q <= 1 GiB bytes (the slot geometry is 32-bit), 8 at a time, one per slot; part p's raw register
        // (from ~init for part 0, from 0 for the others) is carried to the block's end and the parts XORed
        uint64_t q = (L + kPerGroup - 1) / kPerGroup;
        if (q > (1ull << 30)) q = 1ull << 30;
        const uint64_t nparts = (L + q - 1) / q;
        const uintptr_t blk = reinterpret_cast<uintptr_t>(a.base) + boff;
        uint32_t acc = 0;
        for (uint64_t p0 = 0; p0 < nparts; p0 += kPerGroup) {
          const uint64_t p = p0 + slot;
          const uint64_t rs = p < nparts ? p * q : L;
          const uint64_t re = rs + q < L ? rs + q : L;
          NStaged<kG> X;
          nstage<kG, kNT, kAlignN, kL>(X, blk + rs, uint32_t(re - rs), j, dummy);
          uint32_t km = 0, kn = ~0u;
#pragma unroll
          for (uint32_t t = 0; t < kPerGroup; ++t) {
            const uint32_t kk = uint32_t(__builtin_amdgcn_readlane(int(X.K), int(t * kL)));
            km = km > kk ? km : kk;
            kn = kn < kk ? kn : kk;
          }
          uint32_t reg = nfinish<kG, kNT, kAlignN, Lay, kL>(lds, X, p == 0 ? ~binit : 0u, j, lc0, lc1, kn, km, dummy,
                                                         NoMid());
          if (j == kL - 1) reg = gf2_shift(a.tabs, reg, L - re);  // carried to the block's end
#pragma unroll
          for (uint32_t t = 0; t < kPerGroup; ++t)
            acc ^= uint32_t(__builtin_amdgcn_readlane(int(reg), int(t * kL + kL - 1)));
        }
        if (lane == 0) emit_block(a, g + k, ~acc);
        // acc is wave-uniform (a readlane sum); so is the stored word, read through readfirstlane
        if (kVerify) verify_uniform(vacc, g + k, ~acc, uint32_t(__builtin_amdgcn_readfirstlane(int(ld32(a.expect + g + k)))));
      }
    }
  }
}

// Unsplit batches only (every block <= 64 KiB <= piece_bytes); static contiguous runs of 8-block groups.
// Lay: the LDS layout (LdsFull: one workgroup per CU; LdsCompact: two).  The runs follow gridDim, so a grid of more
// workgroups than fit at once is the same computation (the hardware dispatcher then hands out the runs).
// kVerify: the verify form (verify_wave after each group; the stored words are loaded just before the next group's
// staging).
template <int kG, bool kNT, int kThreads, bool kOverlap = false, bool kAlignN = true, typename Lay = LdsFull,
          bool kVerify = false, typename Ext = Exact>
__global__ void __launch_bounds__(kThreads) crc32c_narrow_kernel(PiecesArgs a) {
  constexpr uint32_t kWavesPerWg = kThreads / 64;
  __shared__ __attribute__((aligned(16))) uint8_t lds[Lay::kBytes];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint32_t j = lane & (kNarrowLanes - 1);
  const uint32_t slot = lane / kNarrowLanes;
  const uint32_t lc0 = Lay::lc0(lane);
  const uint32_t lc1 = Lay::lc1(lane);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t nwaves = uint64_t(gridDim.x) * kWavesPerWg;
  const uintptr_t dummy = reinterpret_cast<uintptr_t>(a.tabs);
  constexpr uint32_t kPerGroup = 64 / kNarrowLanes;

  // contiguous run of whole groups per wave.  Runs are numbered wave-major (run w*grid + b), so when there are
  // fewer groups than waves the busy waves are spread over every CU instead of filling the first CUs.
  const uint64_t groups = (a.count + kPerGroup - 1) / kPerGroup;
  const uint64_t gper = (groups + nwaves - 1) / nwaves;
  const uint64_t lo = (uint64_t(wave) * gridDim.x + blockIdx.x) * gper * kPerGroup;
  uint64_t hi = lo + gper * kPerGroup;
  if (hi > a.count) hi = a.count;

  // Descriptors run one group ahead of the staging: taking group g stages its rows from descriptors loaded
  // when group g-8 was taken, then loads those of group g+8 (each lane its slot's block: one 64-B line per
  // array, shared by the slot's 8 lanes), so no descriptor load sits between two groups' row loads.
  // The raw loaded words are kept and only used at the take, a group later: nothing consumes them right
  // after the loads, so the compiler's wait for them lands at the take, not behind the loads.
  // The kernel is chosen on the caller's max_len hint (<= 32 KiB), but a hint is never trusted for exactness: a
  // block longer than the hint (a.hint) is left out of its group and redone by its wave at the end of the run
  // (`deferred`), with its full 64-bit length.  The staged length stays 32-bit: a 64-bit block end spills at 16
  // waves.
  struct Desc {
    uint64_t off;
    uint32_t len, lenhi, init;
  };
  auto load_desc = [&](uint64_t g, Desc& d) {  // block g + slot; past hi: loads stay in bounds, take() empties it
    // slot through an empty asm: otherwise (g + 16 + slot) becomes a hoisted 64-bit lane constant that, at 128
    // VGPRs, is spilled and reloaded per group with a vmcnt(0) wait that drains the next group's row loads
    uint32_t sl = slot;
    asm volatile("" : "+v"(sl));
    const uint64_t b = g + sl;
    const uint64_t bb = b < hi ? b : hi - 1;
    d.off = a.off[bb];
    const uint2 l = *reinterpret_cast<const uint2*>(a.len + bb);  // one 8-B load, both words consumed at the take
    d.len = l.x;
    d.lenhi = l.y;
    d.init = *(a.init ? a.init + bb : &a.tabs->z4[0][0]);  // no init: a word that is 0 (Z_4 of byte 0)
  };
  struct NItem {  // the slot's block is g + slot (g: the group's first block, wave-uniform)
    uint32_t reg0;
    uint32_t kmin, kmax;
    bool over;  // this lane's block exceeds the hint: skipped here, redone at the end of the run
  };
  Desc dn;  // descriptors of the next group to take
  bool deferred = false;  // wave-uniform: some block of this wave's run exceeded the hint
  VAcc vacc;              // the verify form's verdict of this wave
  const uint32_t hint32 = uint32_t(a.hint);  // <= 64 KiB (use_narrow)
  auto take = [&](uint64_t g, NItem& it, NStaged<kG>& st) {
    const bool in = g + slot < hi;
    const bool over = in && (dn.lenhi != 0 || dn.len > hint32);
    deferred |= __builtin_amdgcn_ballot_w64(over) != 0;
    const bool live = in && !over;
    const uintptr_t ps = live ? reinterpret_cast<uintptr_t>(a.base) + dn.off : dummy;
    it.reg0 = ~dn.init;
    it.over = over;
    nstage<kG, kNT, kAlignN>(st, ps, live ? dn.len : 0u, j, dummy);
    uint32_t km = 0, kn = ~0u;
#pragma unroll
    for (uint32_t k = 0; k < kPerGroup; ++k) {
      const uint32_t kk = uint32_t(__builtin_amdgcn_readlane(int(st.K), int(k * kNarrowLanes)));
      km = km > kk ? km : kk;
      kn = kn < kk ? kn : kk;
    }
    it.kmax = km;
    it.kmin = kn;
  };
  auto step = [&](uint64_t g, NItem& ia, NStaged<kG>& A, NItem& ib, NStaged<kG>& B) {
    const uint64_t gn = g + kPerGroup;
    // the next group is staged inside nfinish, after this group's last row loads; unconditional (past the
    // end it is an empty group of dummy loads: see the wide kernel's step())
    // the verify form: this group's stored words (uniform base + a clamped 32-bit lane offset), issued before the
    // group's remaining row loads and the next group's staging, so their latency hides under the group and the wait
    // for them is a counted vmcnt (see verify_wave)
    uint32_t ex = 0;
    if (kVerify) {
      const uint64_t last = hi - 1 - g;
      ex = ld32(a.expect + g + (slot < last ? slot : uint32_t(last)));
      __builtin_amdgcn_sched_barrier(0);
    }
    const uint32_t reg = nfinish<kG, kNT, kAlignN, Lay, kNarrowLanes, Ext>(lds, A, ia.reg0, j, lc0, lc1, ia.kmin,
                                                                         ia.kmax, dummy, [&]() { take(gn, ib, B); });
    const bool mine = j == kNarrowLanes - 1 && g + slot < hi && !ia.over;
    // compare before the store: a store between the stored word's load and its wait (in a branch the wait must also
    // cover when skipped) would make that wait one count short and hold up the next group's first staged load
    if (kVerify) verify_wave(vacc, mine, g, slot, ~reg, ex);
    if (mine) emit_block(a, g + slot, ~reg);
    load_desc(gn + kPerGroup, dn);  // here, where this group's registers are dead
    return gn < hi;
  };

  NItem cur, nxt;
  NStaged<kG> S, T;
  KVSEP_NSTAMP_ENTRY();  // stamp hooks (crc32c_hooks.inc): empty in the shipped library
  // The first group's descriptors are fetched during the LDS fill.  Staging its rows before the fill as well
  // measured 4-7 % slower on 256 MiB-1 GiB batches of 4 KiB blocks: the fill then waits behind them.
  if (kOverlap) {
    // descriptors, then the table loads, then the first group's rows: the LDS stores wait for the tables
    // only, so the first HBM round trip overlaps the fill.  Unconditional (an idle wave stages an empty
    // group), so the store's wait count is the same on every path.
    load_desc(lo, dn);
    auto mid = [&]() {
      take(lo, cur, S);
      load_desc(lo + kPerGroup, dn);
    };
    if constexpr (Lay::kCompact) fill_lds_compact<kThreads>(lds, &a.tabs->znarrow[0][0], a.tabs, tid, mid);
    else fill_lds<kThreads, true>(lds, &a.tabs->znarrow[0][0], a.tabs, tid, mid);
    __syncthreads();
  } else {
    if (lo < hi) load_desc(lo, dn);
    if constexpr (Lay::kCompact) fill_lds_compact<kThreads>(lds, &a.tabs->znarrow[0][0], a.tabs, tid);
    else fill_lds<kThreads, true>(lds, &a.tabs->znarrow[0][0], a.tabs, tid);
    __syncthreads();
    if (lo < hi) {
      take(lo, cur, S);
      load_desc(lo + kPerGroup, dn);
    }
  }
  KVSEP_NSTAMP(1);
  if (lo < hi) {
    for (uint64_t g = lo;; g += 2 * kPerGroup) {
      const bool more = step(g, cur, S, nxt, T);
      KVSEP_NSTEP();
      if (!more) break;
      const bool more2 = step(g + kPerGroup, nxt, T, cur, S);
      KVSEP_NSTEP();
      if (!more2) break;
    }
  }
  KVSEP_NSTAMP(7);
  if (deferred) narrow_deferred<kG, kNT, kAlignN, Lay, kVerify>(a, lds, lo, hi, dummy, vacc);
  if (kVerify) verify_publish<kWavesPerWg>(a, wave, vacc);
}

// Batches of short blocks up to ~1 GiB (narrow_form 10, round 4): the workgroup owns a contiguous run of 8-block
// groups and deals it to its 8 waves through an LDS claim counter (one ds_add per group: lgkmcnt, never in the rows'
// vmcnt stream), so the waves the memory system serves first take more of the run.  Otherwise the narrow kernel's
// pipeline: a group's rows are staged inside the previous group's finish, and the group after that is claimed and its
// descriptors loaded right after the previous group's emit.  Measured against the shipped forms in one process
// (tools/narrow_variants_probe.py, 4 KiB blocks, graph replay; profiles/round4/queue_variants/): 128 MiB 26.1 vs 28.2
// us, 256 MiB (config 2) 45.3 vs 48.4, 512 MiB 82.5 vs 90.5, 1 GiB 154.6 vs 165.3 -- but 2 GiB 346.8 vs 313.8 and 4 GiB
// 641.8 vs 622.1 (the wave-major runs of the 8-wave narrow kernel stream better there).  The same run dealt round-robin
// with no claims measured within 1 % of the claims: most of the gain is the workgroup-contiguous run itself.  Blocks
// over the hint go to narrow_deferred right after their group (8 waves have the VGPRs for it inline).
// kVerify: the verify form (stored words loaded before each group's remaining rows, verify_wave, verify_publish).
// kOverlap (shipped): the first group's rows are staged between the fill's table loads and its LDS stores, so the
// first HBM round trip runs under the fill (diag variant 59 = without: 4 KiB blocks 128 MiB 25.60 -> 24.84 us, 256 MiB
// 44.75 -> 44.15, 512 MiB 81.83 -> 81.29, 1 GiB 156.09 -> 154.77; profiles/round4/claim_shapes/).
// kL: lanes per slot -- 16 makes a group 4 blocks (Z_256 rows, the tree tables' Z_256 replicated; narrow form 11, see
// claim16_route; diag variant 60 is the same kernel).
template <int kG, int kThreads, bool kVerify = false, bool kOverlap = true, int kL = kNarrowLanes>
__global__ void __launch_bounds__(kThreads) crc32c_narrow_claim_kernel(PiecesArgs a) {
  constexpr uint32_t kWaves = kThreads / 64, kPerGroup = 64 / kL, kNone = 0xffffffffu;
  [[maybe_unused]] constexpr uint32_t kWavesPerWg = kWaves;  // the stamp hooks' name for it
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  __shared__ uint32_t claimed;  // groups of the run claimed after each wave's first (static) one
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint32_t j = lane & (kL - 1);
  const uint32_t slot = lane / kL;
  const uint32_t lc0 = LdsFull::lc0(lane), lc1 = LdsFull::lc1(lane);
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uintptr_t dummy = reinterpret_cast<uintptr_t>(a.tabs);
  const uint64_t count = a.count;
  const uint32_t hint32 = uint32_t(a.hint);  // <= 64 KiB (use_narrow)
  // this workgroup's contiguous run of groups [run0, run1); group indices fit 32 bits (count < 2^32)
  const uint32_t groups = uint32_t((count + kPerGroup - 1) / kPerGroup);
  const uint32_t per_wg = (groups + gridDim.x - 1) / gridDim.x;
  const uint32_t run0 = blockIdx.x * per_wg < groups ? blockIdx.x * per_wg : groups;
  const uint32_t run1 = run0 + per_wg < groups ? run0 + per_wg : groups;
  if (tid == 0) claimed = 0;  // before the fill's barrier; every claim comes after it

  bool ended = false;
  auto next_group = [&]() -> uint32_t {  // claims only after the barrier; none once the run is used up
    if (ended) return kNone;
    uint32_t c = 0;
    if (lane == 0) c = atomicAdd(&claimed, 1u);
    c = uint32_t(__builtin_amdgcn_readfirstlane(int(c)));
    const uint32_t g = run0 + kWaves + c;
    ended = g >= run1;
    return ended ? kNone : g;
  };
  struct Desc {
    uint64_t off;
    uint32_t len, lenhi, init;
  };
  auto load_desc = [&](uint32_t g, Desc& d) {  // past the batch: loads stay in bounds, take() empties the slot
    uint32_t sl = slot;
    asm volatile("" : "+v"(sl));  // see load_desc in crc32c_narrow_kernel
    const uint64_t blk = uint64_t(g) * kPerGroup + sl;
    const bool in = g != kNone && blk < count;
    const uint64_t bb = in ? blk : 0;
    d.off = a.off[bb];
    const uint2 l = *reinterpret_cast<const uint2*>(a.len + bb);
    d.len = l.x;
    d.lenhi = l.y;
    d.init = *(a.init && in ? a.init + bb : &a.tabs->z4[0][0]);  // no init: a word that is 0 (Z_4 of byte 0)
  };
  struct CItem {
    uint32_t g, reg0, kmin, kmax;
    bool over, deferred;
  };
  Desc dn;
  auto take = [&](uint32_t g, CItem& it, NStaged<kG>& st) {
    const uint64_t blk = uint64_t(g) * kPerGroup + slot;
    const bool in = g != kNone && blk < count;
    const bool over = in && (dn.lenhi != 0 || dn.len > hint32);
    it.deferred = __builtin_amdgcn_ballot_w64(over) != 0;
    const bool live = in && !over;
    it.g = g;
    it.over = over;
    it.reg0 = ~dn.init;
    nstage<kG, true, true, kL>(st, live ? reinterpret_cast<uintptr_t>(a.base) + dn.off : dummy, live ? dn.len : 0u, j,
                           dummy);
    uint32_t km = 0, kn = ~0u;
#pragma unroll
    for (uint32_t k = 0; k < kPerGroup; ++k) {
      const uint32_t kk = uint32_t(__builtin_amdgcn_readlane(int(st.K), int(k * kL)));
      km = km > kk ? km : kk;
      kn = kn < kk ? kn : kk;
    }
    it.kmax = km;
    it.kmin = kn;
  };
  uint32_t gn = kNone;  // the group staged next (its descriptors are in dn until its take)
  VAcc vacc;            // the verify form's verdict of this wave
  auto step = [&](CItem& ia, NStaged<kG>& A, CItem& ib, NStaged<kG>& B) -> bool {
    const uint64_t g0 = uint64_t(ia.g) * kPerGroup;
    uint32_t ex = 0;
    if (kVerify) {  // this group's stored words, before its remaining rows (see crc32c_narrow_kernel's step)
      const uint64_t last = count - 1 - g0;
      ex = ld32(a.expect + g0 + (slot < last ? slot : uint32_t(last)));
      __builtin_amdgcn_sched_barrier(0);
    }
    const uint32_t reg = nfinish<kG, true, true, LdsFull, kL>(lds, A, ia.reg0, j, lc0, lc1, ia.kmin, ia.kmax, dummy,
                                                    [&]() { take(gn, ib, B); });
    const bool mine = j == kL - 1 && g0 + slot < count && !ia.over;
    if (kVerify) verify_wave(vacc, mine, g0, slot, ~reg, ex);  // before the store
    if (mine) emit_block(a, g0 + slot, ~reg);
    if (ia.deferred)  // wave-uniform: this group's blocks over the hint, whole
      narrow_deferred<kG, true, true, LdsFull, kVerify, kL>(a, lds, g0, g0 + kPerGroup < count ? g0 + kPerGroup : count,
                                                        dummy, vacc);
    gn = next_group();  // the group after ib: claimed now, its descriptors loaded while ib runs
    load_desc(gn, dn);
    return ib.g != kNone;
  };

  // the wave's first group is static (the wave's slot of the run), its descriptors fetched during the LDS fill
  KVSEP_NSTAMP_ENTRY();  // stamp hooks (crc32c_hooks.inc): empty in the shipped library
  uint32_t g0 = run0 + wave < run1 ? run0 + wave : kNone;
  load_desc(g0, dn);
  CItem cur, nxt;
  NStaged<kG> S, T;
  const uint32_t* rep = kL == 8 ? &a.tabs->znarrow[0][0] : &a.tabs->ztree[4][0][0];  // Z_{16 kL}
  if (kOverlap) {  // unconditional: a wave with no group stages an empty one (the stores' wait count is fixed)
    fill_lds<kThreads, kL == 8>(lds, rep, a.tabs, tid, [&]() { take(g0, cur, S); });
    __syncthreads();
  } else {
    fill_lds<kThreads, kL == 8>(lds, rep, a.tabs, tid);
    __syncthreads();
  }
  KVSEP_NSTAMP(1);
  if (g0 != kNone) {
    if (!kOverlap) take(g0, cur, S);
    gn = next_group();
    load_desc(gn, dn);
    for (;;) {  // (stamps: after each group but a wave's last)
      if (!step(cur, S, nxt, T)) break;
      KVSEP_NSTEP();
      if (!step(nxt, T, cur, S)) break;
      KVSEP_NSTEP();
    }
  }
  KVSEP_NSTAMP(7);
  // two-level arrival: the claims balance the run, so the 256 workgroups end within a µs of each other (bunched, as
  // the combine kernel's do), unlike the other narrow forms' staircase of workgroup ends
  if (kVerify) verify_publish<kWaves, kVaccShards>(a, wave, vacc);
}

// Bitonic sort of one (key, idx) pair per lane over the wavefront, ascending by key (ties by idx, so the two
// lanes of every compare-exchange agree): 21 ds_bpermute stages of two values each.
__device__ __forceinline__ void wave_sort64(uint32_t& key, uint32_t& idx, uint32_t lane) {
  asm volatile("" : "+v"(lane));  // opaque: keeps the 21 stages' lane ^ j addresses from being hoisted as constants
#pragma unroll
  for (uint32_t k = 2; k <= 64; k <<= 1) {
#pragma unroll
    for (uint32_t jj = k >> 1; jj > 0; jj >>= 1) {
      const int addr = int((lane ^ jj) << 2);
      const uint32_t pk = uint32_t(__builtin_amdgcn_ds_bpermute(addr, int(key)));
      const uint32_t pi = uint32_t(__builtin_amdgcn_ds_bpermute(addr, int(idx)));
      const bool up = (lane & k) == 0;  // this lane's bitonic block sorts ascending
      const bool low = (lane & jj) == 0;
      const bool pless = pk < key || (pk == key && pi < idx);
      const bool take = (low == up) ? pless : !pless;  // the low lane of an ascending pair keeps the minimum
      key = take ? pk : key;
      idx = take ? pi : idx;
    }
  }
}

// Ragged batches of short blocks (see launch_batch_in): the narrow kernel's 8-block groups, but formed from 64-block
// windows sorted by length, so a group's 8 blocks are of similar length and its slots do not wait for one long
// block.  Lane i holds the descriptor of block W + i of window W (loaded a window ahead); after the sort, group k's
// slot s takes the block at sorted position 8k + s (two ds_bpermutes to find it, four to fetch its descriptor).
// The rows, the slot tree and the end path are the narrow kernel's (nstage / nfinish); blocks over the hint go to
// narrow_deferred as there.
// Ext::sorted_emit / sorted_join / kDrain: empty in Exact; the KVSEP_DIAG build's types put the round-3 bisection's
// compare variants there (crc32c_diag.inc, tools/sorted_vin_bisect.py).
template <int kG, bool kNT, int kThreads, bool kVerify = false, typename Ext = Exact>
__global__ void __launch_bounds__(kThreads) crc32c_narrow_sorted_kernel(PiecesArgs a) {
  constexpr uint32_t kWavesPerWg = kThreads / 64;
  constexpr uint32_t kPerGroup = 64 / kNarrowLanes;
  __shared__ __attribute__((aligned(16))) uint8_t lds[kLdsBytes];
  const uint32_t tid = threadIdx.x;
  const uint32_t lane = tid & 63u;
  const uint32_t j = lane & (kNarrowLanes - 1);
  const uint32_t slot = lane / kNarrowLanes;
  const uint32_t lc0 = (lane & 31u) << 2;
  const uint32_t lc1 = lc0 | 0x10000u;
  const uint32_t wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const uint64_t nwaves = uint64_t(gridDim.x) * kWavesPerWg;
  const uintptr_t dummy = reinterpret_cast<uintptr_t>(a.tabs);
  const uint64_t groups = (a.count + kPerGroup - 1) / kPerGroup;
  const uint64_t gper = (groups + nwaves - 1) / nwaves;
  const uint64_t lo = (uint64_t(wave) * gridDim.x + blockIdx.x) * gper * kPerGroup;  // wave-major runs
  uint64_t hi = lo + gper * kPerGroup;
  if (hi > a.count) hi = a.count;
  const uint32_t hint32 = uint32_t(a.hint);  // <= 64 KiB (use_narrow)
  // window descriptor of block W + lane; len: the length, kOver (longer than the hint: deferred) or kPast (past hi)
  constexpr uint32_t kOver = 0xffffffffu, kPast = 0xfffffffeu;
  struct WDesc {  // (the initial register is loaded per group, a group ahead of its use: two VGPRs less)
    uint64_t off;
    uint32_t len, idx;  // idx: after the sort, the window lane holding sorted position `lane`
  };
  auto load_win = [&](uint64_t W, WDesc& d) {
    const uint64_t b = W + lane;
    const bool in = b < hi;
    const uint64_t bb = in ? b : hi - 1;
    d.off = a.off[bb];
    const uint2 l = *reinterpret_cast<const uint2*>(a.len + bb);
    d.len = !in ? kPast : (l.y != 0 || l.x > hint32) ? kOver : l.x;
  };
  auto sort_win = [&](WDesc& d) {
    uint32_t key = d.len == kOver ? 0u : d.len;  // deferred blocks are empty in this pass: they sort first
    d.idx = lane;
    wave_sort64(key, d.idx, lane);
  };
  struct NItem {
    uint64_t w;    // window base (wave-uniform)
    uint32_t src;  // this lane's slot's block: w + src
    uint32_t reg0, kmin, kmax;
    bool live;
  };
  bool deferred = false;
  VAcc vacc;  // the verify form's verdict of this wave
  auto take = [&](uint64_t W, const WDesc& d, uint32_t k, NItem& it, NStaged<kG>& st) {
    uint32_t sl = slot;
    asm volatile("" : "+v"(sl));  // see load_desc in crc32c_narrow_kernel
    const uint32_t src = uint32_t(__builtin_amdgcn_ds_bpermute(int((k * kPerGroup + sl) << 2), int(d.idx)));
    const int sa = int(src << 2);
    const uint32_t len = uint32_t(__builtin_amdgcn_ds_bpermute(sa, int(d.len)));
    const uint32_t offl = uint32_t(__builtin_amdgcn_ds_bpermute(sa, int(uint32_t(d.off))));
    const uint32_t offh = uint32_t(__builtin_amdgcn_ds_bpermute(sa, int(uint32_t(d.off >> 32))));
    deferred |= __builtin_amdgcn_ballot_w64(len == kOver) != 0;
    it.live = len < kPast;
    it.w = W;
    it.src = src;
    it.reg0 = ~*(a.init && it.live ? a.init + (W + src) : &a.tabs->z4[0][0]);  // z4[0][0] == 0
    const uintptr_t ps = it.live ? reinterpret_cast<uintptr_t>(a.base) + ((uint64_t(offh) << 32) | offl) : dummy;
    nstage<kG, kNT, true>(st, ps, it.live ? len : 0u, j, dummy);
    uint32_t km = 0, kn = ~0u;
#pragma unroll
    for (uint32_t t = 0; t < kPerGroup; ++t) {
      const uint32_t kk = uint32_t(__builtin_amdgcn_readlane(int(st.K), int(t * kNarrowLanes)));
      km = km > kk ? km : kk;
      kn = kn < kk ? kn : kk;
    }
    it.kmax = km;
    it.kmin = kn;
  };

  auto take_empty = [&](NItem& it, NStaged<kG>& st) {  // past the last group: the same loads, all to `dummy`
    it.live = false;
    it.w = 0;
    it.src = 0;
    it.reg0 = 0;
    uintptr_t d = dummy;
    asm volatile("" : "+s"(d));  // opaque: its loop-invariant addresses would otherwise be hoisted (and spilled)
    nstage<kG, kNT, true>(st, d, 0u, j, dummy);
    it.kmax = it.kmin = 0;
  };

  WDesc cw, nw;
  if (lo < hi) load_win(lo, cw);  // its round trip overlaps the LDS fill
  fill_lds<kThreads, true>(lds, &a.tabs->znarrow[0][0], a.tabs, tid);
  __syncthreads();
  if (lo < hi) {
    uint64_t W = lo, Wn = lo + 64;
    if (Wn < hi) load_win(Wn, nw);
    sort_win(cw);
    auto groups_in = [&](uint64_t w) { return uint32_t(((hi - w < 64 ? hi - w : 64) + kPerGroup - 1) / kPerGroup); };
    uint32_t k = 0, nk = groups_in(W);
    NItem cur, nxt;
    NStaged<kG> S, T;
    take(W, cw, 0, cur, S);
    // finish group k of window W (staged in ia / A) while the next group -- k + 1 of W, or the first group of the
    // next window, sorted right there -- is staged into ib / B
    auto step = [&](NItem& ia, NStaged<kG>& A, NItem& ib, NStaged<kG>& B) -> bool {
      const bool here = k + 1 < nk;
      const bool next_win = !here && Wn < hi;
      // the verify form: this group's stored words, issued before the group's remaining row loads and the next group's
      // staging, from one place on every path (so the wait for them is a counted vmcnt, never a drain; see verify_wave)
      uint32_t ex = 0;
      if (kVerify) {
        ex = ld32(a.expect + ia.w + (ia.live ? ia.src : 0u));
        __builtin_amdgcn_sched_barrier(0);
      }
      const uint32_t reg = nfinish<kG, kNT, true>(lds, A, ia.reg0, j, lc0, lc1, ia.kmin, ia.kmax, dummy, [&]() {
        if (here) {
          take(W, cw, k + 1, ib, B);
        } else if (next_win) {
          sort_win(nw);
          take(Wn, nw, 0, ib, B);
        } else {
          take_empty(ib, B);
        }
      });
      if (kVerify) verify_wave(vacc, j == kNarrowLanes - 1 && ia.live, ia.w, ia.src, ~reg, ex);  // before the store
      if (j == kNarrowLanes - 1 && ia.live) {
        emit_block(a, ia.w + ia.src, ~reg);
        Ext::sorted_emit(a, ia.w + ia.src, reg);
      }
      Ext::sorted_join(a, j == kNarrowLanes - 1 && ia.live, ia.w, ia.src, reg, lane);
      if (Ext::kDrain) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (here) {
        ++k;
        return true;
      }
      if (!next_win) return false;
      cw = nw;
      W = Wn;
      Wn += 64;
      k = 0;
      nk = groups_in(W);
      if (Wn < hi) load_win(Wn, nw);
      return true;
    };
    for (;;) {
      if (!step(cur, S, nxt, T)) break;
      if (!step(nxt, T, cur, S)) break;
    }
  }
  if (deferred) narrow_deferred<kG, kNT, true, LdsFull, kVerify>(a, lds, lo, hi, dummy, vacc);
  if (kVerify) verify_publish<kWavesPerWg>(a, wave, vacc);
}

// One thread per block: Horner over the block's pieces, R <- Z_piece(R) ^ R_piece.  kVerify: also the verify form's
// compare for the split blocks (the CRC kernel checked the whole ones).
template <bool kVerify = false>
__global__ void __launch_bounds__(256) crc32c_combine_kernel(PiecesArgs a) {
  __shared__ uint32_t zp[1024];
  for (uint32_t i = threadIdx.x; i < 1024; i += 256) zp[i] = a.zpiece[i];
  __syncthreads();
  const uint64_t b = uint64_t(blockIdx.x) * 256 + threadIdx.x;
  const uint64_t bb = b < a.count ? b : a.count - 1;
  const uint64_t s = a.pstart[bb], e = a.pstart[bb + 1];
  // unsplit blocks (and the unsplit fallback) were emitted -- and checked -- by the CRC kernel
  const bool mine = b < a.count && e - s > 1 && a.pstart[a.count] <= a.max_pieces;
  uint32_t crc = 0;
  if (mine) {
    uint32_t acc = a.partial[s];
    for (uint64_t g = s + 1; g < e; ++g) {
      acc = zp[acc & 255u] ^ zp[256 + ((acc >> 8) & 255u)] ^ zp[512 + ((acc >> 16) & 255u)] ^ zp[768 + (acc >> 24)];
      acc ^= a.partial[g];
    }
    crc = ~acc;
    emit_block(a, b, crc);
  }
  if (kVerify) {
    VAcc vacc;
    verify_wave(vacc, mine, uint64_t(blockIdx.x) * 256, threadIdx.x, crc, ld32(a.expect + bb));
    verify_publish<4, kVaccShards>(a, threadIdx.x >> 6, vacc);  // after the CRC kernel's whole-block posts
  }
}

__global__ void crc32c_plan_count_kernel(const uint64_t* len, uint64_t count, uint64_t piece_bytes,
                                         uint64_t* counts) {
  const uint64_t b = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= count) return;
  const uint64_t n = len[b];
  // floor, not ceil: piece 0 takes the remainder ON TOP of a full piece (length in [P, 2P)), so no block ends
  // up with a short remainder piece that costs a work item of its own (3b: 33-B pieces, one per record);
  // only the later pieces must be exactly P long for the combine's Z_P.
  counts[b] = n < 2 * piece_bytes ? 1u : n / piece_bytes;
}

// Verify form as a separate pass over the u32 results: only for the A/B variants of the KVSEP_DIAG tools build, whose
// kernels have no fused compare (the shipped kernels compare in place: verify_wave / verify_uniform).  Wave-level
// reduction: one atomicMin / atomicAdd per wave that saw a mismatch.
__global__ void __launch_bounds__(256) verify_finish_kernel(const uint32_t* out, const uint32_t* expect,
                                                            uint64_t count, unsigned long long* first_bad,
                                                            unsigned long long* nbad) {
  const uint64_t b = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  const bool bad = b < count && mask_crc(out[b]) != expect[b];
  const uint64_t m = __builtin_amdgcn_ballot_w64(bad);
  if (!m) return;
  const uint32_t lane = threadIdx.x & 63u;
  if (lane == uint32_t(__builtin_ctzll(m))) {  // the wave's first bad block is its lowest bad index
    atomicMin(first_bad, (unsigned long long)b);
    atomicAdd(nbad, (unsigned long long)__builtin_popcountll(m));
  }
}

// SST write side (table/table_builder.cc:222-225): crc = Extend(Value(block), &type, 1); trailer word = Mask(crc).
__global__ void sst_trailer_finish_kernel(const uint32_t* crc, const uint8_t* types, uint32_t* masked,
                                          uint64_t count, const DevTables* tabs) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= count) return;
  uint32_t l = ~crc[i];
  l = tabs->byte1[(l ^ types[i]) & 0xffu] ^ (l >> 8);  // one STEP1 (util/crc32c.cc:287-292)
  masked[i] = mask_crc(~l);
}

// SST read side (table/format.cc:99-106): the block is followed by [type][Mask(crc) LE32] in the file
// image, so the check is Value(data, n + 1) against the stored word.
__global__ void sst_verify_prep_kernel(const uint8_t* base, const uint64_t* off, const uint64_t* len,
                                       uint64_t* len1, uint32_t* stored, uint64_t count) {
  const uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= count) return;
  const uint8_t* t = base + off[i] + len[i] + 1;
  len1[i] = len[i] + 1;
  stored[i] = uint32_t(t[0]) | (uint32_t(t[1]) << 8) | (uint32_t(t[2]) << 16) | (uint32_t(t[3]) << 24);
}

__global__ void crc32c_plan_expand_kernel(const uint64_t* pstart, uint64_t count, uint64_t max_pieces,
                                          uint32_t* pblk) {
  const uint64_t b = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x;
  if (b >= count) return;
  const uint64_t s = pstart[b], e = pstart[b + 1];
  for (uint64_t g = s; g < e && g < max_pieces; ++g) pblk[g] = uint32_t(b);
}

// ------------------------------------------------------------------------------------------------
// support kernels
__device__ __forceinline__ uint64_t splitmix_word(uint64_t seed, uint64_t j) {
  uint64_t z = seed + (j + 1) * 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

// Fast path: dst 16-B aligned and stream_offset % 16 == 0; each thread writes 16 B per step.
// Non-temporal stores: the data goes to HBM without staying dirty in the caches.  With plain stores the first CRC
// pass over a freshly generated batch ran ~5 % slower than the next ones (round 1's "first-pass effect", which config 5
// paid on every slice it regenerates); with nt stores the first pass runs at the later passes' rate
// (tools/cold_probe.py, profiles/round3/cold_first_pass_nt.log).
__global__ void fill_splitmix_fast_kernel(uint4* dst, uint64_t n16, uint64_t seed, uint64_t w0) {
  typedef unsigned v4u __attribute__((ext_vector_type(4)));
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t lo = splitmix_word(seed, w0 + 2 * i), hi = splitmix_word(seed, w0 + 2 * i + 1);
    const v4u v = {uint32_t(lo), uint32_t(lo >> 32), uint32_t(hi), uint32_t(hi >> 32)};
    __builtin_nontemporal_store(v, reinterpret_cast<__attribute__((address_space(1))) v4u*>(
                                       reinterpret_cast<uintptr_t>(dst + i)));
  }
}

__global__ void fill_splitmix_bytes_kernel(uint8_t* dst, uint64_t n, uint64_t seed, uint64_t so) {
  for (uint64_t i = uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n; i += uint64_t(gridDim.x) * blockDim.x) {
    const uint64_t gpos = so + i;
    dst[i] = uint8_t(splitmix_word(seed, gpos >> 3) >> (8 * (gpos & 7)));
  }
}

// The attainable-read ceiling: the fastest read-only streaming pattern of tools/hbm_probe.hip's sweeps.  Each
// 8-wave workgroup owns a contiguous 1 MiB chunk at a time and its waves read interleaved 1 KiB rows (wave w:
// rows w, w+8, ...), 8 rows in flight per wave, non-temporal loads, one workgroup per CU: 7.17-7.22 TB/s on
// 64 GiB, against 6.9-7.1 for per-wave chunks at 16 rows in flight and 6.3 for plain loads.
constexpr int kStreamRows = 8;
__global__ void __launch_bounds__(512) stream_read_kernel(uintptr_t src, uint64_t n16, uint32_t* sink) {
  const uint32_t lane = threadIdx.x & 63u, w = threadIdx.x >> 6;
  constexpr uint64_t kChunk16 = (1u << 20) / 16;
  constexpr uint64_t kStep = 8 * kStreamRows * kRowBytes;  // bytes per round of the workgroup
  const uint64_t nchunks = n16 / kChunk16;
  uint32_t acc = 0;
  for (uint64_t c = blockIdx.x; c < nchunks; c += gridDim.x) {
    const uintptr_t p = src + c * kChunk16 * 16 + uintptr_t(w) * kRowBytes + lane * 16u;
#pragma unroll 1  // one round at a time: software-pipelining rounds (16 rows in flight) measured 5 % slower
    for (uint64_t r = 0; r < kChunk16 * 16; r += kStep) {
      uint4 v[kStreamRows];
#pragma unroll
      for (int u = 0; u < kStreamRows; ++u) v[u] = ld16<true>(p + r + uint64_t(u) * 8 * kRowBytes);
#pragma unroll
      for (int u = 0; u < kStreamRows; ++u) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
  }
  const uint64_t nthreads = uint64_t(gridDim.x) * blockDim.x;
  for (uint64_t i = nchunks * kChunk16 + uint64_t(blockIdx.x) * blockDim.x + threadIdx.x; i < n16; i += nthreads) {
    const uint4 x = ld16<true>(src + i * 16);
    acc ^= x.x ^ x.y ^ x.z ^ x.w;
  }
  if (acc == 0x9e3779b9u) atomicXor(sink, acc);  // keeps the loads live; practically never stores
}


}  // namespace kvsep

// ================================================================================================
// host side
using namespace kvsep;

struct kvsep_crc32c_ctx {
  int device = 0;
  int num_cus = 0;
  DevTables* d_tabs = nullptr;
  uint64_t piece_bytes = 128 * 1024;  // best of 32 KiB .. 1 MiB on configs 3a/3b/4
  bool piece_auto = true;             // smaller pieces for small batches (piece_for); off once set explicitly
  int dynamic = -1;  // -1 auto, 0 static, 1 guided
  int kernel = 0;    // kvsep_crc32c_ctx_set_kernel: 0 auto (use_narrow), 1 wide only, 2-6 narrow when the hint allows
  uint32_t static_contig = 1;  // static schedule: contiguous runs (1) or round-robin items (0, set_schedule(2))
  Scratch sc;  // scratch of the calls made directly on this context (any stream, event-ordered)
  int host_node = -1;        // NUMA node of the device's PCI function (-1: unknown / not bound): host legs go there
  bool inject_failure = false;  // kvsep_crc32c_ctx_inject_failure: the next call fails right after its CRC kernel
  // timing
  bool timing = false;
  std::vector<std::pair<hipEvent_t, hipEvent_t>> ev_pending;
  std::vector<hipEvent_t> ev_pool;
  // host form
  HostStaging staging;
  std::mutex mu;
};

// The KVSEP_DIAG tools build's kernel variants, their per-context selection and host hooks; in the shipped library the
// hooks are constant-false inline functions (no variant exists, no environment variable is read).
#include "crc32c_diag.inc"

namespace {
thread_local std::string g_last_error;

int set_err(int code, const char* what, hipError_t e = hipSuccess) {
  char buf[512];
  if (e != hipSuccess)
    snprintf(buf, sizeof buf, "%s: %s (%d)", what, hipGetErrorString(e), int(e));
  else
    snprintf(buf, sizeof buf, "%s", what);
  g_last_error = buf;
  return code;
}

#define KVSEP_HIP(call)                                              \
  do {                                                               \
    hipError_t _e = (call);                                          \
    if (_e != hipSuccess) return set_err(KVSEP_EHIP, #call, _e);     \
  } while (0)

int upload_tables(kvsep_crc32c_ctx* c) {
  DevTables h;
  gf2::byte_tables(gf2::zero_bytes_map(1024), &h.z1024[0][0]);
  gf2::byte_tables(gf2::zero_bytes_map(4), &h.z4[0][0]);
  for (int j = 0; j < 6; ++j) gf2::byte_tables(gf2::zero_bytes_map(16ull << j), &h.ztree[j][0][0]);
  for (uint32_t b = 0; b < 256; ++b) h.byte1[b] = gf2::byte_table_entry(b);
  gf2::byte_tables(gf2::zero_bytes_map(c->piece_bytes), &h.zpiece[0][0]);
  for (int k = 0; k < 3; ++k) gf2::byte_tables(gf2::zero_bytes_map(kSmallPiece << k), &h.zsmall[k][0][0]);
  gf2::byte_tables(gf2::zero_bytes_map(kNarrowRow), &h.znarrow[0][0]);
  gf2::x2n_table(h.x2n);
  gf2::xinv_table(h.xinv);
  if (!c->d_tabs) KVSEP_HIP(hipMalloc(&c->d_tabs, sizeof(DevTables)));
  KVSEP_HIP(hipMemcpy(c->d_tabs, &h, sizeof(DevTables), hipMemcpyHostToDevice));
  return KVSEP_OK;
}

void free_plan(Scratch& sc) {
  hipFree(sc.d_counts); hipFree(sc.d_pstart); hipFree(sc.d_pblk); hipFree(sc.d_partial);
  hipFree(sc.d_scan_tmp);
  sc.d_counts = sc.d_pstart = nullptr;
  sc.d_pblk = sc.d_partial = nullptr;
  sc.d_scan_tmp = nullptr;
  sc.cap_count = sc.cap_pieces = 0;
  sc.scan_tmp_bytes = 0;
}

// Wait until the scratch's previous user (on whatever stream) is done with it -- before a realloc.
int quiesce(Scratch& sc) {
  if (sc.used && sc.last_use) KVSEP_HIP(hipEventSynchronize(sc.last_use));
  return KVSEP_OK;
}

// Order this call behind the scratch's previous user when it ran on another stream.
int acquire(Scratch& sc, hipStream_t s) {
  if (!sc.last_use) KVSEP_HIP(hipEventCreateWithFlags(&sc.last_use, hipEventDisableTiming));
  if (sc.used && sc.last_stream != s) KVSEP_HIP(hipStreamWaitEvent(s, sc.last_use, 0));
  return KVSEP_OK;
}

int release(Scratch& sc, hipStream_t s) {
  KVSEP_HIP(hipEventRecord(sc.last_use, s));
  sc.last_stream = s;
  sc.used = true;
  return KVSEP_OK;
}

// The verify form's device words (allocated once per scratch, before any capture -- kvsep_crc32c_reserve does it): on
// the first 128-B line the result words of a call whose caller passes none; then kVaccLines sets of the accumulators
// the kernels post to and reset (PiecesArgs::vacc: the lowest-block word and the final arrival word, then 8 shard
// arrival words, each group on a line of its own), which must start in their reset state: ~0 (no mismatch), 0
// (nothing arrived, none bad).  Set 0 serves eager calls, which the scratch's events order one after another; each
// captured call takes one of the other sets in turn, so replays of up to kVaccLines - 1 captured verify calls may
// overlap (two graphs on two streams) without mixing their arrivals.
constexpr uint32_t kVaccLines = 8, kVaccSetWords = kVaccStride * (1 + kVaccShards);
unsigned long long* vacc_set(Scratch& sc, uint32_t line) { return sc.d_verify + kVaccStride + line * kVaccSetWords; }

int ensure_verify(Scratch& sc) {
  if (sc.d_verify) return KVSEP_OK;
  std::vector<unsigned long long> init(kVaccStride + kVaccLines * kVaccSetWords, 0ull);
  init[0] = ~0ull;  // default first_bad
  for (uint32_t l = 0; l < kVaccLines; ++l) init[kVaccStride + l * kVaccSetWords] = ~0ull;  // each set's vacc[0]
  KVSEP_HIP(hipMalloc(&sc.d_verify, init.size() * 8));
  KVSEP_HIP(hipMemcpy(sc.d_verify, init.data(), init.size() * 8, hipMemcpyHostToDevice));
  sc.vacc_dirty = 0;
  return KVSEP_OK;
}

// Puts accumulator set `line` back in its reset state, in stream order (capturable: two memsets).  Needed after a call
// that failed once its CRC kernel was enqueued: the kernel's posts stay in the set, and with no publishing kernel after
// them nothing resets it -- the next verdict would inherit a stale count and first_bad.  Under capture the
// memsets only become graph nodes that may never run, so the set stays marked (every later captured call on it resets
// it first, at the cost of two memset nodes) until an eager call has reset it.
int reset_vacc(Scratch& sc, uint32_t line, hipStream_t s, bool capturing) {
  unsigned long long* v = vacc_set(sc, line);
  KVSEP_HIP(hipMemsetAsync(v, 0, kVaccSetWords * 8, s));
  KVSEP_HIP(hipMemsetAsync(v, 0xff, 8, s));
  if (!capturing) sc.vacc_dirty &= ~(1u << line);
  return KVSEP_OK;
}

// SST verify scratch (len + 1 and the stored trailer words per block).
int ensure_sst(Scratch& sc, uint64_t count) {
  if (count <= sc.cap_sst) return KVSEP_OK;
  int rc = quiesce(sc);
  if (rc) return rc;
  hipFree(sc.d_sst_len1);
  hipFree(sc.d_sst_stored);
  sc.d_sst_len1 = nullptr;
  sc.d_sst_stored = nullptr;
  sc.cap_sst = 0;
  KVSEP_HIP(hipMalloc(&sc.d_sst_len1, count * 8));
  KVSEP_HIP(hipMalloc(&sc.d_sst_stored, count * 4));
  sc.cap_sst = count;
  return KVSEP_OK;
}

int ensure_plan(Scratch& sc, uint64_t piece_bytes, uint64_t count, uint64_t total_bytes) {
  const uint64_t pieces = count + total_bytes / piece_bytes + 1;
  // hipcub's scan takes an int item count; piece and block indices are u32 in the kernels
  if (count > 0x7fffffffull) return set_err(KVSEP_EINVAL, "more than 2^31 - 1 blocks in one batch that needs a plan");
  if (pieces > 0xffffffffull) return set_err(KVSEP_EINVAL, "batch too large for u32 piece indices");
  if (count <= sc.cap_count && pieces <= sc.cap_pieces) return KVSEP_OK;
  const uint64_t nc = std::max<uint64_t>(count, sc.cap_count), np = std::max<uint64_t>(pieces, sc.cap_pieces);
  int rc = quiesce(sc);
  if (rc) return rc;
  free_plan(sc);
  KVSEP_HIP(hipMalloc(&sc.d_counts, nc * 8));
  KVSEP_HIP(hipMalloc(&sc.d_pstart, (nc + 1) * 8));
  KVSEP_HIP(hipMalloc(&sc.d_pblk, np * 4));
  KVSEP_HIP(hipMalloc(&sc.d_partial, np * 4));
  size_t tb = 0;
  KVSEP_HIP(hipcub::DeviceScan::InclusiveSum(nullptr, tb, sc.d_counts, sc.d_pstart + 1, int(nc), hipStream_t(0)));
  KVSEP_HIP(hipMalloc(&sc.d_scan_tmp, tb));
  sc.scan_tmp_bytes = tb;
  sc.cap_count = nc;
  sc.cap_pieces = np;
  return KVSEP_OK;
}

// Narrow or wide kernel for an unsplit batch (every block <= piece_bytes, known from the max_len hint)?  The
// narrow kernel's unit of parallelism is an 8-block group, so it needs many blocks; it wins on short blocks
// when there are enough of them (measured, tools/ab_variants.py on one MI355X):
//   <= 8 KiB blocks from 8 Ki blocks up (8 Ki x 4 KiB: 2.58 vs 2.13 TB/s; 4 Ki x 4 KiB: wide 1.50 vs 1.46),
//   <= 16 KiB blocks from 16 Ki blocks up (16 Ki x 16 KiB: 5.58 vs 5.36; 4 Ki x 16 KiB: wide 3.67 vs 2.58),
//   <= 32 KiB blocks from 32 Ki blocks up (32 Ki x 32 KiB: 6.72 vs 6.35; 16 Ki x 32 KiB: wide 6.12 vs 6.06),
//   64 KiB blocks never (16 Ki x 64 KiB: wide 6.22 vs 4.88).
// The thresholds scale with the CU count (256 on MI355X).  kvsep_crc32c_ctx_set_kernel can force either kernel
// (tests); the choice never changes a result: both are exact for any block, whatever the hint.
// A ragged batch: the max_len hint above 1.25x the mean length total_bytes / count (0 = unknown: not ragged).
bool ragged_batch(uint64_t count, uint64_t total_bytes, uint64_t max_len) {
  return count != 0 && total_bytes != 0 && 4 * max_len > 5 * (total_bytes / count);
}

// The claim kernel with 16-lane slots (form 11: 4-block groups of Z_256 rows) for uniform blocks of 8-12 KiB, from 4 Ki
// of them up to 512 MiB.  Its groups are half the bytes of the 8-lane form's, so the waves' last groups end closer
// together.  Measured against the routing before it in one process (profiles/round4/claim_shapes/claim16*.log, graph
// replay, two boxes): 8 KiB blocks 32 MiB 11.05 vs 11.70 us, 64 MiB 15.73 vs 16.81, 128 MiB 23.94 / 24.14 vs 25.49 /
// 25.29, 256 MiB 41.73 / 42.08 vs 43.78 / 44.08, 512 MiB 80.43 / 80.45 vs 81.73 / 82.07 (1 GiB equal); 10 KiB 64 MiB
// 14.15 vs 19.89, 128 MiB 24.85 vs 31.30, 256 MiB 44.76 vs 44.13, 512 MiB 80.48 vs 82.61; 12 KiB 64 MiB 15.84 vs
// 17.48, 128 MiB 28.88 / 28.12 vs 29.51 / 30.17, 256 MiB 46.01 / 45.68 vs 52.99 / 53.16, 512 MiB 90.06 / 89.33 vs
// 93.73 / 93.18.  Outside that box it loses: 2 KiB and 6-7 KiB blocks at most sizes, 14-32 KiB blocks, 1 GiB.
bool claim16_route(uint64_t count, uint64_t total_bytes, uint64_t max_len) {
  const uint64_t bytes = total_bytes ? total_bytes : count * max_len;
  return max_len >= 8 * 1024 && max_len <= 12 * 1024 && count >= 4096 && bytes <= (512ull << 20);
}

// Narrow-kernel form of a batch that use_narrow() put on the narrow kernels: 6 = 16-wave workgroups, 9 = 8-wave
// workgroups (fill overlapped with the first loads), 10 = workgroup-contiguous runs dealt by LDS claims
// (crc32c_narrow_claim_kernel, 8 waves), 11 = the same with 16-lane slots, 20 = sorted windows
// (crc32c_narrow_sorted_kernel, 16 waves).
int narrow_form(const kvsep_crc32c_ctx* c, uint64_t count, uint64_t total_bytes, uint64_t max_len) {
  if (c->kernel == 3) return 6;
  if (c->kernel == 4) return 9;
  if (c->kernel == 5) return 20;
  if (c->kernel == 6) return 10;
  if (c->kernel == 7) return 11;
  // 16-wave workgroups below 128 Ki blocks of <= 8 KiB (32 Ki blocks of 8-32 KiB), 8-wave ones from there on.  A
  // small batch gives each wave only a couple of 8-block groups, and more waves hide more of the launch/first-load
  // ramp (256 MiB of 4 KiB blocks: 16 waves +2-5 %); a large one streams better with 8 (1 GiB of 4 KiB blocks:
  // +5 %; 32 Ki x 16 KiB +2 %, 32 Ki x 32 KiB +6 %).  The 8-wave kernel overlaps the LDS fill with the first
  // group's loads (+0.3-2 %); at 16 waves that overlap measured -5 %.
  // Ragged batches take the sorted-window kernel at any size: an 8-block group waits for its longest block, and
  // sorting 64-block windows by length makes the groups even (config 4's 902 K blocks <= 32 KiB: 0.93 -> 0.57 ms
  // against the 16-wave narrow kernel, 1.24 ms on the 8-wave one).
  if (ragged_batch(count, total_bytes, max_len)) return 20;
  if (claim16_route(count, total_bytes, max_len)) return 11;
  // The claim kernel (crc32c_narrow_claim_kernel) for uniform blocks of <= 8 KiB from 32 Ki of them up to 384 Ki of
  // <= 4 KiB (128 MiB - 1.5 GiB of 4 KiB blocks) or 64 Ki of 4-8 KiB.  Measured against both forms below in one
  // process (profiles/round4/queue_variants/claim_*.log, graph replay): 4 KiB blocks 128 MiB 26.8 vs 27.8 us, 256 MiB
  // 45.9 vs 48.3, 512 MiB 83.1 vs 91.0, 1 GiB 156.7 vs 166.6, 1.5 GiB 241.4 vs 252.9, but 2 GiB 347.6 vs 314.0 (the
  // wave-major 8-wave kernel streams better from there); 2 KiB blocks 256 MiB 44.9 vs 47.6, 1 GiB 165.1 vs 163.8;
  // 8 KiB blocks 256 MiB 45.2 vs 45.8, 1 GiB 156.9 vs 155.0; 16 KiB blocks never (256 MiB 50.1 vs 44.0).
  if (max_len <= 8 * 1024 && count >= (1u << 15) && count <= (max_len <= 4 * 1024 ? 3u << 17 : 1u << 16)) return 10;
  const bool eight_waves = max_len <= 8 * 1024 ? count >= (1u << 17) : count >= (1u << 15);
  return eight_waves ? 9 : 6;
}

bool use_narrow(const kvsep_crc32c_ctx* c, uint64_t count, uint64_t total_bytes, uint64_t max_len) {
  if (max_len == 0 || max_len > 2 * kNarrowMax) return false;
  if (c->kernel == 1) return false;
  if (c->kernel >= 2) return true;
  const int d = diag_use_narrow(c);  // KVSEP_DIAG build only: -1 (no override) in the shipped library
  if (d >= 0) return d != 0;
  if (claim16_route(count, total_bytes, max_len) && !ragged_batch(count, total_bytes, max_len)) return true;
  const uint64_t cus = uint64_t(c->num_cus);
  return (max_len <= 8 * 1024 && count >= 32 * cus) || (max_len <= 16 * 1024 && count >= 64 * cus) ||
         (max_len <= kNarrowMax && count >= 128 * cus);
}

// Piece size of a planned batch.  With the default setting, a batch too small to give every wave two pieces
// of piece_bytes gets 64, 32 or 16 KiB pieces instead: the largest size that still makes >= 2 pieces per wave
// (64 blocks of 1 MiB: 16 KiB pieces).  Large batches keep piece_bytes.
uint64_t piece_for(const kvsep_crc32c_ctx* c, uint64_t total_bytes, const uint32_t** zp) {
  *zp = &c->d_tabs->zpiece[0][0];
  if (!c->piece_auto) return c->piece_bytes;
  const uint64_t want = 2 * uint64_t(c->num_cus) * (kWgThreads / 64);
  uint64_t P = c->piece_bytes;
  for (int k = 2; k >= 0 && total_bytes / P < want; --k) {
    P = kSmallPiece << k;
    *zp = &c->d_tabs->zsmall[k][0][0];
  }
  return P;
}

hipEvent_t take_event(kvsep_crc32c_ctx* c) {
  if (!c->ev_pool.empty()) {
    hipEvent_t e = c->ev_pool.back();
    c->ev_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

template <bool P, bool D, bool V>
void launch_pieces_v(const kvsep_crc32c_ctx* c, unsigned grid, hipStream_t s, const PiecesArgs& a) {
  // Default (1): 8-wave workgroups (2 waves per SIMD, up to 256 VGPRs), 4-row groups, non-temporal loads, next
  // item staged ahead.  On one MI355X, interleaved in one process (tools/ab_variants.py), 8 waves beat 16 waves
  // by 1.5-2 % on 1 MiB blocks and by 4-5 % on the Zipf batch; 12 waves sit between.  (A 3-slot ring of row groups,
  // 8 rows in flight, was tried and measured -2 to -7 %: the extra VGPRs cost LDS-lookup overlap; so was staging items
  // two ahead, -1.5 % on the Zipf batch.)  Only the default is compiled into the shipped library; the A/B and ablation
  // variants live in crc32c_diag.inc, compiled into the KVSEP_DIAG tools build only.
  constexpr int T = kWgThreads;
  if (V) {  // the verify form: the shipped configuration only
    crc32c_pieces_kernel<P, D, 4, true, true, T, true, true><<<grid, T, 0, s>>>(a);
    return;
  }
  if (diag_launch_pieces<P, D>(c, grid, s, a)) return;  // KVSEP_DIAG build only
  crc32c_pieces_kernel<P, D, 4, true, true, T><<<grid, T, 0, s>>>(a);
}

template <bool V>
void launch_pieces_vv(const kvsep_crc32c_ctx* c, bool planned, bool dyn, unsigned grid, hipStream_t s,
                      const PiecesArgs& a) {
  if (planned) {
    if (dyn) launch_pieces_v<true, true, V>(c, grid, s, a);
    else launch_pieces_v<true, false, V>(c, grid, s, a);
  } else {
    if (dyn) launch_pieces_v<false, true, V>(c, grid, s, a);
    else launch_pieces_v<false, false, V>(c, grid, s, a);
  }
}

void launch_pieces(const kvsep_crc32c_ctx* c, bool planned, bool dyn, bool verify, unsigned grid, hipStream_t s,
                   const PiecesArgs& a) {
  if (verify) launch_pieces_vv<true>(c, planned, dyn, grid, s, a);
  else launch_pieces_vv<false>(c, planned, dyn, grid, s, a);
}

int launch_batch_in(kvsep_crc32c_ctx* c, Scratch& sc, hipStream_t s, bool capturing, const void* base,
                    const uint64_t* off, const uint64_t* len, const uint32_t* init, const uint32_t* expect,
                    uint32_t* out, uint64_t* first_bad, uint64_t* nbad, uint64_t count, uint64_t total_bytes,
                    uint64_t max_len);

// Every use of a Scratch is bracketed by acquire/release (event ordering across streams).
int launch_batch(kvsep_crc32c_ctx* c, Scratch& sc, hipStream_t s, const void* base, const uint64_t* off,
                 const uint64_t* len, const uint32_t* init, const uint32_t* expect, uint32_t* out, uint64_t* first_bad,
                 uint64_t* nbad, uint64_t count, uint64_t total_bytes, uint64_t max_len) {
  if (!base || !off || !len || !out) return set_err(KVSEP_EINVAL, "null pointer argument");
  // block indices travel as u32 through the descriptor windows and the piece table
  if (count > 0xffffffffull) return set_err(KVSEP_EINVAL, "more than 2^32 - 1 blocks in one batch");
  DeviceGuard dg(c->device);
  KVSEP_HIP(dg.err);
  // Under stream capture (hipGraph) the call only records its nodes: the cross-stream scratch events are
  // skipped (a captured wait on an event recorded outside the capture is not allowed), so the graph's user
  // orders its replays against other uses of this context's scratch.  Allocation must not happen either:
  // kvsep_crc32c_reserve first.
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  KVSEP_HIP(hipStreamIsCapturing(s, &cap));
  const bool capturing = cap != hipStreamCaptureStatusNone;
  int rc = capturing ? KVSEP_OK : acquire(sc, s);
  if (rc) return rc;
  rc = launch_batch_in(c, sc, s, capturing, base, off, len, init, expect, out, first_bad, nbad, count, total_bytes,
                       max_len);
  if (rc) {
    if (!capturing) (void)release(sc, s);  // whatever was enqueued stays ordered before the scratch's next user
    return rc;
  }
  return capturing ? KVSEP_OK : release(sc, s);
}

int launch_batch_body(kvsep_crc32c_ctx* c, Scratch& sc, hipStream_t s, PiecesArgs& a, const void* base,
                      const uint64_t* off, const uint64_t* len, const uint32_t* init, const uint32_t* expect,
                      uint32_t* out, uint64_t* first_bad, uint64_t* nbad, uint64_t count, uint64_t total_bytes,
                      uint64_t max_len);

int launch_batch_in(kvsep_crc32c_ctx* c, Scratch& sc, hipStream_t s, bool capturing, const void* base,
                    const uint64_t* off, const uint64_t* len, const uint32_t* init, const uint32_t* expect,
                    uint32_t* out, uint64_t* first_bad, uint64_t* nbad, uint64_t count, uint64_t total_bytes,
                    uint64_t max_len) {
  PiecesArgs a{};
  uint32_t line = 0;
  if (expect) {
    int rc = ensure_verify(sc);
    if (rc) return rc;
    line = capturing ? 1 + (sc.vacc_next++ % (kVaccLines - 1)) : 0;
    if (sc.vacc_dirty & (1u << line)) {
      rc = reset_vacc(sc, line, s, capturing);
      if (rc) return rc;
    }
    a.vacc = vacc_set(sc, line);  // the accumulators, in their reset state: the kernels publish the verdict
  }
  const int rc = launch_batch_body(c, sc, s, a, base, off, len, init, expect, out, first_bad, nbad, count, total_bytes,
                                   max_len);
  if (rc && expect) sc.vacc_dirty |= 1u << line;  // a kernel may have posted to the set: reset it before its next use
  return rc;
}

int launch_batch_body(kvsep_crc32c_ctx* c, Scratch& sc, hipStream_t s, PiecesArgs& a, const void* base,
                      const uint64_t* off, const uint64_t* len, const uint32_t* init, const uint32_t* expect,
                      uint32_t* out, uint64_t* first_bad, uint64_t* nbad, uint64_t count, uint64_t total_bytes,
                      uint64_t max_len) {
  const bool planned = !(max_len != 0 && max_len <= c->piece_bytes);
  a.base = static_cast<const uint8_t*>(base);
  a.off = off;
  a.len = len;
  a.init = init;
  a.out = out;
  a.count = count;
  a.piece_bytes = planned ? piece_for(c, total_bytes, &a.zpiece) : c->piece_bytes;
  a.tabs = c->d_tabs;
  if (expect) {
    if (!first_bad || !nbad) {
      first_bad = reinterpret_cast<uint64_t*>(sc.d_verify);
      nbad = reinterpret_cast<uint64_t*>(sc.d_verify + 1);
    }
    if (count == 0) {          // nothing to check, no kernel: the verdict is "none" (first_bad = ~0, nbad = 0)
      KVSEP_HIP(hipMemsetAsync(first_bad, 0xff, 8, s));
      KVSEP_HIP(hipMemsetAsync(nbad, 0, 8, s));
    }
  }
  a.expect = expect;
  a.first_bad = reinterpret_cast<unsigned long long*>(first_bad);
  a.nbad = reinterpret_cast<unsigned long long*>(nbad);
  // The verify form's compare runs inside the CRC kernels (and the combine kernel for split blocks): `fused`.  Only
  // the A/B variants of the KVSEP_DIAG tools build fall back to the separate verify_finish_kernel pass.
  bool fused = true;
  if (count == 0) return KVSEP_OK;
  if (planned) {
    int rc = ensure_plan(sc, a.piece_bytes, count, total_bytes);
    if (rc) return rc;
    a.pstart = sc.d_pstart;
    a.pblk = sc.d_pblk;
    a.partial = sc.d_partial;
    a.max_pieces = sc.cap_pieces;
    const unsigned nb = unsigned((count + 255) / 256);
    crc32c_plan_count_kernel<<<nb, 256, 0, s>>>(len, count, a.piece_bytes, sc.d_counts);
    KVSEP_HIP(hipGetLastError());
    KVSEP_HIP(hipMemsetAsync(sc.d_pstart, 0, 8, s));
    size_t tb = sc.scan_tmp_bytes;
    KVSEP_HIP(hipcub::DeviceScan::InclusiveSum(sc.d_scan_tmp, tb, sc.d_counts, sc.d_pstart + 1, int(count), s));
    crc32c_plan_expand_kernel<<<nb, 256, 0, s>>>(sc.d_pstart, count, sc.cap_pieces, sc.d_pblk);
    KVSEP_HIP(hipGetLastError());
  } else {
    a.max_pieces = count;
  }
  // auto schedule: guided (one atomic per grab) for planned batches with many pieces; static for the rest --
  // a few thousand small pieces would spend most of the kernel in single-item grabs on one counter
  // (~88 dequeues/us, MI355X_MICROARCH.md dequeue)
  const uint64_t est_items = planned ? count + total_bytes / a.piece_bytes : count;
  const uint64_t nwaves_est = uint64_t(c->num_cus) * (kWgThreads / 64);
  const bool dyn = c->dynamic < 0 ? (planned && est_items >= 8 * nwaves_est) : c->dynamic == 1;
  a.static_contig = c->static_contig;
  a.guided_div = 0;  // adaptive (crc32c_pieces_kernel)
  a.guided_cap = 0;
  if (dyn) {
    if (!sc.d_counter) KVSEP_HIP(hipMalloc(&sc.d_counter, 16));
    a.work_counter = sc.d_counter;
    KVSEP_HIP(hipMemsetAsync(sc.d_counter, 0, 4, s));
  }
  const unsigned grid = unsigned(c->num_cus);  // one workgroup per CU, persistent
  hipEvent_t e0 = nullptr, e1 = nullptr;
  if (c->timing) {
    e0 = take_event(c);
    e1 = take_event(c);
    if (e0 && e1) KVSEP_HIP(hipEventRecord(e0, s));
  }
  if (!planned && use_narrow(c, count, total_bytes, max_len)) {
    int nv = narrow_form(c, count, total_bytes, max_len);
    nv = diag_narrow_form(c, nv);  // KVSEP_DIAG build only
    a.hint = max_len;
    if (expect && (nv == 6 || nv == 9 || nv == 10 || nv == 11 || nv == 20)) {  // verify form of the shipped forms
      switch (nv) {
        case 9: crc32c_narrow_kernel<4, true, 512, true, true, LdsFull, true><<<grid, 512, 0, s>>>(a); break;
        case 10: crc32c_narrow_claim_kernel<4, 512, true><<<grid, 512, 0, s>>>(a); break;
        case 11: crc32c_narrow_claim_kernel<4, 512, true, true, 16><<<grid, 512, 0, s>>>(a); break;
        case 20: crc32c_narrow_sorted_kernel<4, true, 1024, true><<<grid, 1024, 0, s>>>(a); break;
        default: crc32c_narrow_kernel<4, true, 1024, false, true, LdsFull, true><<<grid, 1024, 0, s>>>(a); break;
      }
    } else {
    // KVSEP_DIAG variants only (the shipped forms are 6, 9, 10, 11 and 20): they post to the caller's words directly, from
    // their own in-kernel compare or from verify_finish_kernel, so those words are set first
    if (expect) {
      KVSEP_HIP(hipMemsetAsync(first_bad, 0xff, 8, s));
      KVSEP_HIP(hipMemsetAsync(nbad, 0, 8, s));
    }
    fused = !expect || diag_self_compare(nv);
    if (!diag_launch_narrow(nv, grid, s, a, count))  // KVSEP_DIAG build only
    switch (nv) {
      case 9: crc32c_narrow_kernel<4, true, 512, true><<<grid, 512, 0, s>>>(a); break;
      case 10: crc32c_narrow_claim_kernel<4, 512><<<grid, 512, 0, s>>>(a); break;
      case 11: crc32c_narrow_claim_kernel<4, 512, false, true, 16><<<grid, 512, 0, s>>>(a); break;
      case 20: crc32c_narrow_sorted_kernel<4, true, 1024><<<grid, 1024, 0, s>>>(a); break;
      default: crc32c_narrow_kernel<4, true, 1024><<<grid, 1024, 0, s>>>(a); break;
    }
    }
  } else {
    launch_pieces(c, planned, dyn, expect != nullptr, grid, s, a);
  }
  KVSEP_HIP(hipGetLastError());
  if (c->inject_failure) {  // fault injection (tests): fail between the CRC kernel and the combine kernel
    c->inject_failure = false;
    return set_err(KVSEP_EHIP, "injected failure after the CRC kernel (kvsep_crc32c_ctx_inject_failure)");
  }
  if (c->timing && e0 && e1) {
    KVSEP_HIP(hipEventRecord(e1, s));
    c->ev_pending.emplace_back(e0, e1);
  }
  if (planned) {
    if (expect) crc32c_combine_kernel<true><<<unsigned((count + 255) / 256), 256, 0, s>>>(a);
    else crc32c_combine_kernel<false><<<unsigned((count + 255) / 256), 256, 0, s>>>(a);
    KVSEP_HIP(hipGetLastError());
  }
  if (expect && !fused) {
    verify_finish_kernel<<<unsigned((count + 255) / 256), 256, 0, s>>>(
        out, expect, count, reinterpret_cast<unsigned long long*>(first_bad), reinterpret_cast<unsigned long long*>(nbad));
    KVSEP_HIP(hipGetLastError());
  }
  return KVSEP_OK;
}
}  // namespace

namespace kvsep {
int device_batch_locked(kvsep_crc32c_ctx* c, Scratch& sc, hipStream_t s, const void* base, const uint64_t* off,
                        const uint64_t* len, const uint32_t* init, uint32_t* out, uint64_t count,
                        uint64_t total_bytes, uint64_t max_len) {
  return launch_batch(c, sc, s, base, off, len, init, nullptr, out, nullptr, nullptr, count, total_bytes, max_len);
}

void free_scratch(Scratch& sc) {
  if (sc.used && sc.last_use) (void)hipEventSynchronize(sc.last_use);
  free_plan(sc);
  hipFree(sc.d_counter);
  hipFree(sc.d_verify);
  hipFree(sc.d_sst_len1);
  hipFree(sc.d_sst_stored);
  if (sc.last_use) (void)hipEventDestroy(sc.last_use);
  sc = Scratch();
}
HostStaging& ctx_staging(kvsep_crc32c_ctx* c) { return c->staging; }
std::mutex& ctx_mutex(kvsep_crc32c_ctx* c) { return c->mu; }
int ctx_device(kvsep_crc32c_ctx* c) { return c->device; }
int ctx_host_node(kvsep_crc32c_ctx* c) { return c->host_node; }
uint64_t ctx_piece_bytes(kvsep_crc32c_ctx* c) { return c->piece_bytes; }
void set_last_error(const char* msg) { g_last_error = msg; }
}  // namespace kvsep

extern "C" {

int kvsep_device_count(void) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  return n;
}

int kvsep_crc32c_ctx_create(int device, kvsep_crc32c_ctx** out) {
  if (!out) return set_err(KVSEP_EINVAL, "out is null");
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n <= device || device < 0)
    return set_err(KVSEP_ENODEV, "no HIP device with that ordinal");
  hipDeviceProp_t prop;
  KVSEP_HIP(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    std::string m = std::string("device is ") + prop.gcnArchName + ", this build targets gfx950 only";
    return set_err(KVSEP_ENODEV, m.c_str());
  }
  DeviceGuard dg(device);
  KVSEP_HIP(dg.err);
  auto* c = new kvsep_crc32c_ctx();
  c->device = device;
  c->num_cus = prop.multiProcessorCount;
  c->host_node = kvsep_device_numa_node(device);
  diag_env(c);  // tools build only: no environment variable reaches the shipped library's kernel choice
  int rc = upload_tables(c);
  if (rc) {
    delete c;
    return rc;
  }
  *out = c;
  return KVSEP_OK;
}

void kvsep_crc32c_ctx_destroy(kvsep_crc32c_ctx* c) {
  if (!c) return;
  DeviceGuard dg(c->device);
  hipDeviceSynchronize();
  free_scratch(c->sc);
  hipFree(c->d_tabs);
  for (auto& p : c->ev_pending) { hipEventDestroy(p.first); hipEventDestroy(p.second); }
  for (auto e : c->ev_pool) hipEventDestroy(e);
  release_staging(c->staging);
  diag_forget(c);  // KVSEP_DIAG build only
  delete c;
}

int kvsep_crc32c_ctx_set_piece_bytes(kvsep_crc32c_ctx* c, uint64_t piece_bytes) {
  if (!c || piece_bytes < 1024 || piece_bytes % 1024) return set_err(KVSEP_EINVAL, "piece_bytes must be a multiple of 1 KiB");
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device);
  KVSEP_HIP(dg.err);
  KVSEP_HIP(hipDeviceSynchronize());
  c->piece_bytes = piece_bytes;
  c->piece_auto = false;
  free_plan(c->sc);  // piece tables depend on piece_bytes (device already idle)
  for (auto& sc : c->staging.scratch) free_plan(sc);
  return upload_tables(c);
}

int kvsep_crc32c_ctx_set_schedule(kvsep_crc32c_ctx* c, int dynamic) {
  if (!c) return set_err(KVSEP_EINVAL, "null ctx");
  std::lock_guard<std::mutex> g(c->mu);
  c->dynamic = dynamic < 0 ? -1 : (dynamic == 1 ? 1 : 0);
  c->static_contig = dynamic == 2 ? 0 : 1;
  return KVSEP_OK;
}

int kvsep_crc32c_ctx_set_kernel(kvsep_crc32c_ctx* c, int kernel) {
  if (!c || kernel < 0 || kernel > 7) return set_err(KVSEP_EINVAL, "kernel must be 0..7");
  std::lock_guard<std::mutex> g(c->mu);
  c->kernel = kernel;
  return KVSEP_OK;
}

int kvsep_crc32c_ctx_set_host_node(kvsep_crc32c_ctx* c, int node) {
  if (!c || node < -1) return set_err(KVSEP_EINVAL, "node must be >= -1");
  std::lock_guard<std::mutex> g(c->mu);
  c->host_node = node;
  return KVSEP_OK;
}

int kvsep_crc32c_ctx_inject_failure(kvsep_crc32c_ctx* c) {
  if (!c) return set_err(KVSEP_EINVAL, "null ctx");
  std::lock_guard<std::mutex> g(c->mu);
  c->inject_failure = true;
  return KVSEP_OK;
}

int kvsep_crc32c_reserve(kvsep_crc32c_ctx* c, uint64_t count, uint64_t total_bytes) {
  if (!c) return set_err(KVSEP_EINVAL, "null ctx");
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device);
  KVSEP_HIP(dg.err);
  // everything a later call could allocate, so that the call can be captured into a hipGraph
  if (!c->sc.d_counter) KVSEP_HIP(hipMalloc(&c->sc.d_counter, 16));
  int vr = ensure_verify(c->sc);
  if (vr) return vr;
  if (!c->sc.last_use) KVSEP_HIP(hipEventCreateWithFlags(&c->sc.last_use, hipEventDisableTiming));
  int rc = ensure_sst(c->sc, count);
  if (rc) return rc;
  const uint32_t* zp = nullptr;
  return ensure_plan(c->sc, piece_for(c, total_bytes, &zp), count, total_bytes);
}

int kvsep_crc32c_ctx_set_timing(kvsep_crc32c_ctx* c, int enable) {
  if (!c) return set_err(KVSEP_EINVAL, "null ctx");
  c->timing = enable != 0;
  return KVSEP_OK;
}

int kvsep_crc32c_ctx_get_timing(kvsep_crc32c_ctx* c, double* total_ms, uint64_t* launches) {
  if (!c) return set_err(KVSEP_EINVAL, "null ctx");
  std::lock_guard<std::mutex> g(c->mu);
  double ms = 0;
  uint64_t n = 0;
  for (auto& p : c->ev_pending) {
    KVSEP_HIP(hipEventSynchronize(p.second));
    float t = 0;
    KVSEP_HIP(hipEventElapsedTime(&t, p.first, p.second));
    ms += t;
    ++n;
    c->ev_pool.push_back(p.first);
    c->ev_pool.push_back(p.second);
  }
  c->ev_pending.clear();
  if (total_ms) *total_ms = ms;
  if (launches) *launches = n;
  return KVSEP_OK;
}

int kvsep_crc32c_batch_device(kvsep_crc32c_ctx* c, void* stream, const void* base, const uint64_t* off,
                              const uint64_t* len, const uint32_t* init, uint32_t* out, uint64_t count,
                              uint64_t total_bytes, uint64_t max_len) {
  if (!c) return set_err(KVSEP_EINVAL, "null ctx");
  std::lock_guard<std::mutex> g(c->mu);
  return launch_batch(c, c->sc, static_cast<hipStream_t>(stream), base, off, len, init, nullptr, out, nullptr,
                      nullptr, count, total_bytes, max_len);
}

int kvsep_crc32c_verify_device(kvsep_crc32c_ctx* c, void* stream, const void* base, const uint64_t* off,
                               const uint64_t* len, const uint32_t* init, const uint32_t* expected_masked,
                               uint32_t* out, uint64_t* first_bad, uint64_t* nbad, uint64_t count,
                               uint64_t total_bytes, uint64_t max_len) {
  if (!c || !expected_masked) return set_err(KVSEP_EINVAL, "null ctx or expected_masked");
  std::lock_guard<std::mutex> g(c->mu);
  return launch_batch(c, c->sc, static_cast<hipStream_t>(stream), base, off, len, init, expected_masked, out,
                      first_bad, nbad, count, total_bytes, max_len);
}

int kvsep_fill_splitmix64_device(void* stream, void* dst, uint64_t nbytes, uint64_t seed, uint64_t stream_offset) {
  if (!dst && nbytes) return set_err(KVSEP_EINVAL, "null dst");
  if (!nbytes) return KVSEP_OK;
  hipStream_t s = static_cast<hipStream_t>(stream);
  const unsigned grid = 256 * 8;
  if ((reinterpret_cast<uintptr_t>(dst) & 15) == 0 && (stream_offset & 15) == 0) {
    const uint64_t n16 = nbytes / 16;
    if (n16) fill_splitmix_fast_kernel<<<grid, 256, 0, s>>>(static_cast<uint4*>(dst), n16, seed, stream_offset / 8);
    const uint64_t rest = nbytes - n16 * 16;
    if (rest)
      fill_splitmix_bytes_kernel<<<1, 64, 0, s>>>(static_cast<uint8_t*>(dst) + n16 * 16, rest, seed,
                                                  stream_offset + n16 * 16);
  } else {
    fill_splitmix_bytes_kernel<<<grid, 256, 0, s>>>(static_cast<uint8_t*>(dst), nbytes, seed, stream_offset);
  }
  KVSEP_HIP(hipGetLastError());
  return KVSEP_OK;
}

int kvsep_sst_trailers_device(kvsep_crc32c_ctx* c, void* stream, const void* base, const uint64_t* off,
                              const uint64_t* len, const uint8_t* types, uint32_t* masked_out, uint64_t count,
                              uint64_t total_bytes, uint64_t max_len) {
  if (!c || !types || !masked_out) return set_err(KVSEP_EINVAL, "null argument");
  std::lock_guard<std::mutex> g(c->mu);
  hipStream_t s = static_cast<hipStream_t>(stream);
  int rc = launch_batch(c, c->sc, s, base, off, len, nullptr, nullptr, masked_out, nullptr, nullptr, count,
                        total_bytes, max_len);
  if (rc || !count) return rc;
  sst_trailer_finish_kernel<<<unsigned((count + 255) / 256), 256, 0, s>>>(masked_out, types, masked_out, count,
                                                                          c->d_tabs);
  KVSEP_HIP(hipGetLastError());
  return KVSEP_OK;
}

int kvsep_sst_verify_device(kvsep_crc32c_ctx* c, void* stream, const void* file_base, const uint64_t* off,
                            const uint64_t* len, uint32_t* out, uint64_t* first_bad, uint64_t* nbad, uint64_t count,
                            uint64_t total_bytes, uint64_t max_len) {
  if (!c || !file_base || !off || !len || !out) return set_err(KVSEP_EINVAL, "null argument");
  std::lock_guard<std::mutex> g(c->mu);
  hipStream_t s = static_cast<hipStream_t>(stream);
  DeviceGuard dg(c->device);
  KVSEP_HIP(dg.err);
  Scratch& sc = c->sc;
  // as launch_batch: under capture no cross-stream events and no allocation (kvsep_crc32c_reserve sizes SST
  // scratch too)
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  KVSEP_HIP(hipStreamIsCapturing(s, &cap));
  const bool capturing = cap != hipStreamCaptureStatusNone;
  if (capturing && count > sc.cap_sst) return set_err(KVSEP_EINVAL, "SST verify under capture needs kvsep_crc32c_reserve first");
  int rc = capturing ? KVSEP_OK : acquire(sc, s);
  if (rc) return rc;
  rc = ensure_sst(sc, count);
  if (rc) return rc;
  if (count) {
    sst_verify_prep_kernel<<<unsigned((count + 255) / 256), 256, 0, s>>>(static_cast<const uint8_t*>(file_base), off,
                                                                        len, sc.d_sst_len1, sc.d_sst_stored, count);
    KVSEP_HIP(hipGetLastError());
  }
  rc = launch_batch_in(c, sc, s, capturing, file_base, off, sc.d_sst_len1, nullptr, sc.d_sst_stored, out, first_bad,
                       nbad, count, total_bytes + count, max_len ? max_len + 1 : 0);
  if (rc) {
    if (!capturing) (void)release(sc, s);
    return rc;
  }
  return capturing ? KVSEP_OK : release(sc, s);
}

const char* kvsep_crc32c_kernel_name(kvsep_crc32c_ctx* c, uint64_t count, uint64_t total_bytes, uint64_t max_len) {
  if (!c) return "";
  const bool planned = !(max_len != 0 && max_len <= c->piece_bytes);
  if (planned || !use_narrow(c, count, total_bytes, max_len)) return "crc32c_pieces_kernel";
  const int nf = narrow_form(c, count, total_bytes, max_len);
  return nf == 20 ? "crc32c_narrow_sorted_kernel"
         : nf == 10 || nf == 11 ? "crc32c_narrow_claim_kernel" : "crc32c_narrow_kernel";
}

int kvsep_stream_read_device(kvsep_crc32c_ctx* c, void* stream, const void* src, uint64_t nbytes, uint32_t* sink) {
  if (!c || !src || !sink) return set_err(KVSEP_EINVAL, "null argument");
  hipStream_t s = static_cast<hipStream_t>(stream);
  const uint64_t n16 = nbytes / 16;
  hipEvent_t e0 = nullptr, e1 = nullptr;
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device);
  KVSEP_HIP(dg.err);
  if (c->timing) {
    e0 = take_event(c);
    e1 = take_event(c);
    if (e0 && e1) KVSEP_HIP(hipEventRecord(e0, s));
  }
  if (!diag_stream_read(c, s, reinterpret_cast<uintptr_t>(src), n16, sink))  // KVSEP_DIAG build only
  stream_read_kernel<<<unsigned(c->num_cus), 512, 0, s>>>(reinterpret_cast<uintptr_t>(src), n16, sink);
  KVSEP_HIP(hipGetLastError());
  if (c->timing && e0 && e1) {
    KVSEP_HIP(hipEventRecord(e1, s));
    c->ev_pending.emplace_back(e0, e1);
  }
  return KVSEP_OK;
}

const char* kvsep_last_error(void) { return g_last_error.c_str(); }

}  // extern "C"
