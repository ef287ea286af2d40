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
//
// One translation unit, in parts: crc32c_fold.inc (the shared device code), crc32c_wide.inc (the wide kernel),
// crc32c_narrow.inc (the narrow kernels for short blocks), crc32c_support.inc (combine, plan, helpers), then this
// file's host side -- the context, kernel routing, launches and the device C ABI.  crc32c_hooks.inc holds the
// measurement hook points (empty in the shipped library), crc32c_diag.inc the KVSEP_DIAG build's A/B forms.
#include <hip/hip_runtime.h>
#include <hipcub/hipcub.hpp>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/kvsep_crc32c.h"
#include "gf2.h"
#include "kvsep_testing.h"
#include "kvsep_internal.h"

namespace kvsep {

#include "crc32c_fold.inc"     // shared device code: tables, arguments, fold, staging, verify, LDS fill
#include "crc32c_wide.inc"     // crc32c_pieces_kernel
#include "crc32c_narrow.inc"   // crc32c_narrow_kernel, _claim_kernel, _sorted_kernel
#include "crc32c_support.inc"  // combine, plan, SST helpers, generator, streaming read

}  // namespace kvsep

// ================================================================================================
// host side
using namespace kvsep;

// A graph capture's own scratch (round 6).  Every call captured into one graph -- one capture
// sequence, hipStreamGetCaptureInfo's id -- runs on the same capture set, and no other capture shares it while it is
// held, so two graphs replayed at once never share a plan, a work counter, SST arrays or verdict slots, and replays of
// one graph write identical words.  Sets are sized by kvsep_crc32c_reserve before capture (nothing is allocated under
// capture) and stay held, frozen in size, until kvsep_crc32c_release_captures: a graph keeps the pointers it captured.
struct CaptureSet {
  unsigned long long id = 0;
  bool held = false;
  Scratch sc;
};
constexpr size_t kDefaultCaptureSets = 4;

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
  std::vector<std::unique_ptr<CaptureSet>> caps;  // scratch of captured calls, one set per graph capture
  uint64_t res_count = 0, res_bytes = 0;          // the largest reservation: what capture sets are sized for
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

// The verify form's device words (allocated once per scratch -- kvsep_crc32c_reserve does it for capture sets): on the
// first 128-B line the result words of a call whose caller passes none; then the accumulators eager calls post to and
// reset (PiecesArgs::vacc: the lowest-block word and the final arrival word, then 8 shard arrival words, each group on
// a line of its own), which must start in their reset state: ~0 (no mismatch), 0 (nothing arrived, none bad).  Eager
// calls on one scratch are ordered one after another by its events, so one set serves them all; captured calls publish
// through verdict slots instead (ensure_vslot), which hold no state from one call to the next.
constexpr uint32_t kVaccSetWords = kVaccStride * (1 + kVaccShards);
unsigned long long* vacc_set(Scratch& sc) { return sc.d_verify + kVaccStride; }

int ensure_verify(Scratch& sc) {
  if (sc.d_verify) return KVSEP_OK;
  std::vector<unsigned long long> init(kVaccStride + kVaccSetWords, 0ull);
  init[0] = ~0ull;             // default first_bad
  init[kVaccStride] = ~0ull;   // the set's vacc[0]
  KVSEP_HIP(hipMalloc(&sc.d_verify, init.size() * 8));
  KVSEP_HIP(hipMemcpy(sc.d_verify, init.data(), init.size() * 8, hipMemcpyHostToDevice));
  sc.vacc_dirty = false;
  return KVSEP_OK;
}

// Verdict slots of captured verify calls: one per workgroup of the CRC kernel (num_cus) and of the combine kernel.
uint32_t vslots_needed(const kvsep_crc32c_ctx* c) { return uint32_t(c->num_cus) + kCombineMaxGrid; }

int ensure_vslot(Scratch& sc, uint32_t n) {
  if (sc.cap_vslot >= n) return KVSEP_OK;
  hipFree(sc.d_vslot);
  sc.d_vslot = nullptr;
  sc.cap_vslot = 0;
  KVSEP_HIP(hipMalloc(&sc.d_vslot, uint64_t(n) * 16));
  sc.cap_vslot = n;
  return KVSEP_OK;
}

// Puts the eager accumulator set back in its reset state, in stream order (two memsets).  Needed after an eager call
// that failed once its CRC kernel was enqueued: the kernel's posts stay in the set, and with no publishing kernel after
// them nothing resets it -- the next verdict would inherit a stale count and first_bad.  The failed call
// marks the set (vacc_dirty) and the next eager verify call on the scratch resets it first.  Captured calls never need
// this: their slots are overwritten whole by every replay.
int reset_vacc(Scratch& sc, hipStream_t s) {
  unsigned long long* v = vacc_set(sc);
  KVSEP_HIP(hipMemsetAsync(v, 0, kVaccSetWords * 8, s));
  KVSEP_HIP(hipMemsetAsync(v, 0xff, 8, s));
  sc.vacc_dirty = false;
  return KVSEP_OK;
}

// SST verify scratch (len + 1 and the stored trailer words per block).
int ensure_sst(Scratch& sc, uint64_t count, bool capturing = false) {
  if (count <= sc.cap_sst) return KVSEP_OK;
  if (capturing) return set_err(KVSEP_EINVAL, "SST verify under capture needs kvsep_crc32c_reserve first");
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

int ensure_plan(Scratch& sc, uint64_t piece_bytes, uint64_t count, uint64_t total_bytes, bool capturing = false) {
  const uint64_t pieces = count + total_bytes / piece_bytes + 1;
  // hipcub's scan takes an int item count; piece and block indices are u32 in the kernels
  if (count > 0x7fffffffull) return set_err(KVSEP_EINVAL, "more than 2^31 - 1 blocks in one batch that needs a plan");
  if (pieces > 0xffffffffull) return set_err(KVSEP_EINVAL, "batch too large for u32 piece indices");
  if (count <= sc.cap_count && pieces <= sc.cap_pieces) return KVSEP_OK;
  if (capturing)
    return set_err(KVSEP_EINVAL, "a captured planned batch larger than kvsep_crc32c_reserve sized its capture set for");
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
// (crc32c_narrow_sorted_kernel, 16 waves), 12 = the workgroup's 8 waves on one group (crc32c_narrow_coop_kernel;
// set_kernel only: measured 1.5x the claim kernel's time on config 2, see its header).
int narrow_form(const kvsep_crc32c_ctx* c, uint64_t count, uint64_t total_bytes, uint64_t max_len) {
  if (c->kernel == 3) return 6;
  if (c->kernel == 4) return 9;
  if (c->kernel == 5) return 20;
  if (c->kernel == 6) return 10;
  if (c->kernel == 7) return 11;
  if (c->kernel == 8) return 12;
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

// The claim kernel's shipped levers (crc32c_narrow_claim_kernel's kLean, round 6): the fill fetching each table entry
// once and no head / tail loads for groups without such chunks -- 16 of config 2's 52 non-payload loads per wave.  On
// one MI355X, interleaved in one process against the round-5 form (diag variant 65; tools/narrow_variants_probe.py,
// profiles/round6/claim_lean.log): 4 KiB blocks 128 MiB 24.66 vs 24.88 us, 256 MiB 43.93 vs 44.32, 1 GiB 153.98 vs
// 154.06 -- about 1 % at config 2, the time the loads cost; the rest of config 2's distance to the streaming read is not
// in instruction count.  Bit 2 (no init load for init-less batches) measured nothing and is not shipped.
constexpr uint32_t kClaimLean = 3;

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

// Is `s` capturing, and if so which capture set do its calls run on: the one this capture already holds, else the first
// free one.  No free set is an error at capture time (KVSEP_EINVAL), never a shared set.
int stream_scratch(kvsep_crc32c_ctx* c, hipStream_t s, Scratch& eager, bool* capturing, Scratch** out) {
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  unsigned long long id = 0;
  KVSEP_HIP(hipStreamGetCaptureInfo(s, &cap, &id));
  *capturing = cap != hipStreamCaptureStatusNone;
  *out = &eager;
  if (!*capturing) return KVSEP_OK;
  for (auto& k : c->caps)
    if (k->held && k->id == id) {
      *out = &k->sc;
      return KVSEP_OK;
    }
  for (auto& k : c->caps)
    if (!k->held) {
      k->held = true;
      k->id = id;
      *out = &k->sc;
      return KVSEP_OK;
    }
  return set_err(KVSEP_EINVAL, c->caps.empty()
                                   ? "graph capture needs kvsep_crc32c_reserve first (it sizes the capture sets)"
                                   : "every capture set of this context is held by an earlier graph: "
                                     "kvsep_crc32c_reserve_captures for more, or kvsep_crc32c_release_captures once "
                                     "those graphs are destroyed");
}

// Every use of a Scratch is bracketed by acquire/release (event ordering across streams).
int launch_batch(kvsep_crc32c_ctx* c, Scratch& eager, hipStream_t s, const void* base, const uint64_t* off,
                 const uint64_t* len, const uint32_t* init, const uint32_t* expect, uint32_t* out, uint64_t* first_bad,
                 uint64_t* nbad, uint64_t count, uint64_t total_bytes, uint64_t max_len) {
  if (!base || !off || !len || !out) return set_err(KVSEP_EINVAL, "null pointer argument");
  // block indices travel as u32 through the descriptor windows and the piece table
  if (count > 0xffffffffull) return set_err(KVSEP_EINVAL, "more than 2^32 - 1 blocks in one batch");
  DeviceGuard dg(c->device);
  KVSEP_HIP(dg.err);
  // Under stream capture (hipGraph) the call only records its nodes, on its capture's own set (stream_scratch): the
  // cross-stream scratch events are skipped (a captured wait on an event recorded outside the capture is not allowed)
  // and nothing is allocated -- kvsep_crc32c_reserve sized the set.  Calls captured into one graph share its set, so
  // they must be ordered within the graph (captured on one stream, or joined).
  bool capturing = false;
  Scratch* psc = nullptr;
  int rc = stream_scratch(c, s, eager, &capturing, &psc);
  if (rc) return rc;
  Scratch& sc = *psc;
  rc = capturing ? KVSEP_OK : acquire(sc, s);
  if (rc) return rc;
  rc = launch_batch_in(c, sc, s, capturing, base, off, len, init, expect, out, first_bad, nbad, count, total_bytes,
                       max_len);
  if (rc) {
    if (!capturing) (void)release(sc, s);  // whatever was enqueued stays ordered before the scratch's next user
    return rc;
  }
  return capturing ? KVSEP_OK : release(sc, s);
}

int launch_batch_body(kvsep_crc32c_ctx* c, Scratch& sc, hipStream_t s, bool capturing, PiecesArgs& a,
                      const void* base, const uint64_t* off, const uint64_t* len, const uint32_t* init,
                      const uint32_t* expect, uint32_t* out, uint64_t* first_bad, uint64_t* nbad, uint64_t count,
                      uint64_t total_bytes, uint64_t max_len);

int launch_batch_in(kvsep_crc32c_ctx* c, Scratch& sc, hipStream_t s, bool capturing, const void* base,
                    const uint64_t* off, const uint64_t* len, const uint32_t* init, const uint32_t* expect,
                    uint32_t* out, uint64_t* first_bad, uint64_t* nbad, uint64_t count, uint64_t total_bytes,
                    uint64_t max_len) {
  PiecesArgs a{};
  if (expect) {
    if (capturing) {  // verdict slots (reserved with the capture set), published by the reduce kernel
      if (!sc.d_verify || sc.cap_vslot < vslots_needed(c))
        return set_err(KVSEP_EINVAL, "verify under capture needs kvsep_crc32c_reserve first");
      a.vslot = sc.d_vslot;
    } else {
      int rc = ensure_verify(sc);
      if (rc) return rc;
      if (sc.vacc_dirty) {
        rc = reset_vacc(sc, s);
        if (rc) return rc;
      }
      a.vacc = vacc_set(sc);  // the accumulators, in their reset state: the kernels publish the verdict
    }
  }
  const int rc = launch_batch_body(c, sc, s, capturing, a, base, off, len, init, expect, out, first_bad, nbad, count,
                                   total_bytes, max_len);
  if (rc && expect && !capturing) sc.vacc_dirty = true;  // a kernel may have posted to the set: reset it first next time
  return rc;
}

int launch_batch_body(kvsep_crc32c_ctx* c, Scratch& sc, hipStream_t s, bool capturing, PiecesArgs& a,
                      const void* base, const uint64_t* off, const uint64_t* len, const uint32_t* init,
                      const uint32_t* expect, uint32_t* out, uint64_t* first_bad, uint64_t* nbad, uint64_t count,
                      uint64_t total_bytes, uint64_t max_len) {
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
    if (count == 0) {  // nothing to check, no CRC kernel: the verdict is "none" (first_bad = ~0, nbad = 0)
      start_words_kernel<<<1, 64, 0, s>>>(nullptr, reinterpret_cast<unsigned long long*>(first_bad),
                                          reinterpret_cast<unsigned long long*>(nbad));
      KVSEP_HIP(hipGetLastError());
    }
  }
  a.expect = expect;
  a.first_bad = reinterpret_cast<unsigned long long*>(first_bad);
  a.nbad = reinterpret_cast<unsigned long long*>(nbad);
  // The verify form's compare runs inside the CRC kernels (and the combine kernel for split blocks): `fused`.  Only
  // the A/B variants of the KVSEP_DIAG tools build fall back to the separate verify_finish_kernel pass.
  bool fused = true;
  if (count == 0) return KVSEP_OK;
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
    if (!sc.d_counter && capturing) return set_err(KVSEP_EINVAL, "graph capture needs kvsep_crc32c_reserve first");
    if (!sc.d_counter) KVSEP_HIP(hipMalloc(&sc.d_counter, 16));
    a.work_counter = sc.d_counter;
  }
  // The start-state words (pstart[0], the guided counter) are written by a kernel of the call, never by a memset node
  // (see crc32c_plan_count_kernel).
  if (planned) {
    int rc = ensure_plan(sc, a.piece_bytes, count, total_bytes, capturing);
    if (rc) return rc;
    a.pstart = sc.d_pstart;
    a.pblk = sc.d_pblk;
    a.partial = sc.d_partial;
    a.max_pieces = sc.cap_pieces;
    const unsigned nb = unsigned((count + 255) / 256);
    crc32c_plan_count_kernel<<<nb, 256, 0, s>>>(len, count, a.piece_bytes, sc.d_counts, sc.d_pstart,
                                                dyn ? sc.d_counter : nullptr);
    KVSEP_HIP(hipGetLastError());
    size_t tb = sc.scan_tmp_bytes;
    KVSEP_HIP(hipcub::DeviceScan::InclusiveSum(sc.d_scan_tmp, tb, sc.d_counts, sc.d_pstart + 1, int(count), s));
    crc32c_plan_expand_kernel<<<nb, 256, 0, s>>>(sc.d_pstart, count, sc.cap_pieces, sc.d_pblk);
    KVSEP_HIP(hipGetLastError());
  } else {
    a.max_pieces = count;
    if (dyn) {
      start_words_kernel<<<1, 64, 0, s>>>(sc.d_counter, nullptr, nullptr);
      KVSEP_HIP(hipGetLastError());
    }
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
    if (nv == 12 && a.hint > kCoopMaxLen) a.hint = kCoopMaxLen;  // its rows cover 4 KiB; longer blocks take its wide path
    if (expect && (nv == 6 || nv == 9 || nv == 10 || nv == 11 || nv == 12 || nv == 20)) {  // the shipped forms' verify
      switch (nv) {
        case 9: crc32c_narrow_kernel<4, true, 512, true, true, LdsFull, true><<<grid, 512, 0, s>>>(a); break;
        case 10: crc32c_narrow_claim_kernel<4, 512, true, true, 8, kClaimLean><<<grid, 512, 0, s>>>(a); break;
        case 11: crc32c_narrow_claim_kernel<4, 512, true, true, 16><<<grid, 512, 0, s>>>(a); break;
        case 12:
          if (init) crc32c_narrow_coop_kernel<true, true><<<grid, 512, 0, s>>>(a);
          else crc32c_narrow_coop_kernel<true, false><<<grid, 512, 0, s>>>(a);
          break;
        case 20: crc32c_narrow_sorted_kernel<4, true, 1024, true><<<grid, 1024, 0, s>>>(a); break;
        default: crc32c_narrow_kernel<4, true, 1024, false, true, LdsFull, true><<<grid, 1024, 0, s>>>(a); break;
      }
    } else {
    // KVSEP_DIAG variants only (the shipped forms are 6, 9, 10, 11, 12 and 20): they post to the caller's words directly, from
    // their own in-kernel compare or from verify_finish_kernel, so those words are set first
    if (expect) {
      KVSEP_HIP(hipMemsetAsync(first_bad, 0xff, 8, s));
      KVSEP_HIP(hipMemsetAsync(nbad, 0, 8, s));
    }
    a.vslot = nullptr;  // (their compare posts to the caller's words, captured or not)
    fused = !expect || diag_self_compare(nv);
    if (!diag_launch_narrow(nv, grid, s, a, count))  // KVSEP_DIAG build only
    switch (nv) {
      case 9: crc32c_narrow_kernel<4, true, 512, true><<<grid, 512, 0, s>>>(a); break;
      case 10: crc32c_narrow_claim_kernel<4, 512, false, true, 8, kClaimLean><<<grid, 512, 0, s>>>(a); break;
      case 11: crc32c_narrow_claim_kernel<4, 512, false, true, 16><<<grid, 512, 0, s>>>(a); break;
      case 12:
        if (init) crc32c_narrow_coop_kernel<false, true><<<grid, 512, 0, s>>>(a);
        else crc32c_narrow_coop_kernel<false, false><<<grid, 512, 0, s>>>(a);
        break;
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
  const unsigned cgrid = unsigned(std::min<uint64_t>((count + 255) / 256, kCombineMaxGrid));
  if (planned) {
    a.vslot_base = grid;  // a captured verify call: the combine kernel's slots follow the CRC kernel's
    if (expect) crc32c_combine_kernel<true><<<cgrid, 256, 0, s>>>(a);
    else crc32c_combine_kernel<false><<<cgrid, 256, 0, s>>>(a);
    KVSEP_HIP(hipGetLastError());
  }
  if (expect && fused && a.vslot) {  // a captured verify call's verdict from its slots
    verify_slots_reduce_kernel<<<1, 256, 0, s>>>(a.vslot, grid + (planned ? cgrid : 0u),
                                                 reinterpret_cast<unsigned long long*>(first_bad),
                                                 reinterpret_cast<unsigned long long*>(nbad));
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
  hipFree(sc.d_vslot);
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
  for (auto& k : c->caps) free_scratch(k->sc);
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
  // a captured graph holds this piece size and the table image it reads (Z_piece): it would replay wrong
  for (auto& k : c->caps)
    if (k->held) return set_err(KVSEP_EINVAL, "set_piece_bytes with captured graphs held: kvsep_crc32c_release_captures first");
  DeviceGuard dg(c->device);
  KVSEP_HIP(dg.err);
  KVSEP_HIP(hipDeviceSynchronize());
  c->piece_bytes = piece_bytes;
  c->piece_auto = false;
  free_plan(c->sc);  // piece tables depend on piece_bytes (device already idle)
  for (auto& sc : c->staging.scratch) free_plan(sc);
  for (auto& k : c->caps) free_plan(k->sc);  // none is held (above); kvsep_crc32c_reserve sizes them again
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
  if (!c || kernel < 0 || kernel > 8) return set_err(KVSEP_EINVAL, "kernel must be 0..8");
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
  // a test hook (csrc/kvsep_testing.h, not the public header): inert unless the test environment asks for it
  const char* on = std::getenv("KVSEP_TEST_HOOKS");
  if (!on || std::strcmp(on, "1") != 0) return set_err(KVSEP_EINVAL, "fault injection needs KVSEP_TEST_HOOKS=1");
  std::lock_guard<std::mutex> g(c->mu);
  c->inject_failure = true;
  return KVSEP_OK;
}

}  // extern "C"

namespace {
// Everything a call of up to count blocks / total_bytes could allocate on this scratch.
int reserve_scratch(kvsep_crc32c_ctx* c, Scratch& sc, uint64_t count, uint64_t total_bytes) {
  if (!sc.d_counter) KVSEP_HIP(hipMalloc(&sc.d_counter, 16));
  int rc = ensure_verify(sc);
  if (rc) return rc;
  if (!sc.last_use) KVSEP_HIP(hipEventCreateWithFlags(&sc.last_use, hipEventDisableTiming));
  rc = ensure_sst(sc, count);
  if (rc) return rc;
  rc = ensure_vslot(sc, vslots_needed(c));
  if (rc) return rc;
  const uint32_t* zp = nullptr;
  return ensure_plan(sc, piece_for(c, total_bytes, &zp), count, total_bytes);
}

// At least n capture sets, each free one sized for the context's largest reservation (held ones stay as their graph
// captured them).
int reserve_capture_sets(kvsep_crc32c_ctx* c, size_t n) {
  while (c->caps.size() < n) c->caps.emplace_back(new CaptureSet());
  for (auto& k : c->caps) {
    if (k->held) continue;
    int rc = reserve_scratch(c, k->sc, c->res_count, c->res_bytes);
    if (rc) return rc;
  }
  return KVSEP_OK;
}
}  // namespace

extern "C" {

int kvsep_crc32c_reserve(kvsep_crc32c_ctx* c, uint64_t count, uint64_t total_bytes) {
  if (!c) return set_err(KVSEP_EINVAL, "null ctx");
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device);
  KVSEP_HIP(dg.err);
  // everything a later call could allocate: on the context's own scratch (eager calls), and on every free capture set
  // (the calls of a graph capture, which must not allocate)
  int rc = reserve_scratch(c, c->sc, count, total_bytes);
  if (rc) return rc;
  c->res_count = std::max(c->res_count, count);
  c->res_bytes = std::max(c->res_bytes, total_bytes);
  return reserve_capture_sets(c, std::max(c->caps.size(), kDefaultCaptureSets));
}

int kvsep_crc32c_reserve_captures(kvsep_crc32c_ctx* c, int nsets) {
  if (!c || nsets < 0 || nsets > 4096) return set_err(KVSEP_EINVAL, "nsets must be 0..4096");
  std::lock_guard<std::mutex> g(c->mu);
  DeviceGuard dg(c->device);
  KVSEP_HIP(dg.err);
  return reserve_capture_sets(c, size_t(nsets));
}

int kvsep_crc32c_release_captures(kvsep_crc32c_ctx* c) {
  if (!c) return set_err(KVSEP_EINVAL, "null ctx");
  std::lock_guard<std::mutex> g(c->mu);
  for (auto& k : c->caps) k->held = false;
  return KVSEP_OK;
}

int kvsep_crc32c_capture_sets(kvsep_crc32c_ctx* c, int* held) {
  if (!c) return set_err(KVSEP_EINVAL, "null ctx");
  std::lock_guard<std::mutex> g(c->mu);
  int h = 0;
  for (auto& k : c->caps) h += k->held ? 1 : 0;
  if (held) *held = h;
  return int(c->caps.size());
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
  // as launch_batch: under capture the capture's own set, no cross-stream events and no allocation
  // (kvsep_crc32c_reserve sizes the SST arrays too)
  bool capturing = false;
  Scratch* psc = nullptr;
  int rc = stream_scratch(c, s, c->sc, &capturing, &psc);
  if (rc) return rc;
  Scratch& sc = *psc;
  rc = capturing ? KVSEP_OK : acquire(sc, s);
  if (rc) return rc;
  rc = ensure_sst(sc, count, capturing);
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
         : nf == 10 || nf == 11 ? "crc32c_narrow_claim_kernel"
         : nf == 12             ? "crc32c_narrow_coop_kernel"
                                : "crc32c_narrow_kernel";
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
