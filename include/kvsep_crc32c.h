/*
 * kvsep_crc32c.h -- C ABI of the MI355X-native CRC-32C-over-blocks engine (libkvsep_crc32c.so).
 *
 * Drop-in boundary for the checksum hot path of Buildings-Lei/kv-separate:
 *   util/crc32c.h:17   uint32_t leveldb::crc32c::Extend(uint32_t init_crc, const char* data, size_t n)
 *   util/crc32c.h:20   Value(data, n) = Extend(0, data, n)
 *   util/crc32c.h:22-38 kMaskDelta / Mask / Unmask
 *   port/port_stdcxx.h:142-152  port::AcceleratedCRC32C(crc, buf, size)  -- the reference's own
 *                      plug point for an accelerated backend (self-test util/crc32c.cc:267-274)
 * plus batched entry points that the reference's call sites would bind to when they hold a batch
 * of independent records/blocks:
 *   db/value_log_reader.cc:86-138  vlog record verify (recovery db/db_impl.cc:485-571, GC :880-951)
 *   db/value_log_writer.cc:46-76   vlog record checksum before Append
 *   table/table_builder.cc:209-232, table/format.cc:99-108  SST block trailers
 *   db/log_writer.cc:84-115, db/log_reader.cc:246-259  MANIFEST fragments (per-type init CRC)
 *
 * All pointers are plain; no framework types cross this boundary.  Results are bit-exact with
 * util/crc32c.cc (checked by tests/ against golden vectors captured from the compiled reference).
 */
#ifndef KVSEP_CRC32C_H_
#define KVSEP_CRC32C_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version.  2 (round 3): kvsep_vlog_verify_host takes *drop_bytes (7 arguments) and kvsep_crc32c_kernel_name
 * takes total_bytes before max_len -- both changed in place from ABI 1, so a caller built against ABI 1 must be
 * rebuilt; check kvsep_abi_version() == KVSEP_ABI_VERSION once at startup.  3 (round 5): kvsep_offload_stats counts
 * only calls at or above the offload threshold (since round 4: host_calls no longer includes the calls below it, which
 * are not counted at all); new entry points for the host legs, topology and host placement; no signature changed.
 * 4 (round 6): graph captures get capture sets of their own (kvsep_crc32c_reserve_captures / _release_captures /
 * _capture_sets); the fault-injection hook left this header (csrc/kvsep_testing.h) and works only under
 * KVSEP_TEST_HOOKS=1; no signature changed.
 * The reference's C++ symbol leveldb::crc32c::Extend is not in this library: it is in the libkvsep_leveldb_abi.so
 * shim. */
#define KVSEP_ABI_VERSION 4
int kvsep_abi_version(void);

#define KVSEP_OK 0
#define KVSEP_EINVAL (-1)  /* bad argument */
#define KVSEP_EHIP (-2)    /* a HIP runtime call failed (message via kvsep_last_error) */
#define KVSEP_ENODEV (-3)  /* no usable gfx950 device */
#define KVSEP_ENOMEM (-4)  /* device or pinned allocation failed */

/* ---------------------------------------------------------------- scalar drop-in
 * Same contract as util/crc32c.h:17 / util/crc32c.cc:276: CRC-32C of A||data[0,n) where
 * init_crc = crc32c(A); n == 0 returns init_crc; any alignment; never fails; reentrant.
 * Dispatch: n >= the offload threshold (kvsep_set_offload_threshold, default 64 MiB) goes through
 * the GPU (pinned staging, H2D, kernel, D2H); smaller inputs use the host leg (VPCLMULQDQ folding on CPUs with
 * AVX-512 carry-less multiply, else SSE4.2 crc32 -- the role google/crc32c plays behind port::AcceleratedCRC32C). */
uint32_t kvsep_crc32c_extend(uint32_t init_crc, const char* data, size_t n);
uint32_t kvsep_crc32c_value(const char* data, size_t n); /* util/crc32c.h:20 */
uint32_t kvsep_crc32c_mask(uint32_t crc);                /* util/crc32c.h:29-32 */
uint32_t kvsep_crc32c_unmask(uint32_t masked_crc);       /* util/crc32c.h:35-38 */
/* port/port_stdcxx.h:142: returns Extend(crc, buf, size); never 0 for the self-test buffer. */
uint32_t kvsep_accelerated_crc32c(uint32_t crc, const char* buf, size_t size);
void kvsep_set_offload_threshold(uint64_t nbytes);
/* A call at/above the threshold while another caller holds the device's GPU leg: wait != 0 queues it for the
 * GPU; wait == 0 (the default) runs it on the host leg at once -- the reference calls Extend from the writer,
 * compaction, GC and reader threads concurrently (db/db_impl.cc:1829-1833), and one PCIe link serves one
 * staged copy at a time while every core can run the host leg. */
void kvsep_set_offload_wait(int wait);
/* Counters of the scalar drop-in's calls at/above the offload threshold since load (any may be null): calls
 * served by the GPU, calls diverted to the host leg because the GPU leg was busy, and calls that the GPU could
 * not serve and that finished on the host (set KVSEP_STRICT_GPU=1 to abort on those instead).  Calls below the
 * threshold are not counted (no shared counter on the small-call path). */
void kvsep_offload_stats(uint64_t* gpu_calls, uint64_t* host_calls, uint64_t* gpu_failures);
/* Host-only CRC, the small-input leg of Extend, on the fastest leg this CPU runs (checked once, at first use):
 * "fold" (x86-64 with AVX-512F + VPCLMULQDQ: 4 x 512-bit accumulators), else "sse42" (x86-64 with SSE4.2: the crc32
 * instruction, 3-way interleaved), else "portable" (any CPU: table-driven, slicing-by-8).  KVSEP_HOST_CRC=sse42 or
 * =portable forces a slower leg.  Exact on every leg; never an illegal instruction on a CPU without the extension. */
uint32_t kvsep_crc32c_extend_host(uint32_t init_crc, const char* data, size_t n);
/* The leg kvsep_crc32c_extend_host runs in this process: "fold", "sse42" or "portable". */
const char* kvsep_crc32c_host_path(void);

/* ---------------------------------------------------------------- device context */
typedef struct kvsep_crc32c_ctx kvsep_crc32c_ctx;

int kvsep_crc32c_ctx_create(int device, kvsep_crc32c_ctx** out);
void kvsep_crc32c_ctx_destroy(kvsep_crc32c_ctx* ctx);
/* Work-item ("piece") size for splitting long blocks; default 128 KiB, min 1 KiB, multiple of 1 KiB. */
int kvsep_crc32c_ctx_set_piece_bytes(kvsep_crc32c_ctx* ctx, uint64_t piece_bytes);
/* 0 = static contiguous runs of work items per wave, 2 = static round-robin items, 1 = guided dynamic (one atomic
 * per run of items), -1 = auto (default): guided when long blocks are split into pieces, else static. */
int kvsep_crc32c_ctx_set_schedule(kvsep_crc32c_ctx* ctx, int dynamic);
/* Kernel of unsplit batches: 0 = auto (default; the narrow kernel for many blocks <= 8-32 KiB, its sorted-window
 * form when the batch is ragged: max_len > 1.25 x total_bytes / count), 1 = always the wide kernel, 2 = the narrow
 * kernel whenever max_len <= 64 KiB, 3 / 4 = as 2 with 16- / 8-wave workgroups, 5 = as 2 in the sorted-window form,
 * 6 = as 2 with each workgroup's contiguous run of groups dealt to its waves by an LDS claim counter (round 4; auto
 * takes it for uniform batches of 32 Ki - 384 Ki blocks <= 4 KiB, 32 Ki - 64 Ki blocks of 4-8 KiB), 7 = as 6 with
 * 16 lanes per block, 4-block groups (auto: uniform batches of >= 4 Ki blocks of 8-12 KiB, up to 512 MiB), 8 = the
 * narrow kernel whose workgroup's 8 waves share each 8-block group (round 6; blocks over 4 KiB take its wide path;
 * auto never picks it: 1.5x the claim kernel's time on 4 KiB blocks).
 * A choice of speed only: every kernel is exact for every block.  No environment variable changes it. */
int kvsep_crc32c_ctx_set_kernel(kvsep_crc32c_ctx* ctx, int kernel);
/* NUMA node the context's host legs are placed on: its pinned staging is allocated, and its copier threads run, on
 * the CPUs of this node that the allocating thread may use.  Default: the node of the device's PCI function
 * (kvsep_device_numa_node); -1 = no placement.  Takes effect for staging not yet allocated (set it before the first
 * host-form call).  The group forms also bind each member's host thread to its member's node for the call. */
int kvsep_crc32c_ctx_set_host_node(kvsep_crc32c_ctx* ctx, int node);
/* Where the context's host legs are: *device_node = the node it places them on (-1: none), *staging_node = the node
 * holding its first pinned staging slot (-1: not allocated yet / unknown), cpus[0..cap) = the CPUs its copier threads
 * are bound to.  Returns the number of those CPUs (0: not bound), or KVSEP_EINVAL. */
int kvsep_crc32c_ctx_host_placement(kvsep_crc32c_ctx* ctx, int* device_node, int* staging_node, int* cpus, int cap);
/* Pre-size scratch so later calls of up to `count` blocks / `total_bytes` bytes do not allocate: the context's own
 * scratch (eager calls) and every free capture set (at least 4 are made).  Required before graph capture; covers the
 * planned, narrow, verify and SST-verify forms. */
int kvsep_crc32c_reserve(kvsep_crc32c_ctx* ctx, uint64_t count, uint64_t total_bytes);
/* Graph capture (hipStreamBeginCapture ... EndCapture, torch.cuda.graph): every call captured into one graph runs on
 * that capture's own capture set -- its piece plan, work counter, SST arrays and verify verdict slots -- held by it until
 * kvsep_crc32c_release_captures.  So graphs of one context may be replayed at the same time on different streams, and
 * a verify graph replayed over itself (two streams, two instantiations) writes identical verdicts.  The calls of ONE
 * graph share its set and must be ordered inside the graph (captured on one stream, or joined); a graph holding
 * planned batches (max_len 0 or above the piece size) must not overlap a replay of itself.  A capture that finds no free
 * set fails with KVSEP_EINVAL when its first call is captured.
 * reserve_captures: at least nsets sets, free ones sized by the largest kvsep_crc32c_reserve so far (held sets keep the
 *   size their graph captured).
 * release_captures: every set free again -- call it only once the graphs captured so far are destroyed (a later
 *   reserve may reallocate a free set).
 * capture_sets: returns the number of sets; *held (nullable) = how many a graph holds. */
int kvsep_crc32c_reserve_captures(kvsep_crc32c_ctx* ctx, int nsets);
int kvsep_crc32c_release_captures(kvsep_crc32c_ctx* ctx);
int kvsep_crc32c_capture_sets(kvsep_crc32c_ctx* ctx, int* held);
/* Kernel timing with HIP events on the caller's stream, around the main CRC kernel only. */
int kvsep_crc32c_ctx_set_timing(kvsep_crc32c_ctx* ctx, int enable);
int kvsep_crc32c_ctx_get_timing(kvsep_crc32c_ctx* ctx, double* total_ms, uint64_t* launches); /* syncs + resets */
/* Name of the main kernel a batch of `count` blocks with these total_bytes / max_len hints runs on
 * ("crc32c_pieces_kernel", "crc32c_narrow_kernel", "crc32c_narrow_claim_kernel" or "crc32c_narrow_sorted_kernel"):
 * the kernel the timing above
 * and a rocprofv3 trace refer to. */
const char* kvsep_crc32c_kernel_name(kvsep_crc32c_ctx* ctx, uint64_t count, uint64_t total_bytes, uint64_t max_len);

/* ---------------------------------------------------------------- batched device form
 * out[i] = Extend(init ? init[i] : 0, base + off[i], len[i]) for i < count.
 * base/off/len/init/out are DEVICE pointers; the call is asynchronous on `stream`
 * (a hipStream_t; NULL = default stream).  Blocks may overlap and sit at any byte alignment.
 * total_bytes ~ sum(len) and max_len (an upper bound on len[i], or 0 if unknown) are performance hints:
 * with max_len <= piece size (128 KiB) the planning pass is skipped and short blocks may run on the narrow
 * kernel.  Results are exact whatever the hints say: a block longer than max_len is checksummed whole by
 * the wide kernel or deferred by the narrow one, and an understated total_bytes makes the kernel fall back
 * to one work item per block.  count <= 2^32 - 1, and <= 2^31 - 1 when the batch is planned (max_len 0 or
 * above the piece size); else KVSEP_EINVAL. */
int kvsep_crc32c_batch_device(kvsep_crc32c_ctx* ctx, void* stream, const void* base, const uint64_t* off,
                              const uint64_t* len, const uint32_t* init, uint32_t* out, uint64_t count,
                              uint64_t total_bytes, uint64_t max_len);

/* Verify form: as above, plus Mask(out[i]) is compared with expected_masked[i] (the stored LE32
 * header word of db/value_log_writer.cc:58-59).  *first_bad (device) receives the lowest mismatching
 * index or UINT64_MAX, *nbad the number of mismatches -- the reader truncates at the first bad
 * record (db/value_log_reader.cc:112-122), so callers keep records [0, *first_bad). */
int kvsep_crc32c_verify_device(kvsep_crc32c_ctx* ctx, void* stream, const void* base, const uint64_t* off,
                               const uint64_t* len, const uint32_t* init, const uint32_t* expected_masked,
                               uint32_t* out, uint64_t* first_bad, uint64_t* nbad, uint64_t count,
                               uint64_t total_bytes, uint64_t max_len);

/* ---------------------------------------------------------------- batched host form
 * Host pointers.  Blocks are gathered into pinned staging, copied H2D, checksummed and the
 * u32 results copied back, double-buffered over two streams; blocking. */
int kvsep_crc32c_batch_host(kvsep_crc32c_ctx* ctx, const uint32_t* init, const char* const* ptr,
                            const uint64_t* len, uint32_t* out, uint64_t count);
/* One contiguous host buffer (a vlog file image or a block buffer headed for pwrite):
 * out[i] = Extend(init?init[i]:0, host_base + off[i], len[i]). Blocking. */
int kvsep_crc32c_batch_host_span(kvsep_crc32c_ctx* ctx, const char* host_base, uint64_t span_bytes,
                                 const uint64_t* off, const uint64_t* len, const uint32_t* init, uint32_t* out,
                                 uint64_t count);

/* ---------------------------------------------------------------- framings (batched call sites)
 * vlog records (db/value_log_writer.cc:46-76, db/value_log_reader.cc:86-138):
 *   [Mask(Value(payload)) LE32][len LE32][payload], back to back from offset 0. */
/* Header walk: fills off/len/stored (nullable) for up to `cap` complete records; returns the number of
 * complete records; a truncated header or payload ends the walk (the reader's eof). */
uint64_t kvsep_vlog_walk(const char* buf, uint64_t n, uint64_t* off, uint64_t* len, uint32_t* stored, uint64_t cap,
                         uint64_t* consumed);
/* Recovery / GC scan: walk + one batched GPU checksum + compare.  *ngood = records before the first checksum
 * mismatch (the reader reports "checksum mismatch" there and stops), *good_bytes = end offset of the last good one,
 * *drop_bytes = the byte count VlogReader reports with that "checksum mismatch" (the bad record's payload length,
 * db/value_log_reader.cc:117-120), 0 when every complete record is intact.  Any output may be null. */
int kvsep_vlog_verify_host(kvsep_crc32c_ctx* ctx, const char* buf, uint64_t n, uint64_t* nrecords, uint64_t* ngood,
                           uint64_t* good_bytes, uint64_t* drop_bytes);
/* Group-commit write side: frames `count` payloads into dst (needs sum(8 + len) bytes, *written). */
int kvsep_vlog_frame_host(kvsep_crc32c_ctx* ctx, const char* const* payload, const uint64_t* len, uint64_t count,
                          char* dst, uint64_t dst_cap, uint64_t* written);
/* log / MANIFEST physical records (db/log_reader.cc:189-272): 32 KiB blocks of [crc LE32][len LE16][type][payload],
 * crc = Mask(Value(type || payload)).  Walk returns off = header + 6 (the type byte), len = 1 + payload length. */
uint64_t kvsep_log_walk(const char* buf, uint64_t n, uint64_t* off, uint64_t* len, uint32_t* stored, uint8_t* type,
                        uint64_t cap);
int kvsep_log_verify_host(kvsep_crc32c_ctx* ctx, const char* buf, uint64_t n, uint8_t* ok, uint64_t cap,
                          uint64_t* nrecords);
/* log / MANIFEST write side (db/log_writer.cc:35-115): appends `count` records to a log of current length
 * dest_length (the writer's block_offset_ = dest_length % 32 KiB, log_writer.cc:27-28), fragmenting each record
 * over 32 KiB blocks as FULL / FIRST / MIDDLE / LAST physical records and zero-filling block trailers of
 * fewer than 7 bytes; every fragment's crc = Mask(Extend(Value(&type, 1), fragment)) comes from ONE batched
 * call.  dst receives the appended bytes; *written = their count (also on KVSEP_EINVAL for a short dst). */
int kvsep_log_frame_host(kvsep_crc32c_ctx* ctx, const char* const* payload, const uint64_t* len, uint64_t count,
                         uint64_t dest_length, char* dst, uint64_t dst_cap, uint64_t* written);
/* What log::Reader::ReadPhysicalRecord returns, given the walk (off as from kvsep_log_walk) and each record's
 * checksum verdict ok[i]: a mismatch drops the rest of its 32 KiB block buffer (db/log_reader.cc:250-258), so
 * that record and every later record of the same block get accept[i] = 0.  Returns the bytes reported as
 * dropped with "checksum mismatch" (header of the bad record to the end of its block, or of the file). */
uint64_t kvsep_log_accept(const uint64_t* off, const uint8_t* ok, uint64_t count, uint64_t n, uint8_t* accept);
/* SST block trailers (table/table_builder.cc:209-232): masked_out[i] = Mask(Extend(Value(block_i), &types[i], 1)),
 * the LE32 word written after the type byte.  Device pointers, async on stream. */
int kvsep_sst_trailers_device(kvsep_crc32c_ctx* ctx, void* stream, const void* base, const uint64_t* off,
                              const uint64_t* len, const uint8_t* types, uint32_t* masked_out, uint64_t count,
                              uint64_t total_bytes, uint64_t max_len);
/* SST block read check (table/format.cc:99-106): the file image holds [block][type][trailer word]; out[i] =
 * Value(block, len + 1) (= Unmask(stored) when intact); *first_bad / *nbad as in kvsep_crc32c_verify_device. */
int kvsep_sst_verify_device(kvsep_crc32c_ctx* ctx, void* stream, const void* file_base, const uint64_t* off,
                            const uint64_t* len, uint32_t* out, uint64_t* first_bad, uint64_t* nbad, uint64_t count,
                            uint64_t total_bytes, uint64_t max_len);
/* Host-resident forms of the two above, for blocks the way TableBuilder::WriteRawBlock (table/table_builder.cc:209-232)
 * and ReadBlock (table/format.cc:73-108) hold them: in host memory.  Both go through the pinned staging pipeline of
 * the host forms; blocking.
 *   trailers: block[i] / len[i] host pointers, types[i] the compression type byte; masked_out[i] =
 *             Mask(Extend(Value(block_i), &types[i], 1)).
 *   verify:   `file` is an SST file image in host memory ([block][type][trailer word] at each handle off[i] / len[i];
 *             KVSEP_EINVAL if a handle leaves no room for its 5-byte trailer, format.cc:84-87); out[i] =
 *             Value(block, len + 1); *first_bad = lowest i whose out[i] != Unmask(stored word) (UINT64_MAX if none),
 *             *nbad their number -- each such block is what ReadBlock reports as "block checksum mismatch". */
int kvsep_sst_trailers_host(kvsep_crc32c_ctx* ctx, const char* const* block, const uint64_t* len, const uint8_t* types,
                            uint32_t* masked_out, uint64_t count);
int kvsep_sst_verify_host(kvsep_crc32c_ctx* ctx, const char* file, uint64_t n, const uint64_t* off, const uint64_t* len,
                          uint32_t* out, uint64_t* first_bad, uint64_t* nbad, uint64_t count);

/* ---------------------------------------------------------------- several GPUs in one process
 * Blocks are independent, so a batch is cut into contiguous block ranges balanced by bytes and each range runs on
 * its own device; payload never crosses between GPUs, only the u32 results come back (into ONE array).  For a
 * single KVDB process scanning whole vlogs (GC db/db_impl.cc:880-951, recovery :485-571) on every GPU it has. */
/* bounds[0..parts]: part p = blocks [bounds[p], bounds[p+1]), each ~sum(len)/parts bytes (the cut nearest to each
 * p/parts point of the prefix sum of len).  Host arrays; no device needed. */
int kvsep_crc32c_partition(const uint64_t* len, uint64_t count, int parts, uint64_t* bounds);
typedef struct kvsep_crc32c_group kvsep_crc32c_group;
/* One context (and stream) per listed device; a device may be listed twice (two independent contexts on it). */
int kvsep_crc32c_group_create(const int* devices, int ndev, kvsep_crc32c_group** out);
void kvsep_crc32c_group_destroy(kvsep_crc32c_group* g);
int kvsep_crc32c_group_size(kvsep_crc32c_group* g);
kvsep_crc32c_ctx* kvsep_crc32c_group_ctx(kvsep_crc32c_group* g, int i); /* member i's context (tuning knobs) */
/* kvsep_crc32c_batch_host_span over the whole group: part i through member i's pinned staging on its own PCIe link,
 * one host thread per member; blocking. */
int kvsep_crc32c_group_batch_host_span(kvsep_crc32c_group* g, const char* host_base, uint64_t span_bytes,
                                       const uint64_t* off, const uint64_t* len, const uint32_t* init, uint32_t* out,
                                       uint64_t count);
/* ... plus Mask(out[i]) == expected_masked[i]: *first_bad = lowest mismatching index (UINT64_MAX if none), *nbad. */
int kvsep_crc32c_group_verify_host_span(kvsep_crc32c_group* g, const char* host_base, uint64_t span_bytes,
                                        const uint64_t* off, const uint64_t* len, const uint32_t* init,
                                        const uint32_t* expected_masked, uint32_t* out, uint64_t* first_bad,
                                        uint64_t* nbad, uint64_t count);
/* kvsep_vlog_verify_host with the checksums spread over the group. */
int kvsep_vlog_verify_host_group(kvsep_crc32c_group* g, const char* buf, uint64_t n, uint64_t* nrecords,
                                 uint64_t* ngood, uint64_t* good_bytes, uint64_t* drop_bytes);
/* Device-resident shards: member i's blocks live on ITS device (base[i], off[i], len[i], init[i] (nullable array or
 * entries), out[i] are device pointers there, count[i] blocks, total_bytes[i] / max_len[i] hints as in
 * kvsep_crc32c_batch_device).  Runs every shard on its member's stream and returns when all are done. */
int kvsep_crc32c_group_batch_device(kvsep_crc32c_group* g, const void* const* base, const uint64_t* const* off,
                                    const uint64_t* const* len, const uint32_t* const* init, uint32_t* const* out,
                                    const uint64_t* count, const uint64_t* total_bytes, const uint64_t* max_len);
/* ... verify form: shard i's block k is global block index_base[i] + k; *first_bad = the lowest global mismatching
 * index over all shards (UINT64_MAX if none), *nbad = the total -- the reduction SURVEY §8e puts on RCCL between
 * ranks, done here between the members of one process.  expected_masked may be NULL (then = batch_device). */
int kvsep_crc32c_group_verify_device(kvsep_crc32c_group* g, const void* const* base, const uint64_t* const* off,
                                     const uint64_t* const* len, const uint32_t* const* init,
                                     const uint32_t* const* expected_masked, uint32_t* const* out,
                                     const uint64_t* index_base, const uint64_t* count, const uint64_t* total_bytes,
                                     const uint64_t* max_len, uint64_t* first_bad, uint64_t* nbad);

/* ---------------------------------------------------------------- topology and host placement (round 5)
 * Which physical GPU a caller runs on, and the NUMA node its host legs belong on.  sysfs is read under
 * $KVSEP_SYSFS_ROOT (default /sys). */
/* PCI bus ID of a device ("0000:75:00.0", lower case, as sysfs spells it) into buf (len >= 13). */
int kvsep_device_pci_bus_id(int device, char* buf, int len);
/* NUMA node of a PCI function / of a device (sysfs numa_node), -1 when unknown. */
int kvsep_pci_numa_node(const char* pci_bus_id);
int kvsep_device_numa_node(int device);
/* CPUs of a NUMA node (sysfs cpulist) into cpus[0..cap); returns how many it has (0: unknown node). */
int kvsep_numa_node_cpus(int node, int* cpus, int cap);
/* Binds every thread of the calling process to the CPUs of `node` that the calling thread may run on, and makes
 * `node` the calling thread's preferred memory node (its later allocations, pinned host buffers included, land there
 * first).  Returns the number of CPUs bound to; 0 (nothing changed) for an unknown node or one that shares no CPU
 * with the current affinity.  For a process that drives one GPU (a bench rank): call it right after selecting the
 * device, before allocating pinned memory. */
int kvsep_bind_process_numa(int node);
/* NUMA node of the page holding p (faulted in if never touched), -1 if unknown. */
int kvsep_host_page_node(const void* p);

/* Pinned (page-locked) host memory for file images: read a vlog / SST file straight into it and the
 * host-span entry points DMA from it directly, without the staging memcpy.  NULL on failure. */
void* kvsep_host_alloc_pinned(uint64_t bytes);
void kvsep_host_free_pinned(void* p);

/* ---------------------------------------------------------------- support
 * Synthetic data: byte i of the stream is byte (i&7) of splitmix64 word (i>>3) of `seed`
 * (word j = mix(seed + (j+1)*0x9E3779B97F4A7C15)); writes bytes [stream_offset, +nbytes) to dst. */
int kvsep_fill_splitmix64_device(void* stream, void* dst, uint64_t nbytes, uint64_t seed, uint64_t stream_offset);
/* Read-only streaming kernel over [src, src+nbytes) (16-B loads, XOR-reduced into *sink):
 * the attainable HBM-read ceiling the CRC kernel is compared with. */
int kvsep_stream_read_device(kvsep_crc32c_ctx* ctx, void* stream, const void* src, uint64_t nbytes, uint32_t* sink);
const char* kvsep_last_error(void);
const char* kvsep_build_info(void);
int kvsep_device_count(void);

#ifdef __cplusplus
}  /* extern "C" */
#endif
#endif /* KVSEP_CRC32C_H_ */
