#!/usr/bin/env python3
"""bench.py -- CRC32C GiB/s, device-resident, batched 1 MiB blocks (BASELINE.json metric).

One step = one pass of the CRC engine (libkvsep_crc32c, C ABI) over one batch that already sits in HBM:
config 3 of BASELINE.json, 65,536 x 1 MiB blocks (64 GiB) per GPU (`--config 3a`, default).  Other configs:
  3b  the vlog-framed variant (1,048,609-B payloads at 8 + i*(8+len): odd offsets)
  2   65,536 x 4 KiB SST blocks
  4   the ragged Zipf batch: ONE global batch of N x 2^20 blocks cut into byte-balanced contiguous block ranges
      (kvsep_crc32c_partition), one per rank -- at N = 1 exactly config 4
  5   the 512 GiB vlog (524,288 x 1,048,609-B records) split over the N ranks (strong scaling): each rank owns
      8/N distinct 64 GiB slices; with more than one, every pass regenerates its slice in HBM at its true stream
      offset outside the timed region, so all 512 GiB checksummed are distinct data
N > 1: one process per GPU, each rank checksums its own shard; no data-path collective.  The ranks come from torchrun,
or -- `bench.py --gpus N` with no WORLD_SIZE in the environment -- from bench.py itself (launch_ranks), over RCCL.

Outside the timed region: RCCL all-gather of every rank's u32 results (4 B per block) and a check of EVERY block of
every rank against the reference's whole-batch outputs (tests/golden/full_cfg*.u32 per block at up to 8 ranks;
config 4 beyond its first 2^20 blocks by the reference's per-rank digests, full_cfg4_ranks.json -- all computed by the
compiled util/crc32c.cc); the read-only streaming ceiling; the host
round-trip rate; and -- rank 0 at N = 1 -- the compiled reference's CPU throughput on a bounded sample
(cpu_baseline) at 1 thread and at every core this process may run on.
"""
from __future__ import annotations

import argparse
import ctypes
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "kv-separate_amd"))

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

import kvsep  # noqa: E402
from kvsep import shard  # noqa: E402
from kvsep import workloads as W  # noqa: E402

GIB = float(1 << 30)
HBM_PEAK_GBPS = 8000.0  # MI355X spec HBM3E peak (MI355X_MICROARCH.md: 8.0 TB/s)
GOLDEN = os.path.join(ROOT, "tests", "golden")
METRIC = "CRC32C GiB/s device-resident, batched 1 MiB blocks, 1/2/4/8 MI355X"


def log(*a):
    print(*a, file=sys.stderr, flush=True)


_CFG4 = {}


def _cfg4_global(world):
    """Config 4 over `world` ranks: one packed batch of world x 2^20 Zipf blocks (its first 2^20 ARE config 4)."""
    if world not in _CFG4:
        glen = W.zipf_lengths(world * W.CFG4_BLOCKS)
        goff = np.zeros(glen.size, np.uint64)
        goff[1:] = np.cumsum(glen[:-1], dtype=np.uint64)
        _CFG4[world] = (goff, glen)
    return _CFG4[world]


def _cfg4_digest(world, rank):
    """The reference's crc_of_crcs over this rank's block range of the N-rank config-4 batch
    (tests/golden/full_cfg4_ranks.json, make_fullsize_golden.py): 8 Mi blocks of u32s are too many to commit."""
    path = os.path.join(GOLDEN, "full_cfg4_ranks.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        parts = json.load(f)["ranks"].get(str(world))
    return parts[rank] if parts else None


class Plan:
    """What this rank checksums: a local block layout over one buffer, and one (stream_base, index_base) per pass
    -- the global stream offset of the buffer's first byte and the global index of its first block."""

    def __init__(self, cfg: str, world: int, rank: int):
        self.cfg = cfg
        self.passes = [(0, 0)]
        self.golden = None  # file of the reference's per-block CRCs of the global batch, indexed globally
        self.digest = None  # {lo, hi, crc_of_crcs}: the reference's digest of this rank's block range
        if cfg in ("2", "3a", "3b"):
            if cfg == "2":
                self.off, self.ln = W.cfg2_layout()
                self.seed, self.golden = W.SEED, "full_cfg2.u32"
                self.desc = "65536 x 4 KiB SST blocks (config 2)"
            elif cfg == "3a":
                self.off, self.ln = W.cfg3_layout()
                self.seed, self.golden = W.SEED + 1, "full_cfg3a.u32"
                self.desc = "65536 x 1 MiB blocks, 16-B aligned (config 3, variant A)"
            else:
                self.off, self.ln = W.cfg3_layout(vlog=True)
                self.seed, self.golden = W.SEED + 1, "full_cfg5.u32"  # rank r = slice r of the 512 GiB vlog
                self.desc = "65536 x 1,048,609-B vlog payloads at 8 + i*(8+len) (config 3, variant B)"
            span = int(self.off[-1] + self.ln[-1])
            self.passes = [(shard.stream_offset(rank, span), rank * self.off.size)]
            self.scaling = "weak"
        elif cfg == "4":
            goff, glen = _cfg4_global(world)
            self.off, self.ln, base, ib = shard.partition_layout(goff, glen, world, rank)
            self.passes = [(base, ib)]
            self.seed, self.golden = W.SEED + 2, "full_cfg4.u32"
            self.digest = _cfg4_digest(world, rank)
            self.desc = (f"{world} x 1,048,576 Zipf(1.1) blocks, 32 B - 4 MiB, one batch cut into byte-balanced block "
                         f"ranges (config 4)")
            self.scaling = "weak"
        elif cfg == "5":
            if 8 % world:
                raise SystemExit("--config 5 needs 1, 2, 4 or 8 ranks")
            per = 8 // world
            self.off, self.ln = W.cfg3_layout(vlog=True)
            span = int(self.off[-1] + self.ln[-1])
            slices = [rank * per + p for p in range(per)]
            self.passes = [(s * span, s * self.off.size) for s in slices]
            self.seed, self.golden = W.SEED + 1, "full_cfg5.u32"
            self.desc = (f"512 GiB vlog batch (524,288 x 1,048,609-B records) over {world} GPU(s): {per} distinct "
                         f"64 GiB slice(s) per GPU (config 5)")
            self.scaling = "strong"
        else:
            raise SystemExit(f"unknown config {cfg}")
        self.count = int(self.off.size)
        self.useful = int(self.ln.sum())
        self.span = int(self.off[-1] + self.ln[-1]) if self.count else 0


def to_dev_u64(a, dev):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)


def load_oracle():
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from conftest import load_oracle as _lo  # test infrastructure: the checker / CPU baseline only
    return _lo()


class RefBatch:
    """oracle/_ref/libref_crc32c.so: the reference's own util/crc32c.cc compiled -O3 (oracle/Makefile)
    plus a threaded batch driver (oracle/ref_shim.cc).  Built in the dev container, shipped as a binary."""

    PATH = os.path.join(ROOT, "oracle", "_ref", "libref_crc32c.so")

    def __init__(self):
        self.lib = ctypes.CDLL(self.PATH)
        self.lib.ref_crc32c_batch.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_int]
        self.lib.ref_crc32c_batch.restype = ctypes.c_int

        f = self.lib.ref_crc32c_timed_local
        f.restype = ctypes.c_int
        f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_size_t, ctypes.c_int, ctypes.c_void_p, ctypes.c_double,
                                              ctypes.c_void_p, ctypes.c_void_p]

    def batch(self, buf, off, length, init=None, threads=1):
        out = np.zeros(off.size, dtype=np.uint32)
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint64)
        assert self.lib.ref_crc32c_batch(buf.ctypes.data, off.ctypes.data, length.ctypes.data, None,
                                         out.ctypes.data, off.size, threads) == 0
        return out

    def timed_local(self, buf, off, length, cpus, seconds):
        """ref_crc32c_timed_local: len(cpus) threads, thread t pinned to cpus[t], each on its own first-touched copy of
        its byte-balanced block range, repeated passes for `seconds` -> (bytes, elapsed s)."""
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint64)
        c = np.ascontiguousarray(cpus, dtype=np.int32)
        b, t = ctypes.c_uint64(), ctypes.c_double()
        assert self.lib.ref_crc32c_timed_local(buf.ctypes.data, off.ctypes.data, length.ctypes.data, off.size, c.size,
                                               c.ctypes.data, seconds, ctypes.byref(b), ctypes.byref(t)) == 0
        return b.value, t.value


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _read(path):
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return None


def _cpulist(text):
    out = []
    for part in (text or "").split(","):
        if "-" in part:
            a, b = part.split("-")
            out.extend(range(int(a), int(b) + 1))
        elif part.strip():
            out.append(int(part))
    return out


def cpu_quota():
    """The cgroup CPU limit this process runs under: cgroup v2 cpu.max ("quota period" or "max period"), else v1
    cfs_quota_us / cfs_period_us -> (raw text, CPUs or None when unlimited)."""
    v2 = _read("/sys/fs/cgroup/cpu.max")
    if v2:
        q, per = (v2.split() + ["100000"])[:2]
        return v2, (None if q == "max" else int(q) / int(per))
    q, per = _read("/sys/fs/cgroup/cpu/cpu.cfs_quota_us"), _read("/sys/fs/cgroup/cpu/cpu.cfs_period_us")
    if q and per:
        return f"cfs_quota_us={q} cfs_period_us={per}", (None if int(q) < 0 else int(q) / int(per))
    return None, None


def numa_nodes():
    """{node: [cpus]} from /sys/devices/system/node (one node "0" with every CPU when absent)."""
    base = "/sys/devices/system/node"
    nodes = {}
    try:
        for d in sorted(os.listdir(base)):
            if d.startswith("node") and d[4:].isdigit():
                nodes[int(d[4:])] = _cpulist(_read(os.path.join(base, d, "cpulist")))
    except OSError:
        pass
    return nodes or {0: list(range(os.cpu_count() or 1))}


def spread_cpus(allowed):
    """The CPUs this process may run on, ordered so that any prefix spreads over the NUMA nodes (round-robin) and
    takes one hardware thread of each physical core before any SMT sibling."""
    node_of = {c: n for n, cs in numa_nodes().items() for c in cs}
    per_node = {}
    for c in sorted(allowed):
        sib = _cpulist(_read(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list")) or [c]
        rank = sorted(sib).index(c) if c in sib else 0  # 0: the core's first hardware thread
        per_node.setdefault(node_of.get(c, 0), []).append((rank, c))
    queues = [sorted(v) for _, v in sorted(per_node.items())]
    order = []
    while any(queues):
        for q in queues:
            if q:
                order.append(q.pop(0)[1])
    return order, node_of


def place_rank(device: int, mode: str) -> dict:
    """NUMA placement of this rank's host legs (round 5): every thread of the process onto the CPUs of the NUMA node of
    its GPU's PCI function, and that node the main thread's preferred memory node, so the pinned round-trip image and
    the library's pinned staging (which its context also places there, kvsep_crc32c_ctx_set_host_node) sit next to
    the GPU's PCIe root.  Called right after selecting the device and before any pinned allocation; an affinity call
    in this process, never a re-exec.  -> what was done, for the line."""
    info = {"numa_node": None, "bound_cpus": 0, "mode": mode}
    try:
        info["numa_node"] = kvsep.device_numa_node(device)
        if mode != "off" and info["numa_node"] is not None and info["numa_node"] >= 0:
            info["bound_cpus"] = kvsep.bind_process_numa(info["numa_node"])
    except Exception as e:  # placement is an optimisation: the line never depends on it
        info["error"] = str(e)[:200]
    return info


def rank_record(rank, local, device, placement, kern_avg_ms, own_s, t_start, t_end, nbytes, kernel_name,
                launch_bytes=0):
    """This rank's entry of the line's `per_rank`: which physical GPU (PCI bus ID), where its host legs run (NUMA node,
    CPU affinity), and its own timing -- kernel time by HIP events, elapsed from the start barrier to its own last
    synchronize (before the end barrier), the GiB/s that gives, and wall-clock start / end stamps (one host clock)."""
    rec = {"rank": rank, "local_rank": local, "device": device, "pid": os.getpid(),
           "pci_bus_id": None, "numa_node": placement.get("numa_node"), "bound_cpus": placement.get("bound_cpus"),
           "cpu_affinity": kvsep.format_cpulist(os.sched_getaffinity(0)),
           "kernel": kernel_name, "kernel_avg_ms": None if kern_avg_ms is None else round(kern_avg_ms, 5),
           "elapsed_s": None if own_s is None else round(own_s, 6),
           "GiBps": None if not own_s else round(nbytes / GIB / own_s, 3),
           "kernel_GBps": round(launch_bytes / (kern_avg_ms * 1e-3) / 1e9, 1) if kern_avg_ms and launch_bytes else None,
           "t_start": t_start, "t_end": t_end}
    if device is not None:
        try:
            rec["pci_bus_id"] = kvsep.pci_bus_id(device)
        except Exception as e:
            rec["pci_bus_id_error"] = str(e)[:120]
    return rec


def cpu_baseline(oracle, data_dev, off, ln, sample_blocks, thread_counts, seconds, allowed=None):
    """CPU CRC on host cores over a sample of the batch: the compiled reference (kind "reference") when oracle/_ref
    was built, else the oracle restatement (kind "port"), at each thread count in `thread_counts`.  The reference runs
    through ref_crc32c_timed_local: threads pinned spread over the NUMA nodes (spread_cpus), each checksumming its own
    first-touched copy of its byte range, so every thread reads memory local to it."""
    idx = np.linspace(0, off.size - 1, sample_blocks).astype(np.int64)
    lens = ln[idx]
    host = np.empty(int(lens.sum()), dtype=np.uint8)
    hoff = np.zeros(sample_blocks, dtype=np.uint64)
    pos = 0
    for k, i in enumerate(idx):  # gather the sampled blocks to host memory (untimed)
        n = int(ln[i])
        host[pos:pos + n] = data_dev[int(off[i]):int(off[i]) + n].cpu().numpy()
        hoff[k] = pos
        pos += n
    out = {}
    impl, kind = oracle, "port"
    if os.path.exists(RefBatch.PATH):
        impl, kind = RefBatch(), "reference"
        order, node_of = spread_cpus(allowed or os.sched_getaffinity(0))
        impl.batch(host, hoff[:8], lens[:8], threads=1)  # warm tables
        for t in thread_counts:
            cpus = order[:t] if t <= len(order) else (order * (t // len(order) + 1))[:t]
            nb, dt = impl.timed_local(host, hoff, lens, cpus, seconds)
            out[t] = (nb / GIB / dt, nb, dt, sorted({node_of.get(c, 0) for c in cpus}))
        return out, host, hoff, lens, idx, kind
    for t in thread_counts:
        sub = sample_blocks if t > 1 else max(1, sample_blocks // 4)
        sb = int(lens[:sub].sum())
        impl.batch(host, hoff[:min(sub, 8)], lens[:min(sub, 8)], threads=1)  # warm tables
        # repeated passes over the host sample (GiBs: no cache holds it) until `seconds` of CPU work
        passes, t0 = 0, time.perf_counter()
        while True:
            impl.batch(host, hoff[:sub], lens[:sub], threads=t)
            passes += 1
            dt = time.perf_counter() - t0
            if dt >= seconds:
                break
        out[t] = (passes * sb / GIB / dt, passes * sb, dt, None)
    return out, host, hoff, lens, idx, kind


def host_leg_path() -> str:
    """Which host leg kvsep_crc32c_extend_host runs here (crc32c_host.cpp fold_available): the VPCLMULQDQ fold on
    CPUs with AVX-512F + VPCLMULQDQ (unless KVSEP_HOST_CRC=sse42), else the SSE4.2 3-way crc32q loop."""
    flags = set()
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("flags"):
                flags = set(line.split(":", 1)[1].split())
                break
    except OSError:
        pass
    fold = {"avx512f", "vpclmulqdq", "pclmulqdq", "sse4_2"} <= flags and os.environ.get("KVSEP_HOST_CRC") != "sse42"
    return ("VPCLMULQDQ fold (4 x 512-bit accumulators, 256 B per round) + crc32q tail" if fold
            else "SSE4.2 crc32q, 3-way interleaved")


def host_leg_rate(host, hoff, lens, threads, seconds):
    """Informational: the library's own host leg (the drop-in's small-input path, i.e. the "accelerated" CPU path
    google/crc32c would give the reference) over the same host sample; GiB/s."""
    fn = kvsep.lib().kvsep_crc32c_extend_host
    base = host.ctypes.data
    items = [(base + int(o), int(n)) for o, n in zip(hoff, lens)]
    parts = [items[t::threads] for t in range(threads)]
    fn(0, items[0][0], min(items[0][1], 4096))  # warm

    def work(part, stop_at, acc):
        while True:
            for a, n in part:
                fn(0, a, n)
            acc.append(sum(n for _, n in part))
            if time.perf_counter() >= stop_at:
                return

    t0 = time.perf_counter()
    accs = [[] for _ in range(threads)]
    ths = [threading.Thread(target=work, args=(parts[t], t0 + seconds, accs[t])) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    return sum(sum(a) for a in accs) / GIB / dt


def roundtrip_setup(ctx, nbytes_target: int):
    """A pinned host vlog image (config 3b records) and its device-resident reference results."""
    off, ln = W.cfg3_layout(vlog=True, count=max(1, nbytes_target // (W.VLOG_PAYLOAD + 8)))
    span = int(off[-1] + ln[-1])
    buf = torch.empty(span, dtype=torch.uint8, pin_memory=True)
    dev = torch.empty(span, dtype=torch.uint8, device="cuda")
    kvsep.fill_splitmix64(dev.data_ptr(), span, 77, 0)
    buf.copy_(dev)
    ref = torch.zeros(off.size, dtype=torch.int32, device="cuda")  # same records, device-resident path
    ctx.batch_device(dev.data_ptr(), to_dev_u64(off, dev.device), to_dev_u64(ln, dev.device), ref,
                     total_bytes=int(ln.sum()), max_len=int(ln.max()))
    torch.cuda.synchronize()
    ref = ref.cpu().numpy().view(np.uint32)
    del dev
    arr = buf.numpy()
    ctx.batch_host_span(arr, off, ln)  # warm staging
    return buf, arr, off, ln, ref


def roundtrip_time(ctx, state, reps=3):
    """Pinned host image -> H2D -> CRC kernel -> D2H of the u32 results (two streams): seconds per pass."""
    _, arr, off, ln, ref = state
    t0 = time.perf_counter()
    for _ in range(reps):
        res = ctx.batch_host_span(arr, off, ln)
    return (time.perf_counter() - t0) / reps, bool(np.array_equal(res, ref))


def check_results(plan_all, results, oracle):
    """Every rank's u32 results (gathered), rank 0, untimed: per block against the reference's whole-batch outputs
    where the golden file covers the block's global index (configs 2 / 3a / 3b / 5 at up to 8 ranks, config 4's first
    2^20 blocks); where it does not, the rank's whole range against the reference's digest of it (config 4 at N > 1);
    an oracle recompute of 16 sampled blocks per (rank, pass) only where neither exists."""
    checked = by_digest = mism = bad_ranges = sampled = total = 0
    gold_cache = {}
    for plan, res in zip(plan_all, results):
        k = plan.count
        gold = None
        if plan.golden:
            gold = gold_cache.setdefault(plan.golden, np.fromfile(os.path.join(GOLDEN, plan.golden), dtype="<u4"))
        for p, (base, ib) in enumerate(plan.passes):
            got = res[p * k:(p + 1) * k]
            total += k
            n_gold = 0 if gold is None else max(0, min(k, gold.size - ib))
            if n_gold:
                mism += int(np.count_nonzero(got[:n_gold] != gold[ib:ib + n_gold]))
                checked += n_gold
            if n_gold == k:
                continue
            dg = plan.digest
            if dg is not None and dg["lo"] == ib and dg["hi"] == ib + k:
                by_digest += k - n_gold
                if shard.crc_of_crcs(got, kvsep.extend_host) != dg["crc_of_crcs"]:
                    bad_ranges += 1
                continue
            rest = np.arange(n_gold, k)
            for i in rest[np.linspace(0, rest.size - 1, min(16, rest.size)).astype(np.int64)] if rest.size else []:
                d = kvsep.splitmix64_bytes(int(plan.ln[i]), plan.seed, base + int(plan.off[i]))
                mism += int(oracle.extend_addr(0, d.ctypes.data, d.size) != int(got[i]))
                sampled += 1
    return {"blocks_total": total, "blocks_checked_vs_reference": checked,
            "blocks_checked_vs_reference_digest": by_digest, "blocks_sampled_vs_oracle": sampled,
            "every_block_checked": checked + by_digest == total, "mismatches": mism,
            "mismatching_digest_ranges": bad_ranges}


def live_pmc_traffic(args, timeout_s=240):
    """HBM bytes per launch of the CRC kernel, measured on THIS box in this run: one separate
    `rocprofv3 --pmc FETCH_SIZE --kernel-trace` pass (counters in their own run, MI355X_MICROARCH.md HBM section) of
    the same config, as a child process after the timed region and after this process freed its batch; gfx950
    FETCH_SIZE counts half the bytes of a wide coalesced stream, so bytes = FETCH_SIZE (KB) x 1024 x 2, averaged over
    the CRC kernel's dispatches of the pass.  -> (bytes per launch, dispatches, None) or (None, 0, reason)."""
    import csv
    import shutil
    import statistics
    import subprocess
    import tempfile
    exe = shutil.which("rocprofv3") or "/opt/rocm/bin/rocprofv3"
    if not os.path.exists(exe):
        return None, 0, "rocprofv3 not found"
    d = tempfile.mkdtemp(prefix="kvsep_pmc_", dir="/tmp")
    cmd = ["timeout", "-s", "KILL", str(timeout_s), exe, "--pmc", "FETCH_SIZE", "--kernel-trace", "-d", d, "-o", "pmc",
           "--output-format", "csv", "--", sys.executable, os.path.abspath(__file__), "--config", args.config,
           "--steps", "3", "--warmup", "1", "--no-cpu", "--roundtrip-gib", "0", "--pmc-live", "off", "--launch", "eager",
           "--schedule", args.schedule, "--form", args.form] + \
          (["--piece-kib", str(args.piece_kib)] if args.piece_kib else []) + \
          (["--no-plan-hint"] if args.no_plan_hint else [])
    env = {k: v for k, v in os.environ.items()
           if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "GROUP_RANK", "GROUP_WORLD_SIZE",
                        "ROLE_RANK", "ROLE_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT", "TORCHELASTIC_RUN_ID")}
    env["TMPDIR"] = "/tmp"
    try:
        r = subprocess.run(cmd, cwd="/tmp", env=env, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE,
                           timeout=timeout_s + 30)
        if r.returncode:
            tail = r.stderr.decode(errors="replace").strip().splitlines()[-1:] or [""]
            return None, 0, f"rocprofv3 pass exited {r.returncode}: {tail[0][:200]}"
        vals = {}
        with open(os.path.join(d, "pmc_counter_collection.csv")) as fh:
            for row in csv.DictReader(fh):
                if row["Counter_Name"] == "FETCH_SIZE" and ("crc32c_pieces_kernel" in row["Kernel_Name"] or
                                                            "crc32c_narrow" in row["Kernel_Name"]):
                    vals[row["Dispatch_Id"]] = vals.get(row["Dispatch_Id"], 0.0) + float(row["Counter_Value"])
        if not vals:
            return None, 0, "no CRC kernel dispatch in the pass"
        return int(statistics.mean(vals.values()) * 1024 * 2), len(vals), None
    except Exception as e:  # the headline line never depends on the profiler
        return None, 0, f"rocprofv3 pass failed: {e}"
    finally:
        shutil.rmtree(d, ignore_errors=True)


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` without an outside launcher: start N ranks of this script as child processes (one per GPU,
    RANK / LOCAL_RANK / WORLD_SIZE / MASTER_* in their environment, rendezvous on 127.0.0.1), wait for all of them
    and return the worst exit status.  Runs before this process makes any GPU call (it never initialises the GPU, so
    the children are plain subprocesses, not an exec).  A rank that fails takes the others down."""
    import signal
    import socket
    import subprocess
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      start_new_session=True))
    worst = 0
    live = set(range(n))
    while live:
        for r in sorted(live):
            rc = procs[r].poll()
            if rc is None:
                continue
            live.discard(r)
            if rc != 0:
                log(f"[launcher] rank {r} exited {rc}; stopping the other ranks")
                worst = worst or (rc if rc > 0 else 128 - rc)
                for q in live:
                    try:
                        os.killpg(procs[q].pid, signal.SIGTERM)
                    except ProcessLookupError:
                        pass
        time.sleep(0.2)
    return worst


def line_failures(line: dict, world: int, same_device: bool) -> list:
    """Why a printed line is not a clean measurement: bench.py prints the line and then exits
    non-zero when any of these holds, so a driver that takes its rc and value from this process never records a
    wrong-result or mis-placed run as clean.  A checksum mismatch is Corruption in the reference
    (/root/reference/db/value_log_reader.cc:112-122), never a number."""
    bad = []
    parity = line.get("parity")
    if parity is not None and not parity.get("all_blocks_match"):
        bad.append(f"parity: {parity.get('mismatches')} mismatching blocks, "
                   f"{parity.get('mismatching_digest_ranges')} mismatching digest ranges")
    verdict = line.get("verify")
    if verdict is not None and not verdict.get("ok"):
        bad.append(f"verify: first_bad {verdict.get('first_bad')} nbad {verdict.get('nbad')}, expected "
                   f"{verdict.get('expected_first_bad')} / {verdict.get('expected_nbad')}")
    if line.get("host_roundtrip_parity") is False:
        bad.append("host round trip: results differ from the device-resident run")
    per_rank = line.get("per_rank") or []
    got = sorted(r.get("rank") for r in per_rank if isinstance(r, dict) and r.get("rank") is not None)
    if got != list(range(world)):
        bad.append(f"per-rank records: got ranks {got} of {world}")
    summary = line.get("per_rank_summary") or {}
    if world > 1 and not same_device and not summary.get("distinct_devices"):
        bad.append(f"{world} ranks but not on distinct devices (PCI bus IDs {summary.get('pci_bus_ids')}); a "
                   f"same-device rehearsal sets KVSEP_BENCH_SAME_DEVICE")
    return bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="3a", choices=["3a", "3b", "2", "4", "5"],
                    help="BASELINE.json config; 5 = the 512 GiB vlog batch split over the ranks (strong scaling)")
    ap.add_argument("--piece-kib", type=int, default=0, help="work-item size (0 = library default)")
    ap.add_argument("--schedule", default="default", choices=["default", "static", "dynamic"])
    ap.add_argument("--no-plan-hint", action="store_true", help="pass max_len = 0 (force the planning pass)")
    ap.add_argument("--pmc-live", default="auto", choices=["auto", "on", "off"],
                    help="roofline.traffic from a rocprofv3 --pmc FETCH_SIZE pass of this config run here after the "
                         "timed region (auto: at N = 1 when not itself under rocprofv3); else from the committed "
                         "profiles/pmc_cfg<config>.json")
    ap.add_argument("--launch", default="graph", choices=["graph", "eager"],
                    help="timed steps as hipGraph replays (default; eager launches if capture fails) or eager")
    ap.add_argument("--graph-steps", type=int, default=0,
                    help="steps captured per hipGraph (0 = all timed steps in one graph when --steps <= 64, so the "
                         "GPU runs them back to back; 1 = one replay per step)")
    ap.add_argument("--cpu-sample-blocks", type=int, default=4096)
    ap.add_argument("--cpu-threads", type=int, default=0, help="0 = every core this process may run on")
    ap.add_argument("--cpu-seconds", type=float, default=3.0, help="CPU work per thread count (>= 1 pass)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--roundtrip-gib", type=float, default=4.0)
    ap.add_argument("--form", default="batch", choices=["batch", "verify"],
                    help="verify: each step is the verify form (Mask(crc) compared with stored words inside the CRC "
                         "kernels, db/value_log_reader.cc:109-122) against the reference's words with 2 planted "
                         "mismatches per rank; first_bad / nbad reduced over the ranks (all-reduce MIN / SUM)")
    ap.add_argument("--numa-bind", default="auto", choices=["auto", "off"],
                    help="auto: bind each rank's threads (and its pinned memory) to its GPU's NUMA node (place_rank)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher check without a GPU: each rank joins a gloo group, the ranks agree on the world "
                         "size and rank 0 prints a JSON line with n_gpus / backend (tests/test_bench_launch.py)")
    ap.add_argument("--pmc-json", default=None,
                    help="PMC summary of the same config (default profiles/pmc_cfg<config>.json, written by "
                         "kv-separate_amd/tools/pmc_summary.py from separate rocprofv3 --pmc passes)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            # one process per GPU, started from here; nothing above touched the GPU (device_count does not)
            if not (args.dry_run or os.environ.get("KVSEP_BENCH_SAME_DEVICE")) and torch.cuda.device_count() < args.gpus:
                log(f"--gpus {args.gpus}: only {torch.cuda.device_count()} GPU(s) visible")
                sys.exit(2)
            sys.exit(launch_ranks(args.gpus))
    elif int(os.environ["WORLD_SIZE"]) != args.gpus:
        log(f"--gpus {args.gpus} but WORLD_SIZE={os.environ['WORLD_SIZE']}: refusing to report a line for a different "
            f"number of ranks")
        sys.exit(2)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.dry_run:
        if os.environ.get("KVSEP_BENCH_DRYRUN_FAIL_RANK") == str(rank):  # launcher test: this rank dies at start
            sys.exit(3)
        if world > 1:
            dist.init_process_group("gloo")
            t = torch.tensor([world, rank], dtype=torch.int64)
            seen = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
            dist.all_gather(seen, t)
            ranks = sorted(int(x[1]) for x in seen)
            assert ranks == list(range(world)) and all(int(x[0]) == world for x in seen), seen
        # the per-rank records travel the same way as on the GPU path (no device: no bus ID, no kernel)
        t_start = time.time()
        rec = rank_record(rank, local, None, {"numa_node": None, "bound_cpus": 0}, None, 1.0, t_start, time.time(),
                          GIB, None)
        ids = os.environ.get("KVSEP_BENCH_DRYRUN_BUS_IDS")  # launcher test: the bus ID each rank's GPU would report
        if ids:
            rec["pci_bus_id"] = (ids.split(",") + [None] * world)[rank]
        per_rank = shard.gather_objects(rec, dist if world > 1 else None)
        failures = []
        if rank == 0:
            same = bool(os.environ.get("KVSEP_BENCH_SAME_DEVICE"))
            line = {"dry_run": True, "n_gpus": world, "world_size": world,
                    "backend": dist.get_backend() if world > 1 else None, "per_rank": per_rank,
                    "per_rank_summary": shard.rank_summary(per_rank, same_device=same)}
            failures = line["failures"] = line_failures(line, world, same)
            print(json.dumps(line), flush=True)
        if world > 1:
            dist.destroy_process_group()
        if failures:
            log(f"[rank 0] the line above is not a clean measurement: {'; '.join(failures)}")
            sys.exit(1)
        return
    # Started by a launcher (torchrun, launch_ranks): a process group, RCCL with one rank per GPU -- also at one rank,
    # so `torchrun --nproc-per-node 1 bench.py` runs the same RCCL init and collectives as eight ranks do
    # (tests/test_gpu_rccl.py).  A plain `python bench.py` (N = 1) makes no process group and no collective.
    if "WORLD_SIZE" in os.environ:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if os.environ.get("KVSEP_BENCH_SAME_DEVICE"):  # rehearsal: every rank on cuda:0, gloo for results
            local = 0
            dist.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    dd = dist if dist.is_initialized() else None
    dev = torch.device("cuda", local)
    torch.cuda.set_device(dev)
    coll_dev = dev if dd is None or dist.get_backend() == "nccl" else torch.device("cpu")
    allowed_cpus = os.sched_getaffinity(0)  # before placement: the CPU baseline spreads over every node
    placement = place_rank(local, args.numa_bind)
    same_device = bool(os.environ.get("KVSEP_BENCH_SAME_DEVICE"))

    ctx = kvsep.Context(local)
    if args.piece_kib:
        ctx.set_piece_bytes(args.piece_kib * 1024)
    if args.schedule != "default":
        ctx.set_schedule(args.schedule == "dynamic")

    plan = Plan(args.config, world, rank)
    off, ln, count, useful, span = plan.off, plan.ln, plan.count, plan.useful, plan.span
    npass = len(plan.passes)
    max_len = 0 if args.no_plan_hint else (int(ln.max()) if count else 0)
    log(f"[rank {rank}] {plan.desc}: {useful / GIB:.2f} GiB useful per pass x {npass}, span {span / GIB:.2f} GiB")

    # synthetic data, generated in HBM: the buffer holds global stream bytes [stream_base, stream_base + span)
    data = torch.empty(span + 64, dtype=torch.uint8, device=dev)

    def fill(p):
        kvsep.fill_splitmix64(data.data_ptr(), span, plan.seed, plan.passes[p][0])

    fill(0)
    d_off, d_len = to_dev_u64(off, dev), to_dev_u64(ln, dev)
    out = torch.zeros((npass, max(count, 1)), dtype=torch.int32, device=dev)
    ctx.reserve(count, useful)
    stream = torch.cuda.current_stream()
    verify = args.form == "verify"
    planted = []
    if verify:
        if npass != 1 or not count:
            raise SystemExit("--form verify needs a one-pass configuration (2, 3a, 3b, 4)")
        ib = plan.passes[0][1]
        gold = None
        if plan.golden:
            g = np.fromfile(os.path.join(GOLDEN, plan.golden), dtype="<u4")
            if g.size >= ib + count:
                gold = g[ib:ib + count]
        if gold is None:  # no reference words for this range (config 4 past its first 2^20 blocks): the batch form's
            ctx.batch_device(data.data_ptr(), d_off, d_len, out[0], count=count, total_bytes=useful, max_len=max_len)
            torch.cuda.synchronize()  # (checked against the reference's digest below, like every result)
            gold = out[0, :count].cpu().numpy().view(np.uint32).copy()
        rot = (gold >> np.uint32(15)) | (gold << np.uint32(17))
        stored = (rot + np.uint32(0xA282EAD8)).astype(np.uint32)  # Mask, util/crc32c.h:29-32
        planted = sorted({(rank * 7919 + 13) % count, count - 1 - (rank * 31) % count})
        stored[planted] ^= np.uint32(0x00010000)
        d_expect = torch.from_numpy(stored.view(np.int32)).to(dev)
        d_fb = torch.zeros(1, dtype=torch.int64, device=dev)
        d_nb = torch.zeros(1, dtype=torch.int64, device=dev)

    def crc(p, st):
        if verify:
            ctx.verify_device(data.data_ptr(), d_off, d_len, d_expect, out[p], d_fb, d_nb, count=count,
                              total_bytes=useful, max_len=max_len, stream=st)
        else:
            ctx.batch_device(data.data_ptr(), d_off, d_len, out[p], count=count, total_bytes=useful, max_len=max_len,
                             stream=st)

    # ---- warm-up
    for _ in range(args.warmup):
        for p in range(npass):
            if npass > 1:
                fill(p)
            crc(p, stream)
    torch.cuda.synchronize()

    piece = args.piece_kib * 1024 or kvsep.DEFAULT_PIECE_BYTES
    graphable = npass == 1
    span_timing = args.launch == "graph" and graphable and 0 < max_len <= piece
    launch = "eager"
    ev = [torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)]
    if npass == 1:
        # kernel-only time of the CRC kernel, HIP events on the stream it runs on.  A step of an unsplit batch is the
        # CRC kernel alone: under graph replay, one event pair around the timed region gives its average over the
        # back-to-back launches.  A split batch also runs planning and combine kernels, so its CRC kernel is timed
        # with an event pair per launch over the same number of eager steps.
        ctx.get_timing()
        ctx.set_timing(True)
        for _ in range(args.steps if args.launch == "graph" and not span_timing else 0):
            crc(0, stream)
        torch.cuda.synchronize()
        # the timed steps as hipGraph replays: each captured step is a full pass of the hot path (planning kernels,
        # memsets, CRC kernel(s), combine; kvsep_crc32c_reserve made every allocation beforehand).  By default all K
        # timed steps are captured into ONE graph, so the GPU runs them back to back instead of waiting on a host
        # replay per step (a 50 us config-2 step otherwise pays ~7 us of replay turnaround); or eager launches.
        run = lambda: crc(0, stream)  # noqa: E731
        n_calls = args.steps
        if args.launch == "graph":
            ctx.set_timing(False)  # no timing events inside the graph
            per = args.graph_steps or (args.steps if args.steps <= 64 else 1)
            if args.steps % per:
                per = 1
            try:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    for _ in range(per):
                        crc(0, torch.cuda.current_stream())
                g.replay()  # warm replay
                torch.cuda.synchronize()
                run, launch, n_calls = g.replay, f"hipGraph ({per} step(s) per replay)", args.steps // per
            except Exception as e:  # keep the measurement: fall back to eager launches
                log(f"[rank {rank}] graph capture failed ({e}); timing eager launches")
                torch.cuda.synchronize()
                span_timing = False
                ctx.set_timing(True)
        if dd:
            dist.barrier()
        torch.cuda.synchronize()
        t_start = time.time()
        t0 = time.perf_counter()
        if span_timing:
            ev[0].record()  # the graph replays on the current stream
        for _ in range(n_calls):
            run()
        if span_timing:
            ev[1].record()
        torch.cuda.synchronize()
        own = time.perf_counter() - t0  # this rank's own time, before waiting for the others
        t_end = time.time()
        if dd:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        ctx.set_timing(False)
        kern_ms, launches = ctx.get_timing()
        if span_timing:
            kern_ms, launches = ev[0].elapsed_time(ev[1]), args.steps
        timing_note = ("one HIP event pair around the timed graph replay of back-to-back single-kernel steps"
                       if span_timing else "a HIP event pair around each launch of the CRC kernel")
    else:
        # Config 5 with several distinct slices per GPU: a step is one CRC pass over each of this rank's slices.  A
        # pass's slice is (re)generated in HBM before its timed region opens -- the data "arriving" -- so every
        # timed pass starts with its input resident, like every other config; each pass is bracketed by barrier +
        # synchronize, the step time is the sum of its passes.
        elapsed = own = 0.0
        t_start = t_end = None
        ctx.get_timing()
        for _ in range(args.steps):
            for p in range(npass):
                fill(p)
                torch.cuda.synchronize()
                if dd:
                    dist.barrier()
                ctx.set_timing(True)
                t_start = time.time() if t_start is None else t_start
                t0 = time.perf_counter()
                crc(p, stream)
                torch.cuda.synchronize()
                own += time.perf_counter() - t0
                t_end = time.time()
                if dd:
                    dist.barrier()
                elapsed += time.perf_counter() - t0
                ctx.set_timing(False)
        kern_ms, launches = ctx.get_timing()
        timing_note = ("a HIP event pair around each launch of the CRC kernel; each slice regenerated in HBM "
                       "outside the timed passes")
    elapsed = shard.max_over_ranks(elapsed, dd, coll_dev)
    total_useful = useful * npass
    total_useful = int(shard.sum_over_ranks(total_useful, dd, coll_dev))
    ms_per_step = elapsed * 1e3 / args.steps
    value = total_useful * args.steps / GIB / elapsed
    kern_avg_ms = kern_ms / max(1, launches)
    kernel_name = ctx.kernel_name(count, max_len, useful)
    achieved_gbps = useful / (kern_avg_ms * 1e-3) / 1e9
    my_record = rank_record(rank, local, local, placement, kern_avg_ms, own, t_start, t_end,
                            useful * npass * args.steps, kernel_name, launch_bytes=useful)

    # ---- outside the timed region: u32 results of every rank gathered (RCCL), every block checked
    verdict = None
    if verify:  # the last step's verdict, reduced over the ranks: the global lowest bad index and the total
        fb, nb = int(d_fb.item()), int(d_nb.item())
        local_first = -1 if fb in (-1, (1 << 64) - 1) else fb
        ib = plan.passes[0][1]
        gnb, gfb = shard.verify_over_ranks(nb, -1 if local_first < 0 else ib + local_first, dd, coll_dev)
        want = [(r, Plan(args.config, world, r)) for r in range(world)]
        exp_first = min(pl.passes[0][1] + min({(r * 7919 + 13) % pl.count, pl.count - 1 - (r * 31) % pl.count})
                        for r, pl in want if pl.count)
        exp_n = sum(len({(r * 7919 + 13) % pl.count, pl.count - 1 - (r * 31) % pl.count}) for r, pl in want if pl.count)
        verdict = {"first_bad": gfb, "nbad": gnb, "planted_per_rank": len(planted), "expected_first_bad": exp_first,
                   "expected_nbad": exp_n, "ok": gfb == exp_first and gnb == exp_n,
                   "reduction": "all-reduce MIN of first_bad (global index) and SUM of nbad over the ranks"
                   if dd else "one rank"}
    crcs = out[:, :count].cpu().numpy().view(np.uint32).reshape(-1)
    if os.environ.get("KVSEP_BENCH_CORRUPT_RESULT") == str(rank) and crcs.size:  # test hook: one wrong gathered word
        crcs = crcs.copy()
        crcs[crcs.size // 2] ^= np.uint32(1)
    results = shard.gather_results(crcs, dd, coll_dev)
    digests = [shard.crc_of_crcs(r, kvsep.extend_host) for r in results]

    # The attainable read rate over the same allocation: stream_read_kernel, the fastest read-only pattern of
    # tools/hbm_probe.hip, over the batch's span.  From 8 GiB up, three eager launches timed by HIP events; below,
    # the way the CRC kernel of an unsplit small batch is timed -- K launches captured into one hipGraph, one event
    # pair around the replay -- so the ceiling carries the same launch ramp and drain per launch (config 2: the
    # same-size streaming read).
    read_ceiling_gbps = ceiling_note = None
    if span >= 8 * (1 << 30):
        sink = torch.zeros(4, dtype=torch.int32, device=dev)
        ctx.stream_read(data.data_ptr(), span, sink, stream=stream)  # warm
        torch.cuda.synchronize()
        ctx.set_timing(True)
        for _ in range(3):
            ctx.stream_read(data.data_ptr(), span, sink, stream=stream)
        torch.cuda.synchronize()
        ctx.set_timing(False)
        sr_ms, sr_n = ctx.get_timing()
        read_ceiling_gbps = (span // 16 * 16) / (sr_ms / sr_n * 1e-3) / 1e9
        ceiling_note = "stream_read_kernel over the same span, 3 eager launches, HIP events"
    elif span and npass == 1:
        try:
            sink = torch.zeros(4, dtype=torch.int32, device=dev)
            reps = max(args.steps, 10)
            gs = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gs):
                for _ in range(reps):
                    ctx.stream_read(data.data_ptr(), span, sink, stream=torch.cuda.current_stream())
            gs.replay()  # warm
            torch.cuda.synchronize()
            best = None
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                gs.replay()
                e1.record()
                torch.cuda.synchronize()
                t = e0.elapsed_time(e1) / reps
                best = t if best is None else min(best, t)
            read_ceiling_gbps = (span // 16 * 16) / (best * 1e-3) / 1e9
            ceiling_note = (f"stream_read_kernel over the same {span / (1 << 20):.0f} MiB span, {reps} launches per "
                            f"hipGraph replay, one HIP event pair, best of 3 replays: {best * 1e3:.2f} us per launch")
            del gs
        except Exception as e:  # the headline line never depends on the ceiling
            log(f"[rank {rank}] small-span read ceiling failed: {e}")

    # Single pass (round 6): the timed graph re-reads one buffer, and a launch finds part of it (translations, the
    # 256 MB Infinity Cache) left by the launch before.  Here launch i of a captured graph reads copy i mod 8 of the
    # batch, so no launch does: the rate of one pass over data not already cached, for the CRC kernel and the streaming
    # read alike (profiles/round6/README.md, claim_pipeline_ab/rot_*: config 2 44.2 -> 48.0 us).  Small one-pass batch
    # forms only; reported beside the line's value, never as it.
    single_pass = None
    if span and npass == 1 and not verify and span <= (1 << 30) and args.launch == "graph":
        try:
            copies = [data] + [torch.empty_like(data) for _ in range(7)]
            for c in copies[1:]:
                c.copy_(data)
            tmp_out = torch.empty_like(out[0])
            sink = torch.zeros(4, dtype=torch.int32, device=dev)
            reps = 16

            def graph_ms(fn):
                g2 = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g2):
                    for i in range(reps):
                        fn(i, torch.cuda.current_stream())
                g2.replay()  # warm
                torch.cuda.synchronize()
                best = None
                for _ in range(3):
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                    e0.record()
                    g2.replay()
                    e1.record()
                    torch.cuda.synchronize()
                    t = e0.elapsed_time(e1) / reps
                    best = t if best is None else min(best, t)
                del g2
                return best

            crc_ms = graph_ms(lambda i, st: ctx.batch_device(copies[i % 8].data_ptr(), d_off, d_len, tmp_out,
                                                             count=count, total_bytes=useful, max_len=max_len,
                                                             stream=st))
            sr_ms = graph_ms(lambda i, st: ctx.stream_read(copies[i % 8].data_ptr(), span, sink, stream=st))
            single_pass = {"copies": 8, "launches_per_replay": reps, "crc_us": round(crc_ms * 1e3, 2),
                           "crc_GiBps": round(useful / (crc_ms * 1e-3) / 2**30, 1),
                           "stream_read_us": round(sr_ms * 1e3, 2),
                           "frac_of_stream_read": round(sr_ms / crc_ms, 4),
                           "timing": "hipGraph of 16 launches, launch i on copy i mod 8 of the batch, best of 3 "
                                     "replays; the CRC launches write a scratch output"}
            del copies, tmp_out
        except Exception as e:  # the headline line never depends on it
            log(f"[rank {rank}] single-pass measurement failed: {e}")

    parity = None
    cpu = None
    if rank == 0:
        oracle = load_oracle()
        parity = check_results([Plan(args.config, world, r) for r in range(world)], results, oracle)
        parity["all_blocks_match"] = parity["mismatches"] == 0 and parity["mismatching_digest_ranges"] == 0
        res = None
        if not args.no_cpu and world == 1:
            aff = len(allowed_cpus)
            most = args.cpu_threads or aff
            quota_raw, quota = cpu_quota()
            counts = {1, most} | {t for t in (8, 16, 32, 64, 128) if t < most}
            if quota and int(quota) < most:
                counts.add(max(1, int(quota)))  # the cgroup's CPU share: the scaling must flatten there
            counts = sorted(counts)
            nsample = min(args.cpu_sample_blocks, count)
            try:
                res, host, hoff, lens, idx, kind = cpu_baseline(oracle, data, off, ln, nsample, counts,
                                                                args.cpu_seconds, allowed=allowed_cpus)
            except Exception as e:  # the headline line never depends on the CPU leg
                log(f"[rank 0] cpu baseline failed: {e}")
                res = None
        if res is not None:
            threads = max(counts, key=lambda t: res[t][0])  # the baseline is the CPU's best thread count
            vt, sbt, dtt, _ = res[threads]
            impl_desc = ("util/crc32c.cc of the reference (portable path, g++ -O3, oracle/_ref), each thread pinned "
                         "(spread over the NUMA nodes, one hardware thread per core first) and checksumming its own "
                         "first-touched copy of its byte range"
                         if kind == "reference" else
                         "oracle/crc32c_oracle.c (restated util/crc32c.cc portable path, gcc -O3)")
            nodes = numa_nodes()
            cpu = {"value": round(vt, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
                   "sample": f"{nsample} blocks of the same batch ({int(lens.sum()) / GIB:.2f} GiB) copied to host "
                             f"memory, {impl_desc}; blocks split over threads by bytes, repeated passes of "
                             f"{args.cpu_seconds:.0f} s per thread count, 1 to {most} threads (every CPU this process "
                             f"may run on); best: {threads} threads, {sbt / GIB:.1f} GiB in {dtt:.1f} s",
                   "by_threads_GiBps": {str(t): round(res[t][0], 3) for t in counts},
                   "by_threads_numa_nodes": {str(t): res[t][3] for t in counts},
                   "single_thread_GiBps": round(res[1][0], 3),
                   "nproc": os.cpu_count(), "affinity_cores": aff, "cpu_model": cpu_model(),
                   "cgroup_cpu_max": quota_raw, "cgroup_cpu_limit": quota,
                   "numa_nodes": {str(n): _read(f"/sys/devices/system/node/node{n}/cpulist") or f"{len(c)} cpus"
                                  for n, c in nodes.items() if c},
                   "limit_note": (f"this process may use {quota:g} CPUs' worth of time (cgroup cpu.max) of the {aff} "
                                  f"it may run on: rates flatten from {int(quota)} threads on" if quota and quota < aff
                                  else "no cgroup CPU limit below the affinity set")}
            s1 = host_leg_rate(host, hoff[:max(1, nsample // 4)], lens[:max(1, nsample // 4)], 1, 2.0)
            sn = host_leg_rate(host, hoff, lens, threads, 2.0)
            cpu["host_leg_GiBps"] = {"1": round(s1, 3), str(threads): round(sn, 3), "path": host_leg_path(),
                                     "note": "informational, not the baseline: the library's own host leg (the "
                                             "drop-in's small-input path) on the same sample; the reference build "
                                             "here has no accelerated path (HAVE_CRC32C=0)"}

    # host round trip (PCIe-inclusive).  At N > 1 every rank streams its own pinned image through its own GPU
    # at the same time (each GPU has its own PCIe link); the rate is the sum over ranks / the slowest rank.
    # Every rank runs the same collectives whatever fails locally, so a failure cannot leave a rank waiting.
    rt = None
    rt_ok = None
    if args.roundtrip_gib > 0:
        state = None
        try:
            state = roundtrip_setup(ctx, int(args.roundtrip_gib * GIB))
        except Exception as e:  # keep the headline line even if pinned allocation is refused
            log(f"[rank {rank}] host round trip setup failed: {e}")
        if shard.min_over_ranks(1 if state is not None else 0, dd, coll_dev):
            if dd:
                dist.barrier()
            dt, good = float("inf"), False
            try:
                dt, good = roundtrip_time(ctx, state)
            except Exception as e:
                log(f"[rank {rank}] host round trip failed: {e}")
            if dt != float("inf"):
                my_record["roundtrip_GiBps"] = round(float(state[3].sum()) / GIB / dt, 3)
                my_record["roundtrip_image_numa_node"] = kvsep.host_page_node(state[0].data_ptr())
            dt = shard.max_over_ranks(dt, dd, coll_dev)
            rt_ok = bool(shard.min_over_ranks(1 if good else 0, dd, coll_dev))
            if dt != float("inf"):
                rt = round(world * float(state[3].sum()) / GIB / dt, 3)
        state = None
    # every rank's record (bus ID, NUMA node, affinity, its own kernel time / elapsed / GiB/s, its host staging), so
    # an N-rank line can tell one slow GPU from launch skew or a shared-host effect
    try:
        st = ctx.host_placement()
        st["copier_cpus"] = kvsep.format_cpulist(st["copier_cpus"])
        my_record["staging"] = st
    except Exception:
        pass
    per_rank = shard.gather_objects(my_record, dd)

    traffic = None
    traffic_src = None
    traffic_profile = None
    pmc_cfg = "3b" if args.config == "5" else args.config  # config 5's launches are config-3b launches
    if args.pmc_json is None:
        args.pmc_json = os.path.join(ROOT, "profiles", f"pmc_cfg{pmc_cfg}.json")
    if os.path.exists(args.pmc_json):
        try:
            pm = json.load(open(args.pmc_json))
            if pm.get("config") == pmc_cfg:
                traffic = traffic_profile = pm.get("hbm_bytes_per_launch")
                traffic_src = os.path.relpath(args.pmc_json, ROOT) + " (rocprofv3 --pmc passes of the same config)"
        except Exception:
            traffic = None
    # auto: at N = 1, and never when this process itself runs under a profiler (rocprofv3 exports ROCPROF_* to the
    # program it profiles; a nested profiler pass would fight it for the counters)
    under_profiler = any(k.startswith("ROCPROF") for k in os.environ)
    if rank == 0 and (args.pmc_live == "on" or (args.pmc_live == "auto" and world == 1 and not under_profiler)):
        # the child allocates its own batch: free this one first (config 4 is 150 GiB of the 288)
        data = d_off = d_len = out = None  # noqa: F841
        torch.cuda.synchronize()
        torch.cuda.empty_cache()
        live, nl, why = live_pmc_traffic(args)
        if live is not None:
            traffic = live
            traffic_src = (f"live: rocprofv3 --pmc FETCH_SIZE --kernel-trace pass of this config on this box after the "
                           f"timed region (child process, {nl} CRC dispatches), FETCH_SIZE x 1024 x 2")
        else:
            log(f"[rank 0] live PMC pass unavailable ({why}); traffic from the committed profile")

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 3),
            "unit": "GiB/s",
            "n_gpus": world,
            "world_size": world,
            "backend": dist.get_backend() if dd else None,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "launch": launch,
            "higher_is_better": True,
            "scaling": plan.scaling,
            "vs_baseline": None,
            "dtype": "u8",
            "data": "synthetic (splitmix64 byte stream generated in HBM)",
            "config": {"workload": plan.desc, "config": args.config, "blocks_per_gpu": count * npass,
                       "bytes_per_gpu": useful * npass, "total_bytes": total_useful,
                       "piece_bytes": args.piece_kib * 1024 or kvsep.DEFAULT_PIECE_BYTES,
                       "parallelism": f"shard{world} (independent blocks per GPU, no data-path collective)"},
            "roofline": {"bound": "hbm", "achieved": round(achieved_gbps, 1), "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                         "frac": round(achieved_gbps / HBM_PEAK_GBPS, 4), "traffic": traffic,
                         "traffic_source": traffic_src, "traffic_committed_profile": traffic_profile,
                         "traffic_over_algorithmic": traffic and round(traffic / useful, 4),
                         "kernel": kernel_name, "kernel_avg_ms": round(kern_avg_ms, 4), "kernel_timing": timing_note,
                         "algorithmic_bytes_per_launch": useful},
            "cpu_baseline": cpu,
            "read_ceiling_GBps": read_ceiling_gbps and round(read_ceiling_gbps, 1),
            "read_ceiling_timing": ceiling_note,
            "frac_of_read_ceiling": read_ceiling_gbps and round(achieved_gbps / read_ceiling_gbps, 4),
            "single_pass": single_pass,
            "host_roundtrip_GiBps": rt,
            "host_roundtrip_ranks": world if rt is not None else None,
            "host_roundtrip_parity": rt_ok,
            "parity": parity,
            "parity_spot_check": bool(parity and parity["all_blocks_match"]),
            "digests": [hex(d) for d in digests],
            "per_rank": per_rank,
            "per_rank_summary": shard.rank_summary(per_rank, same_device=same_device),
            "form": args.form,
            "verify": verdict,
        }
        failures = line_failures(line, world, same_device)
        line["failures"] = failures
        print(json.dumps(line), flush=True)
    ctx.close()
    if dd:
        dist.destroy_process_group()
    if rank == 0 and failures:
        log(f"[rank 0] the line above is not a clean measurement: {'; '.join(failures)}")
        sys.exit(1)


if __name__ == "__main__":
    main()
