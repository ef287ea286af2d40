"""Multi-GPU sharding of a CRC batch: blocks are independent, so each rank checksums its own
shard from its own HBM; only the u32 results (4 B per block), verify counts and timings cross the interconnect.

Two ways a batch is spread over ranks, both one logical batch of the whole job:
  * uniform configs (2, 3a, 3b): every rank holds the same block layout over its own slice of one global
    splitmix64 stream -- rank r's byte j is global stream byte r*span + j (weak scaling);
  * ragged config 4: one global batch of world x 2^20 Zipf blocks, cut into contiguous block ranges balanced by
    bytes (kvsep_crc32c_partition, a prefix sum of len), one range per rank.
Used by bench.py on RCCL and by tests/test_multiprocess_cpu.py on gloo.
"""
from __future__ import annotations

import numpy as np


def _active(dist) -> bool:
    """A collective runs whenever a process group is up -- also a one-rank group (so a one-rank RCCL communicator
    runs the same all_gather / all_reduce code as eight ranks do: tests/test_gpu_rccl.py); no group, no collective."""
    return dist is not None and dist.is_initialized()


def stream_offset(rank: int, span: int) -> int:
    """Global stream position of rank `rank`'s first data byte."""
    return rank * span


def global_layout(off: np.ndarray, length: np.ndarray, span: int, world: int):
    """The single logical batch the world checksums (for checking a sharded run)."""
    off = np.asarray(off, dtype=np.uint64)
    length = np.asarray(length, dtype=np.uint64)
    offs = np.concatenate([off + np.uint64(stream_offset(r, span)) for r in range(world)])
    return offs, np.tile(length, world)


def partition_layout(goff: np.ndarray, glen: np.ndarray, world: int, rank: int):
    """Rank `rank`'s part of one global batch (global offsets goff into one stream, lengths glen), balanced by bytes:
    -> (local offsets from the part's first byte, lengths, stream base = global byte offset of that first byte,
    index base = global index of the part's first block)."""
    from kvsep import partition

    b = partition(glen, world)
    b0, b1 = int(b[rank]), int(b[rank + 1])
    goff = np.asarray(goff, dtype=np.uint64)
    glen = np.asarray(glen, dtype=np.uint64)
    if b1 == b0:
        return np.zeros(0, np.uint64), np.zeros(0, np.uint64), 0, b0
    base = int(goff[b0])
    return goff[b0:b1] - np.uint64(base), glen[b0:b1].copy(), base, b0


def gather_results(crcs: np.ndarray, dist, device) -> list[np.ndarray]:
    """All-gather every rank's u32 results (any lengths) -> the list of per-rank arrays on every rank: the result
    traffic of SURVEY.md §8e, 4 B per block (2 MiB for config 5's 524,288 records)."""
    import torch

    crcs = np.ascontiguousarray(crcs, dtype=np.uint32)
    if not _active(dist):
        return [crcs]
    world = dist.get_world_size()
    n = torch.tensor([crcs.size], dtype=torch.int64, device=device)
    ns = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(ns, n)
    ns = [int(x.item()) for x in ns]
    m = max(ns)
    t = torch.zeros(m, dtype=torch.int32, device=device)
    if crcs.size:
        t[:crcs.size] = torch.from_numpy(crcs.view(np.int32)).to(device)
    outs = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(outs, t)
    return [o[:k].cpu().numpy().view(np.uint32).copy() for o, k in zip(outs, ns)]


def crc_of_crcs(crcs: np.ndarray, extend_host) -> int:
    """Size-independent digest of a result vector: CRC-32C over the little-endian u32 results."""
    a = np.ascontiguousarray(crcs, dtype="<u4")
    return int(extend_host(0, a.tobytes()))


def max_over_ranks(value: float, dist, device) -> float:
    import torch

    if not _active(dist):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def min_over_ranks(value: float, dist, device) -> float:
    import torch

    if not _active(dist):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return float(t.item())


def sum_over_ranks(value: float, dist, device) -> float:
    import torch

    if not _active(dist):
        return value
    t = torch.tensor([value], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.SUM)
    return float(t.item())


def verify_over_ranks(nbad: int, first_bad: int, dist, device) -> tuple[int, int]:
    """The verify form across ranks: total mismatches (all-reduce SUM) and the lowest mismatching GLOBAL
    block index (all-reduce MIN; each rank's first_bad already offset by its index base, -1 = none) -- what a reader
    that stops at the first bad record needs (db/value_log_reader.cc:109-122), and the reduction
    kvsep_crc32c_group_verify_device does between the members of one process.  Identity with no process group."""
    import torch

    if not _active(dist):
        return nbad, first_bad
    big = np.iinfo(np.int64).max
    n = torch.tensor([nbad], dtype=torch.int64, device=device)
    f = torch.tensor([big if first_bad < 0 else first_bad], dtype=torch.int64, device=device)
    dist.all_reduce(n, op=dist.ReduceOp.SUM)
    dist.all_reduce(f, op=dist.ReduceOp.MIN)
    fb = int(f.item())
    return int(n.item()), (-1 if fb == big else fb)


def gather_objects(obj, dist) -> list:
    """All-gather one picklable object per rank (the per-rank records of a bench line) -> the list in rank order on
    every rank; [obj] with no process group.  Over RCCL (the nccl backend) the pickled bytes travel as a device
    tensor, over gloo on the host."""
    if not _active(dist):
        return [obj]
    out = [None] * dist.get_world_size()
    dist.all_gather_object(out, obj)
    return out


def _spread(vals):
    vals = [v for v in vals if v is not None]
    if not vals:
        return None, None, None
    lo, hi = min(vals), max(vals)
    return lo, hi, ((hi - lo) / hi if hi else 0.0)


def rank_summary(records: list, same_device: bool = False) -> dict:
    """What a multi-GPU line needs to diagnose itself from its per-rank records (bench.py `per_rank`): whether every
    rank ran on its own physical GPU (distinct PCI bus IDs; a same-device rehearsal says so instead), the spread of
    the ranks' own rates and kernel times (skew = (max - min) / max), how far apart they started and finished (wall
    clock, one host), and the slowest rank."""
    ids = [r.get("pci_bus_id") for r in records]
    distinct = all(ids) and len(set(ids)) == len(ids)
    g_lo, g_hi, g_skew = _spread([r.get("GiBps") for r in records])
    k_lo, k_hi, k_skew = _spread([r.get("kernel_avg_ms") for r in records])
    starts = [r["t_start"] for r in records if r.get("t_start") is not None]
    ends = [r["t_end"] for r in records if r.get("t_end") is not None]
    rated = [r for r in records if r.get("GiBps") is not None]
    out = {
        "ranks": len(records),
        "distinct_devices": bool(distinct),
        "same_device_rehearsal": bool(same_device),
        "pci_bus_ids": sorted(set(i for i in ids if i)),
        "numa_nodes": sorted(set(r.get("numa_node") for r in records if r.get("numa_node") is not None)),
        "GiBps_min": g_lo, "GiBps_max": g_hi, "GiBps_skew": g_skew,
        "kernel_avg_ms_min": k_lo, "kernel_avg_ms_max": k_hi, "kernel_skew": k_skew,
        "start_skew_ms": (max(starts) - min(starts)) * 1e3 if starts else None,
        "end_skew_ms": (max(ends) - min(ends)) * 1e3 if ends else None,
        "slowest_rank": min(rated, key=lambda r: r["GiBps"])["rank"] if rated else None,
    }
    for k in ("GiBps_min", "GiBps_max", "kernel_avg_ms_min", "kernel_avg_ms_max"):
        if out[k] is not None:
            out[k] = round(out[k], 4)
    for k in ("GiBps_skew", "kernel_skew", "start_skew_ms", "end_skew_ms"):
        if out[k] is not None:
            out[k] = round(out[k], 5)
    return out
