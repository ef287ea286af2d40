#!/usr/bin/env python3
"""Diag (KVSEP_DIAG build): WHAT the sorted-window kernel with the round-1 in-kernel verify compare (KVSEP_NARROW=24)
writes for the blocks it gets wrong -- same binary as tools/sorted_vin_probe.py, no instrumentation in the kernel.

The output array starts as a sentinel; after the run every wrong block is classified on the host:
  unwritten     out[b] is still the sentinel
  other-block   out[b] is the CRC of another block of the batch (which one: same window? which group/slot?)
  other         anything else; then it is tested against Extend(init, data) for the block's bytes with the length of
                the block at every other sorted position of its window, and against CRCs of prefixes/suffixes.
Runs are reconstructed from the kernel's schedule (grid = CUs, 16-wave workgroups, wave-major runs of whole 8-block
groups; windows of 64 from each run's start), so each wrong block is reported with its window, group k and slot.
usage: sorted_vin_forensics.py [variant ...]   (default 24 20)"""
import collections
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import _diag  # noqa: E402,F401
import kvsep  # noqa: E402
from conftest import load_oracle  # noqa: E402  (the checker)
from kvsep import splitmix64_bytes  # noqa: E402

SENT = 0xA5A5A5A5
dev = torch.device("cuda:0")
oracle = load_oracle()
host = splitmix64_bytes(64 << 20, 5, 0)
d = torch.from_numpy(host).to(dev)
u64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)  # noqa: E731
ncu = torch.cuda.get_device_properties(0).multi_processor_count
variants = sys.argv[1:] or ["24", "20"]


def schedule(n, nwaves, grid):
    """block -> (run lo, window base, group k in window, sorted position) per the kernel's run/window rules."""
    groups = (n + 7) // 8
    gper = (groups + nwaves - 1) // nwaves
    info = {}
    runs = []
    for wave in range(nwaves // grid):
        for b in range(grid):
            lo = (wave * grid + b) * gper * 8
            hi = min(lo + gper * 8, n)
            if lo < hi:
                runs.append((lo, hi))
    return runs


def sorted_positions(ln, lo, hi, hint):
    """window W -> list of block indices in sorted order (the kernel's wave_sort64 on (len key, lane))."""
    out = {}
    for W in range(lo, hi, 64):
        m = min(64, hi - W)
        keys = []
        for i in range(64):
            b = W + i
            if i >= m:
                key = 0xFFFFFFFE
            else:
                L = int(ln[b])
                key = 0 if L > hint else L
            keys.append((key, i))
        keys.sort()
        out[W] = [W + i for key, i in keys]
    return out


rng = np.random.default_rng(1)
for n, maxlen in ((70000, 39), (70000, 200), (200000, 39)):
    ln = rng.integers(0, maxlen + 1, n).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    exp = oracle.batch(host, off, ln, None, threads=8)
    masked = np.array([kvsep.mask(int(x)) for x in exp], dtype=np.uint32)
    nwaves = ncu * 16
    runs = schedule(n, nwaves, ncu)
    where = {}
    for lo, hi in runs:
        sp = sorted_positions(ln, lo, hi, maxlen)
        for W, order in sp.items():
            for pos, b in enumerate(order):
                if b < hi:
                    where[b] = (lo, W, pos // 8, pos % 8)
    crc_to_blocks = collections.defaultdict(list)
    for b in range(n):
        crc_to_blocks[int(exp[b])].append(b)
    for v in variants:
        os.environ["KVSEP_NARROW"], os.environ["KVSEP_CRC_VARIANT"] = v, "1"
        ctx = kvsep.Context(0)
        ctx.set_kernel("narrow")
        out = torch.full((n,), SENT - (1 << 32), dtype=torch.int32, device=dev)
        fb = torch.zeros(1, dtype=torch.int64, device=dev)
        nb = torch.zeros(1, dtype=torch.int64, device=dev)
        ctx.verify_device(d.data_ptr(), u64(off), u64(ln), torch.from_numpy(masked.view(np.int32)).to(dev),
                          out, fb, nb, max_len=int(ln.max()), total_bytes=int(ln.sum()))
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        bad = np.nonzero(got != exp)[0]
        print(f"variant {v} n={n} maxlen={maxlen}: {len(bad)} wrong, nbad={int(nb.item())}, "
              f"first_bad={int(fb.item())}", flush=True)
        ctx.close()
        if not len(bad):
            continue
        cls = collections.Counter()
        bygroup = collections.Counter()
        byslot = collections.Counter()
        rel = collections.Counter()
        examples = []
        for b in bad[:4000]:  # a sample is enough to classify
            b = int(b)
            lo, W, k, s = where[b]
            bygroup[k] += 1
            byslot[s] += 1
            g = int(got[b])
            if g == SENT:
                cls["unwritten"] += 1
                continue
            others = [o for o in crc_to_blocks.get(g, []) if o != b]
            if others:
                o = min(others, key=lambda x: abs(x - b))
                if o in where:
                    lo2, W2, k2, s2 = where[o]
                    rel[("same window" if W2 == W else "other window", k2 - k, s2 - s)] += 1
                cls["other-block"] += 1
                if len(examples) < 8:
                    examples.append((b, where[b], "crc of", o, where.get(o)))
                continue
            # same bytes, another length / start?
            L = int(ln[b])
            o0 = int(off[b])
            hit = None
            for L2 in range(0, maxlen + 64):
                if oracle.extend(0, host[o0:o0 + L2].tobytes()) == g:
                    hit = ("len", L2 - L)
                    break
            if hit is None:
                for dlt in range(-64, 65):
                    if 0 <= o0 + dlt and oracle.extend(0, host[o0 + dlt:o0 + dlt + L].tobytes()) == g:
                        hit = ("shift", dlt)
                        break
            cls["other:" + (str(hit) if hit else "?")] += 1
            if len(examples) < 8:
                examples.append((b, where[b], L, hex(g), hit))
        print("  classes:", dict(cls.most_common(12)))
        print("  by group k:", dict(sorted(bygroup.items())), " by slot:", dict(sorted(byslot.items())))
        if rel:
            print("  other-block relation (window, dk, dslot):", dict(rel.most_common(10)))
        for e in examples:
            print("   e.g.", e)
