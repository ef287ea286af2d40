#!/usr/bin/env python3
"""Per-block CRCs of the WHOLE BASELINE batches, computed by the REAL reference (util/crc32c.cc compiled into
oracle/_ref/libref_crc32c.so by oracle/Makefile; the data generated block by block by ref_crc32c_stream_batch in
oracle/ref_shim.cc, so no batch is ever held in memory).  Runs only where /root/reference exists (this container).

The files cover the GLOBAL batch bench.py builds at up to 8 ranks, so every block of an N-rank bench line (N = 1, 2,
4, 8) is checked against the reference:
  full_cfg2.u32   config 2 over 8 ranks: rank r's 65,536 x 4 KiB blocks sit at stream bytes r*256 MiB + i*4096 of
                  stream SEED, i.e. one packed batch of 8 x 65,536 blocks; entry r*65,536 + i          (2 MiB)
  full_cfg3a.u32  config 3a over 8 ranks: 8 x 65,536 x 1 MiB packed, stream SEED+1 from 0 (512 GiB)     (2 MiB)
  full_cfg5.u32   config 5: the 512 GiB vlog, 524,288 records of 1,048,609 B at 8 + i*(8+len) of stream SEED+1;
                  slice s (records [s*65,536, (s+1)*65,536)) is a config-3b batch at stream offset s*span, and
                  slice 0 IS config 3b; config 3b at N ranks is slices 0..N-1                           (2 MiB)
  full_cfg4.u32   config 4: 1,048,576 Zipf blocks packed, stream SEED+2 from 0                          (4 MiB)
  full_cfg4_ranks.json
                  config 4 at N = 1, 2, 4, 8 ranks: ONE global batch of N x 2^20 Zipf blocks (its first 2^20 are
                  config 4), cut by kvsep_crc32c_partition into byte-balanced block ranges.  The reference's
                  per-block CRCs of the 8-rank batch (8 Mi blocks, 1.2 TiB) are 32 MiB, too much to commit, so the
                  file holds, for every (N, rank), the range [lo, hi) and crc_of_crcs -- the reference's
                  Extend(0, LE u32 CRCs of blocks lo..hi-1) (kvsep/shard.py crc_of_crcs) -- plus the xor of them.
The seeds and stream offsets are the ones bench.py uses, so a bench run can be checked against these too.

  python3 tests/golden/make_fullsize_golden.py [--only full_cfg3a.u32 ...]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "kv-separate_amd"))
from kvsep import workloads as W  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_crc32c.so")
CFG5_SLICES = 8
MAX_RANKS = 8
RANK_COUNTS = (1, 2, 4, 8)


def stream_batch(r, seed, base, off, ln, threads):
    out = np.zeros(off.size, np.uint32)
    off = np.ascontiguousarray(off, np.uint64)
    ln = np.ascontiguousarray(ln, np.uint64)
    assert r.ref_crc32c_stream_batch(seed, base, off.ctypes.data, ln.ctypes.data, off.size, out.ctypes.data,
                                     threads) == 0
    return out


def ref_digest(r, crcs):
    """crc_of_crcs (kvsep/shard.py) computed by the reference's Extend over the little-endian u32 results."""
    b = np.ascontiguousarray(crcs, dtype="<u4").tobytes()
    return int(r.ref_crc32c_extend(0, b, len(b)))


def cfg4_ranks(r, threads):
    """The 8-rank global config-4 batch through the reference, then per-(N, rank) digests of the partition bench.py
    uses (kvsep.partition = kvsep_crc32c_partition, host code: no GPU call)."""
    import kvsep
    glen = W.zipf_lengths(MAX_RANKS * W.CFG4_BLOCKS)
    goff = np.zeros(glen.size, np.uint64)
    goff[1:] = np.cumsum(glen[:-1], dtype=np.uint64)
    crcs = stream_batch(r, W.SEED + 2, 0, goff, glen, threads)
    first = np.fromfile(os.path.join(HERE, "full_cfg4.u32"), dtype="<u4")
    assert np.array_equal(crcs[:first.size], first), "the 8-rank batch must extend config 4"
    out = {"seed": W.SEED + 2, "blocks_per_rank": W.CFG4_BLOCKS, "digest": "crc_of_crcs", "ranks": {}}
    for n in RANK_COUNTS:
        b = kvsep.partition(glen[:n * W.CFG4_BLOCKS], n)
        parts = []
        for k in range(n):
            lo, hi = int(b[k]), int(b[k + 1])
            parts.append({"lo": lo, "hi": hi, "bytes": int(glen[lo:hi].sum()), "crc_of_crcs": ref_digest(r, crcs[lo:hi]),
                          "xor": int(np.bitwise_xor.reduce(crcs[lo:hi])) if hi > lo else 0})
        out["ranks"][str(n)] = parts
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", nargs="*", default=None)
    args = ap.parse_args()
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"])
    r = ctypes.CDLL(REF_SO)
    r.ref_crc32c_stream_batch.restype = ctypes.c_int
    r.ref_crc32c_stream_batch.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
    r.ref_crc32c_extend.restype = ctypes.c_uint32
    r.ref_crc32c_extend.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
    threads = len(os.sched_getaffinity(0))

    def packed(layout, seed):
        off, ln = layout()
        span = int(off[-1] + ln[-1])  # rank r's block i is global block r*count + i at stream bytes r*span + off[i]
        return np.concatenate([stream_batch(r, seed, k * span, off, ln, threads) for k in range(MAX_RANKS)])

    def cfg5():
        off, ln = W.cfg3_layout(vlog=True)
        span = int(off[-1] + ln[-1])
        return np.concatenate([stream_batch(r, W.SEED + 1, s * span, off, ln, threads) for s in range(CFG5_SLICES)])

    jobs = {"full_cfg2.u32": lambda: packed(W.cfg2_layout, W.SEED),
            "full_cfg3a.u32": lambda: packed(W.cfg3_layout, W.SEED + 1),
            "full_cfg4.u32": lambda: stream_batch(r, W.SEED + 2, 0, *W.cfg4_layout(), threads),
            "full_cfg5.u32": cfg5,
            "full_cfg4_ranks.json": lambda: cfg4_ranks(r, threads)}
    for name, fn in jobs.items():
        if args.only is not None and name not in args.only:
            continue
        t = time.time()
        a = fn()
        path = os.path.join(HERE, name)
        if name.endswith(".json"):
            with open(path, "w") as f:
                json.dump(a, f, indent=1)
            print(f"{name}: written in {time.time() - t:.1f} s", flush=True)
        else:
            a.astype("<u4").tofile(path)
            print(f"{name}: {a.size} blocks in {time.time() - t:.1f} s", flush=True)


if __name__ == "__main__":
    main()
