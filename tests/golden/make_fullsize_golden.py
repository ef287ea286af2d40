#!/usr/bin/env python3
"""Per-block CRCs of the WHOLE BASELINE batches, computed by the REAL reference (util/crc32c.cc compiled into
oracle/_ref/libref_crc32c.so by oracle/Makefile; the data generated block by block by ref_crc32c_stream_batch in
oracle/ref_shim.cc, so no batch is ever held in memory).  Runs only where /root/reference exists (this container).

Files (little-endian u32, one per block, in block order):
  full_cfg2.u32   config 2: 65,536 x 4 KiB packed, stream SEED from 0                         (256 KiB)
  full_cfg3a.u32  config 3a: 65,536 x 1 MiB packed, stream SEED+1 from 0                      (256 KiB)
  full_cfg5.u32   config 5: the 512 GiB vlog, 524,288 records of 1,048,609 B at 8 + i*(8+len) of stream SEED+1;
                  slice s (records [s*65,536, (s+1)*65,536)) is a config-3b batch at stream offset s*span, and
                  slice 0 IS config 3b                                                         (2 MiB)
  full_cfg4.u32   config 4: 1,048,576 Zipf blocks packed, stream SEED+2 from 0                 (4 MiB)
The seeds and stream offsets are the ones bench.py uses, so a bench run can be checked against these too.
"""
import ctypes
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


def stream_batch(r, seed, base, off, ln, threads):
    out = np.zeros(off.size, np.uint32)
    off = np.ascontiguousarray(off, np.uint64)
    ln = np.ascontiguousarray(ln, np.uint64)
    assert r.ref_crc32c_stream_batch(seed, base, off.ctypes.data, ln.ctypes.data, off.size, out.ctypes.data,
                                     threads) == 0
    return out


def main():
    subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "ref"])
    r = ctypes.CDLL(REF_SO)
    r.ref_crc32c_stream_batch.restype = ctypes.c_int
    r.ref_crc32c_stream_batch.argtypes = [ctypes.c_uint64, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_size_t, ctypes.c_void_p, ctypes.c_int]
    threads = len(os.sched_getaffinity(0))
    jobs = {"full_cfg2.u32": lambda: stream_batch(r, W.SEED, 0, *W.cfg2_layout(), threads),
            "full_cfg3a.u32": lambda: stream_batch(r, W.SEED + 1, 0, *W.cfg3_layout(), threads),
            "full_cfg4.u32": lambda: stream_batch(r, W.SEED + 2, 0, *W.cfg4_layout(), threads)}

    def cfg5():
        off, ln = W.cfg3_layout(vlog=True)
        span = int(off[-1] + ln[-1])
        return np.concatenate([stream_batch(r, W.SEED + 1, s * span, off, ln, threads) for s in range(CFG5_SLICES)])

    jobs["full_cfg5.u32"] = cfg5
    for name, fn in jobs.items():
        t = time.time()
        a = fn()
        a.astype("<u4").tofile(os.path.join(HERE, name))
        print(f"{name}: {a.size} blocks in {time.time() - t:.1f} s", flush=True)


if __name__ == "__main__":
    main()
