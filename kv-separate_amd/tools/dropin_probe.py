#!/usr/bin/env python3
"""Where should the scalar drop-in (kvsep_crc32c_extend, the util/crc32c.h:17 replacement) hand a single buffer
to the GPU?  Times one Extend over a pageable buffer of each size on the host leg and through the GPU
(threshold forced to 0), single caller and with 8 concurrent callers (the reference calls Extend from the
writer, compaction, GC and reader threads at once, db/db_impl.cc:1829-1833).  Prints one line per size."""
import json
import os
import sys
import threading
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402

GIB = float(1 << 30)


def rate(fn, nbytes, threads, seconds=0.6):
    fn()
    stop = time.perf_counter() + seconds
    done = [0] * threads

    def work(t):
        while time.perf_counter() < stop:
            fn()
            done[t] += 1

    t0 = time.perf_counter()
    ths = [threading.Thread(target=work, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    for th in ths:
        th.join()
    dt = time.perf_counter() - t0
    return sum(done) * nbytes / GIB / dt, dt * 1e6 / max(1, sum(done)) * threads


def main():
    L = kvsep.lib()
    rows = []
    for n in (256 << 10, 1 << 20, 4 << 20, 16 << 20, 64 << 20, 256 << 20):
        buf = np.random.default_rng(n).integers(0, 256, n, dtype=np.uint8)
        p = buf.ctypes.data
        want = kvsep.extend_host(0, buf)
        row = {"bytes": n}
        # gpu: every call queues for the GPU leg (wait 1); divert: the default policy, a caller that finds the GPU
        # leg busy runs the host leg (wait 0)
        for name, thr, wait in (("host", 1 << 62, 1), ("gpu", 0, 1), ("divert", 0, 0)):
            L.kvsep_set_offload_threshold(thr)
            L.kvsep_set_offload_wait(wait)
            assert L.kvsep_crc32c_extend(0, p, n) == want
            for threads in (1, 8):
                g, us = rate(lambda: L.kvsep_crc32c_extend(0, p, n), n, threads)
                row[f"{name}_{threads}t_GiBps"] = round(g, 2)
                row[f"{name}_{threads}t_us_per_call"] = round(us, 1)
        print(json.dumps(row), flush=True)
        rows.append(row)
    L.kvsep_set_offload_threshold(64 << 20)
    L.kvsep_set_offload_wait(0)
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(rows, f, indent=1)


if __name__ == "__main__":
    torch.cuda.init()
    main()
