#!/usr/bin/env python3
"""Many consecutive config-2 batches (256 MiB of 4 KiB blocks each, as a compaction emits SST blocks): issued on
one stream, or alternated over two streams (one context per stream), so each batch's launch ramp can run under
the previous one's tail.  Wall time over N batches (HIP events on the issuing side, all work resident in HBM),
every result checked against the single-stream results.  Usage: stream_overlap_probe.py [batches] [reps]"""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from kvsep import workloads as W  # noqa: E402


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 16
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
    dev = torch.device("cuda:0")
    off, ln = W.cfg2_layout()
    per = int(ln.sum())
    data = torch.empty(nb * per + 64, dtype=torch.uint8, device=dev)
    kvsep.fill_splitmix64(data.data_ptr(), data.numel(), 5, 0)
    d_off = torch.from_numpy(off.view(np.int64)).to(dev)
    d_len = torch.from_numpy(ln.view(np.int64)).to(dev)
    outs = [torch.zeros(off.size, dtype=torch.int32, device=dev) for _ in range(nb)]
    ctxs = [kvsep.Context(0), kvsep.Context(0)]
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    for c in ctxs:
        c.reserve(off.size, per)

    def run(nstreams):
        for i in range(nb):
            k = i % nstreams
            ctxs[k].batch_device(data.data_ptr() + i * per, d_off, d_len, outs[i], total_bytes=per,
                                 max_len=int(ln.max()), stream=streams[k])

    ref = None
    for nstreams in (1, 2, 1, 2):
        times = []
        for _ in range(reps + 1):
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for s in streams:
                s.wait_event(e0)
            run(nstreams)
            for s in streams:
                e = torch.cuda.Event()
                e.record(s)
                torch.cuda.current_stream().wait_event(e)
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1))
        got = torch.stack(outs).cpu().numpy()
        if ref is None:
            ref = got.copy()
        assert np.array_equal(got, ref)
        ms = float(np.median(times[1:]))
        print(f"{nstreams} stream(s): {nb} batches of 256 MiB in {ms:.3f} ms = {ms * 1e3 / nb:.1f} us per batch, "
              f"{nb * per / (ms * 1e-3) / 1e9:.0f} GB/s", flush=True)


if __name__ == "__main__":
    main()
