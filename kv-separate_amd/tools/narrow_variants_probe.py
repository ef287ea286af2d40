#!/usr/bin/env python3
"""Narrow-kernel variants of the KVSEP_DIAG build (KVSEP_NARROW=<k>) on small-block batches: bit-exactness against
the oracle on ragged blocks at every offset mod 128 (every variant must pass before its time means anything), then
the per-launch time of each variant averaged over 20 back-to-back launches in one hipGraph replay (bench.py's
config-2 timing), interleaved in one process over the same buffers.
usage: narrow_variants_probe.py --variants 6,30,31 [--sizes 256,1024] [--rounds 5]"""
import argparse
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
from kvsep import workloads as W  # noqa: E402

dev = torch.device("cuda:0")
u64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)  # noqa: E731


def contexts(variants):
    ctxs = {}
    for v in variants:
        os.environ["KVSEP_NARROW"], os.environ["KVSEP_CRC_VARIANT"] = str(v), "1"
        ctxs[v] = kvsep.Context(0)
    return ctxs


def parity(ctxs):
    oracle = load_oracle()
    rng = np.random.default_rng(11)
    n = 30000
    ln = rng.integers(0, 9000, n).astype(np.uint64)
    ln[: n // 2] = rng.choice([0, 1, 15, 16, 17, 100, 127, 128, 129, 255, 256, 4096, 4097, 4111, 8192], n // 2)
    ln[-5:] = [70000, 3, 200000, 5, 1 << 20]  # longer than the hint: the deferred walk
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1] + rng.integers(0, 130, n - 1).astype(np.uint64), dtype=np.uint64)
    host = splitmix64_bytes(int(off[-1] + ln[-1]) + 256, 5, 0)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    exp = oracle.batch(host, off, ln, init, threads=8)
    d = torch.from_numpy(host).to(dev)
    ok = True
    for v, ctx in ctxs.items():
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        ctx.batch_device(d.data_ptr(), u64(off), u64(ln), out, init=torch.from_numpy(init.view(np.int32)).to(dev),
                         max_len=8192, total_bytes=int(ln.sum()))
        torch.cuda.synchronize()
        bad = int((out.cpu().numpy().view(np.uint32) != exp).sum())
        print(f"parity n{v}: {bad} / {n} mismatches", flush=True)
        ok &= bad == 0
    # many groups per wave (dynamic schedules grab most of them): 400 K blocks of 0..2000 B, hint 1024 (a third of the
    # blocks over it: the deferred path) and the true hint
    n = 400000
    ln = rng.integers(0, 2001, n).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1] + rng.integers(0, 3, n - 1).astype(np.uint64), dtype=np.uint64)
    host = splitmix64_bytes(int(off[-1] + ln[-1]) + 256, 6, 0)
    exp = oracle.batch(host, off, ln, None, threads=8)
    d = torch.from_numpy(host).to(dev)
    for v, ctx in ctxs.items():
        for hint in (1024, 2000):
            out = torch.zeros(n, dtype=torch.int32, device=dev)
            for rep in range(3):  # back to back: each launch must leave the queue words as it found them
                ctx.batch_device(d.data_ptr(), u64(off), u64(ln), out, max_len=hint, total_bytes=int(ln.sum()))
            torch.cuda.synchronize()
            bad = int((out.cpu().numpy().view(np.uint32) != exp).sum())
            print(f"parity n{v} 400K hint {hint}: {bad} / {n} mismatches", flush=True)
            ok &= bad == 0
    return ok


def graph_us(fn, ctx, reps=20):
    fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for _ in range(reps):
                fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    del g  # the graph is gone: its capture set may serve the next capture
    ctx.release_captures()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="6,30,31")
    ap.add_argument("--sizes", default="256,1024")
    ap.add_argument("--block", type=int, default=4096)
    ap.add_argument("--stride", type=int, default=0)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    variants = [int(v) for v in args.variants.split(",")]
    ctxs = contexts(variants)
    if not parity(ctxs):
        sys.exit(1)
    for mib in (int(x) for x in args.sizes.split(",")):
        count = mib * (1 << 20) // args.block
        off, ln = W.uniform_layout(count, args.block, args.stride or None)
        span = int(off[-1] + ln[-1])
        total = int(ln.sum())
        data = torch.empty(span + 64, dtype=torch.uint8, device=dev)
        kvsep.fill_splitmix64(data.data_ptr(), span, 1, 0)
        d_off, d_len = u64(off), u64(ln)
        outs = {v: torch.zeros(count, dtype=torch.int32, device=dev) for v in variants}
        times = {v: [] for v in variants}
        for v in variants:
            ctxs[v].reserve(count, total)
        for _ in range(args.rounds):
            for v in variants:
                times[v].append(graph_us(lambda v=v: ctxs[v].batch_device(
                    data.data_ptr(), d_off, d_len, outs[v], count=count, total_bytes=total, max_len=args.block,
                    stream=torch.cuda.current_stream()), ctxs[v]))
        ref = outs[variants[0]].cpu()
        for v in variants:
            t = sorted(times[v])
            print(f"{mib:5d} MiB of {args.block}-B blocks{' stride ' + str(args.stride) if args.stride else ''} n{v:<3d}"
                  f" min {t[0]:8.2f} us  med {t[len(t) // 2]:8.2f} us  {total / t[len(t) // 2] / 1e6:6.3f} TB/s"
                  f"  same={bool(torch.equal(outs[v].cpu(), ref))}", flush=True)
        del data, d_off, d_len, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
