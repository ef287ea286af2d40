#!/usr/bin/env python3
"""The cooperative narrow kernel (set_kernel("coop"), narrow form 12) against the claim kernel on the shipped library:
bit-exactness against the oracle first (ragged blocks at every offset mod 128 with per-block initial CRCs, blocks over
the hint, empty blocks, a verify call with planted mismatches; every kernel must pass before its time means
anything), then graph-replay launch times on uniform blocks, interleaved in one process over the same buffers.
usage: coop_probe.py [--kernels claim,coop] [--sizes 128,256,1024] [--block 4096] [--rounds 5] [--lib PATH]
(--lib: another build of the library, e.g. an A/B copy of the same sources at another commit)"""
import argparse
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from conftest import load_oracle  # noqa: E402  (the checker)
from kvsep import splitmix64_bytes  # noqa: E402
from kvsep import workloads as W  # noqa: E402

dev = torch.device("cuda:0")
u64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)  # noqa: E731


def contexts(kernels):
    ctxs = {}
    for k in kernels:
        ctxs[k] = kvsep.Context(0)
        ctxs[k].set_kernel(k)
    return ctxs


def parity(ctxs):
    oracle = load_oracle()
    rng = np.random.default_rng(12)
    ok = True
    for case in ("ragged", "uniform"):
        if case == "ragged":
            n = 40000
            ln = rng.integers(0, 4097, n).astype(np.uint64)
            ln[: n // 2] = rng.choice([0, 1, 15, 16, 17, 100, 127, 128, 129, 255, 256, 1000, 4095, 4096], n // 2)
            ln[-6:] = [4097, 70000, 3, 200000, 5, 1 << 20]  # longer than the hint: the combining wave's wide path
            gap = rng.integers(0, 130, n - 1).astype(np.uint64)
            hint = 4096
        else:
            n = 100003
            ln = np.full(n, 4096, np.uint64)
            gap = np.full(n - 1, 5, np.uint64)
            hint = 4096
        off = np.zeros(n, np.uint64)
        off[1:] = np.cumsum(ln[:-1] + gap, dtype=np.uint64)
        host = splitmix64_bytes(int(off[-1] + ln[-1]) + 256, 7, 0)
        init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
        exp_i = oracle.batch(host, off, ln, init, threads=8)
        exp = oracle.batch(host, off, ln, None, threads=8)
        d = torch.from_numpy(host).to(dev)
        d_init = torch.from_numpy(init.view(np.int32)).to(dev)
        stored = np.array([kvsep.mask(int(c)) for c in exp], np.uint32)
        bad = [3, n // 2, n - 7]
        stored[bad] ^= np.uint32(0x100)
        d_exp = torch.from_numpy(stored.view(np.int32)).to(dev)
        for k, ctx in ctxs.items():
            for with_init in (False, True):
                out = torch.zeros(n, dtype=torch.int32, device=dev)
                for _ in range(2):
                    ctx.batch_device(d.data_ptr(), u64(off), u64(ln), out, init=d_init if with_init else None,
                                     max_len=hint, total_bytes=int(ln.sum()))
                torch.cuda.synchronize()
                want = exp_i if with_init else exp
                nb = int((out.cpu().numpy().view(np.uint32) != want).sum())
                print(f"parity {k} {case} init={with_init}: {nb} / {n} mismatches", flush=True)
                ok &= nb == 0
            out = torch.zeros(n, dtype=torch.int32, device=dev)
            fb = torch.zeros(1, dtype=torch.int64, device=dev)
            nbad = torch.zeros(1, dtype=torch.int64, device=dev)
            ctx.verify_device(d.data_ptr(), u64(off), u64(ln), d_exp, out, fb, nbad, max_len=hint,
                              total_bytes=int(ln.sum()))
            torch.cuda.synchronize()
            v = (int(fb.item()), int(nbad.item()))
            good = v == (bad[0], len(bad)) and np.array_equal(out.cpu().numpy().view(np.uint32), exp)
            print(f"verify {k} {case}: verdict {v} want {(bad[0], len(bad))} crcs {'exact' if good else 'WRONG'}",
                  flush=True)
            ok &= good
    return ok


def graph_us(fn, ctx, reps=20):
    fn(0)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g, stream=s):
            for i in range(reps):
                fn(i)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    g.replay()
    e1.record()
    torch.cuda.synchronize()
    del g
    ctx.release_captures()
    return e0.elapsed_time(e1) * 1e3 / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--kernels", default="claim,coop")
    ap.add_argument("--sizes", default="128,256,1024")
    ap.add_argument("--block", type=int, default=4096)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--no-parity", action="store_true")
    ap.add_argument("--lib", default=None)
    ap.add_argument("--rotate", type=int, default=1,
                    help="launch i reads copy i mod N of the batch (N copies: no launch finds the previous one's data "
                         "in the 256 MB Infinity Cache once N x batch is well past it)")
    args = ap.parse_args()
    if args.lib:
        kvsep.LIB_PATH = os.path.abspath(args.lib)
    print(f"library {kvsep.LIB_PATH}", flush=True)
    kernels = args.kernels.split(",")
    ctxs = contexts(kernels)
    if not args.no_parity and not parity(ctxs):
        sys.exit(1)
    for mib in (int(x) for x in args.sizes.split(",")):
        count = mib * (1 << 20) // args.block
        off, ln = W.uniform_layout(count, args.block)
        span = int(off[-1] + ln[-1])
        total = int(ln.sum())
        datas = [torch.empty(span + 64, dtype=torch.uint8, device=dev) for _ in range(args.rotate)]
        for data in datas:
            kvsep.fill_splitmix64(data.data_ptr(), span, 1, 0)
        d_off, d_len = u64(off), u64(ln)
        outs = {k: torch.zeros(count, dtype=torch.int32, device=dev) for k in kernels}
        times = {k: [] for k in kernels}
        for k in kernels:
            ctxs[k].reserve(count, total)
        for _ in range(args.rounds):
            for k in kernels:
                times[k].append(graph_us(lambda i, k=k: ctxs[k].batch_device(
                    datas[i % args.rotate].data_ptr(), d_off, d_len, outs[k], count=count, total_bytes=total,
                    max_len=args.block, stream=torch.cuda.current_stream()), ctxs[k]))
        ref = outs[kernels[0]].cpu()
        for k in kernels:
            t = sorted(times[k])
            print(f"{mib:5d} MiB of {args.block}-B blocks x{args.rotate} {k:<8s} min {t[0]:8.2f} us  med {t[len(t) // 2]:8.2f} us"
                  f"  {total / t[len(t) // 2] / 1e6:6.3f} TB/s  same={bool(torch.equal(outs[k].cpu(), ref))}",
                  flush=True)
        del datas, d_off, d_len, outs
        torch.cuda.empty_cache()
    for c in ctxs.values():
        c.close()


if __name__ == "__main__":
    main()
