#!/usr/bin/env python3
"""Interleaved A/B of kernel variants in ONE process (cdna_hip_programming.md §5.4 rule 24).

usage: python ab_variants.py --variants 1,2 --configs 3a,2 --rounds 5 --steps 5
Prints per (config, variant) the median / min kernel time and GB/s (kernel-only HIP events).
A variant written "b<N>" runs variant N of a second build of the library (--lib-b), so two source versions
are compared in one process on one box; "n<K>" selects narrow-kernel variant K (KVSEP_NARROW) for short blocks;
"<N>p<KiB>" runs variant N with its own piece size; a trailing "s" / "d" forces the static / guided schedule, and a
final "w" the wide kernel.
"""
import argparse
import os
import statistics
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from kvsep import workloads as W  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import _diag  # noqa: E402,F401  -- variant "a" is the KVSEP_DIAG build (its default = the shipped kernels)


def layout(cfg):
    if cfg.startswith("u"):  # "u<count>x<len>[s<stride>][f<first>]": uniform blocks (packed unless s), e.g. u4096x4096
        import re
        m = re.fullmatch(r"u(\d+)x(\d+)(?:s(\d+))?(?:f(\d+))?", cfg)
        count, length, stride, first = m.groups()
        return W.uniform_layout(int(count), int(length), int(stride) if stride else None, int(first or 0))
    if cfg.startswith("r"):  # "r<count>x<max>": ragged, lengths uniform in [1, max], packed
        count, mx = (int(x) for x in cfg[1:].split("x"))
        ln = np.random.default_rng(3).integers(1, mx + 1, count).astype(np.uint64)
        off = np.zeros(count, np.uint64)
        off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
        return off, ln
    if cfg == "4s":  # config 4's blocks of <= 32 KiB only (86 % of its blocks, 1 % of its bytes)
        off, ln = W.cfg4_layout()
        return off[ln <= 32768], ln[ln <= 32768]
    return {"3a": W.cfg3_layout, "3b": lambda: W.cfg3_layout(vlog=True), "2": W.cfg2_layout,
            "4": W.cfg4_layout}[cfg]()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variants", default="1,2")
    ap.add_argument("--configs", default="3a,2")
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--piece-kib", type=int, default=0)
    ap.add_argument("--lib-b", default=os.path.join(os.path.dirname(os.path.abspath(__file__)), "libkvsep_b.so"))
    args = ap.parse_args()
    variants = args.variants.split(",")
    libs = {"a": kvsep.lib()}
    if any(v.startswith("b") for v in variants):
        saved = kvsep.LIB_PATH, kvsep._lib
        kvsep.LIB_PATH, kvsep._lib = args.lib_b, None
        libs["b"] = kvsep.lib()
        kvsep.LIB_PATH, kvsep._lib = saved

    def use(v):  # point the binding at the build variant v belongs to
        kvsep._lib = libs["b" if v.startswith("b") else "a"]

    ctxs = {}
    for v in variants:
        use(v)
        code = v[1:] if v.startswith("b") else v
        piece_kib = args.piece_kib
        sched = None
        wide = code.endswith("w")  # "<variant>w": the wide kernel even where the narrow one would be chosen
        if wide:
            code = code[:-1]
        if code[-1:] in ("s", "d", "r"):  # "<variant>s" / "d" / "r": static contiguous / guided / static round-robin
            sched, code = {"s": False, "d": True, "r": "rr"}[code[-1]], code[:-1]
        if "p" in code:  # "<variant>p<KiB>": that variant with its own piece size, e.g. 1p128 vs 1p1024
            code, pk = code.split("p")
            piece_kib = int(pk)
        if code.startswith("n"):  # "n<k>": narrow-kernel variant k (KVSEP_NARROW), default wide variant
            os.environ["KVSEP_NARROW"], os.environ["KVSEP_CRC_VARIANT"] = code[1:], "1"
        else:
            os.environ["KVSEP_NARROW"], os.environ["KVSEP_CRC_VARIANT"] = "1", code
        ctxs[v] = kvsep.Context(0)
        if piece_kib:
            ctxs[v].set_piece_bytes(piece_kib * 1024)
        if sched is not None:
            ctxs[v].set_schedule(sched)
        if wide:
            ctxs[v].set_kernel("wide")
    dev = torch.device("cuda:0")
    for cfg in args.configs.split(","):
        off, ln = layout(cfg)
        span = int(off[-1] + ln[-1])
        useful = int(ln.sum())
        data = torch.empty(span + 64, dtype=torch.uint8, device=dev)
        kvsep.fill_splitmix64(data.data_ptr(), span, 5, 0)
        d_off = torch.from_numpy(off.view(np.int64)).to(dev)
        d_len = torch.from_numpy(ln.view(np.int64)).to(dev)
        outs = {v: torch.zeros(off.size, dtype=torch.int32, device=dev) for v in variants}
        res = {v: [] for v in variants}
        for v in variants:
            use(v)
            ctxs[v].reserve(off.size, useful)
            ctxs[v].batch_device(data.data_ptr(), d_off, d_len, outs[v], total_bytes=useful, max_len=int(ln.max()))
        torch.cuda.synchronize()
        for _ in range(args.rounds):
            for v in variants:
                use(v)
                c = ctxs[v]
                c.set_timing(True)
                for _ in range(args.steps):
                    c.batch_device(data.data_ptr(), d_off, d_len, outs[v], total_bytes=useful, max_len=int(ln.max()))
                torch.cuda.synchronize()
                c.set_timing(False)
                ms, n = c.get_timing()
                res[v].append(ms / n)
        ref = outs[variants[0]].cpu()
        for v in variants:
            same = bool(torch.equal(outs[v].cpu(), ref))
            med, mn = statistics.median(res[v]), min(res[v])
            print(f"cfg {cfg:3s} variant {v:>3s}: median {med:.4f} ms ({useful / med / 1e6:.1f} GB/s)  "
                  f"min {mn:.4f} ms ({useful / mn / 1e6:.1f} GB/s)  same_as_v{variants[0]}={same}", flush=True)
        del data, d_off, d_len, outs
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
