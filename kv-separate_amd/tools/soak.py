#!/usr/bin/env python3
"""Randomised bit-exactness soak of the shipped library against the oracle, time-bounded: batch shapes the test
suite samples only sparsely -- up to 200 K blocks, length mixes (uniform, Zipf, around 4 KiB, tiny, mixed with
long), any byte offset, overlapping blocks, random or no inits -- through every kernel choice (auto, wide, narrow16,
narrow8, sorted), every hint kind (none, exact, loose, understated), three piece sizes, the verify form with
corrupted expectations, the host forms (pinned-staged span, pointer per block, a two-member device group), a
hipGraph-captured device call, and the SST forms (trailer words; the read check over a file image with planted bad
trailers).  Every result is compared with the oracle on the same bytes; prints one line per case and
a summary, exits non-zero on the first mismatch.  usage: soak.py [--seconds 240] [--seed N]
tests/test_gpu_soak.py runs a fixed, seeded number of these cases (soak(seed, max_cases=...)) in the -m gpu suite."""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from conftest import load_oracle  # noqa: E402  (the checker)
from kvsep import splitmix64_bytes  # noqa: E402

POOL = 192 << 20
KERNELS = ("auto", "wide", "narrow16", "narrow8", "sorted", "claim", "claim16", "coop")


def lengths(rng, n, kind):
    if kind == "uniform":
        return rng.integers(0, int(rng.choice([64, 4096, 40000, 300000])) + 1, n)
    if kind == "zipf":  # SURVEY config-4 style classes, capped
        k = rng.choice(14, n, p=(np.arange(1, 15) ** -1.1) / (np.arange(1, 15) ** -1.1).sum())
        lo = 32 * (1 << k)
        return rng.integers(lo, 2 * lo)
    if kind == "sst":  # ~4 KiB blocks
        return 4096 + rng.integers(-300, 300, n)
    if kind == "tiny":
        return rng.integers(0, 40, n)
    # mixed: mostly short, a few long
    ln = rng.integers(0, 5000, n)
    m = rng.random(n) < 0.02
    ln[m] = rng.integers(100000, 3 << 20, int(m.sum()))
    return ln


def bad_rate(rng):
    """Fraction of planted mismatches in a verify case: none, a few, 1 %, a third, or every block (round 5: the verify
    form posts one verdict per workgroup, so the all-bad batch is its own path)."""
    return float(rng.choice([0.0, 1e-4, 0.01, 0.33, 1.01], p=[0.15, 0.2, 0.35, 0.15, 0.15]))


class Mismatch(AssertionError):
    pass


def soak(seed, seconds=None, max_cases=None, log=print, pool=POOL):
    """Random cases until `seconds` elapse or `max_cases` ran; raises Mismatch on the first wrong result.
    -> (cases, blocks, bytes)."""
    POOL = pool  # noqa: N806
    rng = np.random.default_rng(seed)
    oracle = load_oracle()
    dev = torch.device("cuda:0")
    host = splitmix64_bytes(POOL, seed, 0)
    d = torch.from_numpy(host).to(dev)
    ctxs = {}
    for piece in (None, 4096, 64 * 1024):
        for k in KERNELS:
            c = kvsep.Context(0)
            if piece:
                c.set_piece_bytes(piece)
            c.set_kernel(k)
            ctxs[(piece, k)] = c
    group = kvsep.Group([0, 0])  # two contexts on the one GPU: the byte-balanced split and the merged results
    u64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)  # noqa: E731
    t_end = time.time() + seconds if seconds else float("inf")
    cases = blocks = nbytes = 0
    while time.time() < t_end and (max_cases is None or cases < max_cases):
        n = int(rng.choice([1, 7, 64, 513, 4096, 20000, 70000, 200000]))
        kind = str(rng.choice(["uniform", "zipf", "sst", "tiny", "mixed"]))
        ln = np.clip(lengths(rng, n, kind), 0, POOL // 4).astype(np.uint64)
        if int(ln.sum()) > 2 * POOL:  # keep the oracle pass short
            ln = (ln // np.uint64(max(1, int(ln.sum()) // POOL + 1))).astype(np.uint64)
        if rng.random() < 0.5:  # packed (optionally with gaps), else random (overlapping) offsets
            gaps = rng.integers(0, 2 if rng.random() < 0.5 else 129, n).astype(np.uint64)
            off = np.zeros(n, np.uint64)
            off[1:] = np.cumsum(ln[:-1] + gaps[:-1], dtype=np.uint64)
            off += np.uint64(rng.integers(0, 128))
            if int(off[-1] + ln[-1]) > POOL:
                off = (rng.integers(0, POOL, n).astype(np.uint64) % (np.uint64(POOL + 1) - ln))
        else:
            off = (rng.integers(0, POOL, n).astype(np.uint64) % (np.uint64(POOL + 1) - ln))
        init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32) if rng.random() < 0.6 else None
        hint = str(rng.choice(["none", "exact", "loose", "under"]))
        mx = int(ln.max())
        max_len = {"none": 0, "exact": mx, "loose": 2 * mx + 1, "under": max(1, mx // 3)}[hint]
        piece = [None, 4096, 64 * 1024][int(rng.integers(0, 3))]
        kern = str(rng.choice(KERNELS))
        ctx = ctxs[(piece, kern)]
        exp = oracle.batch(host, off, ln, init, threads=8)
        d_init = torch.from_numpy(init.view(np.int32)).to(dev) if init is not None else None
        out = torch.zeros(n, dtype=torch.int32, device=dev)
        form = str(rng.choice(["device", "device", "device", "host_span", "host_ptrs", "group", "graph", "sst"]))
        if form == "sst" and n > 20000:
            form = "device"
        verify = form == "device" and rng.random() < 0.4
        if form != "device":
            if form == "host_span":
                got = ctx.batch_host_span(host, off, ln, init)
            elif form == "host_ptrs":
                k = min(n, 4096)  # one Python buffer object per block
                sub = [memoryview(host)[int(off[i]):int(off[i] + ln[i])] for i in range(k)]
                got = np.concatenate([ctx.batch_host(sub, None if init is None else init[:k]),
                                      np.asarray(exp[k:], np.uint32)])
            elif form == "group":
                got = group.batch_host_span(host, off, ln, init)
            elif form == "sst":  # table/table_builder.cc:209-232 and table/format.cc:99-108 over a file image
                types = rng.integers(0, 2, n).astype(np.uint8)
                pos = np.zeros(n, np.uint64)
                pos[1:] = np.cumsum(ln[:-1] + np.uint64(5), dtype=np.uint64)
                pos += np.uint64(rng.integers(0, 16))
                img = splitmix64_bytes(int(pos[-1] + ln[-1]) + 5, seed + cases, 0).copy()
                img[(pos + ln).astype(np.int64)] = types
                crc = oracle.batch(img, pos, ln + np.uint64(1))  # Value(block || type)
                c64 = crc.astype(np.uint64)
                stored = ((((c64 >> np.uint64(15)) | (c64 << np.uint64(17))) + np.uint64(0xA282EAD8))
                          & np.uint64(0xFFFFFFFF))
                for k in range(4):
                    img[(pos + ln + np.uint64(1 + k)).astype(np.int64)] = ((stored >> np.uint64(8 * k)) & 0xFF).astype(np.uint8)
                bad = rng.random(n) < bad_rate(rng)
                img[(pos[bad] + ln[bad] + np.uint64(1)).astype(np.int64)] ^= np.uint8(1)
                d_img = torch.from_numpy(img).to(dev)
                tw = torch.zeros(n, dtype=torch.int32, device=dev)
                ctx.sst_trailers_device(d_img.data_ptr(), u64(pos), u64(ln), torch.from_numpy(types).to(dev), tw,
                                        total_bytes=int(ln.sum()), max_len=max_len)
                fb = torch.zeros(1, dtype=torch.int64, device=dev)
                nb = torch.zeros(1, dtype=torch.int64, device=dev)
                ctx.sst_verify_device(d_img.data_ptr(), u64(pos), u64(ln), out, fb, nb, total_bytes=int(ln.sum()),
                                      max_len=max_len)
                torch.cuda.synchronize()
                got = out.cpu().numpy().view(np.uint32)
                exp = crc
                tw_ok = np.array_equal(tw.cpu().numpy().view(np.uint32), stored.astype(np.uint32))
                want_fb = int(np.argmax(bad)) if bad.any() else -1
                if not tw_ok or int(nb.item()) != int(bad.sum()) or (bad.any() and int(fb.item()) != want_fb):
                    raise Mismatch(f"seed {seed}: case {cases + 1} sst: trailers {'ok' if tw_ok else 'WRONG'}, nbad "
                                   f"{int(nb.item())} vs {int(bad.sum())}, first_bad {int(fb.item())} vs {want_fb}")
            else:  # graph: capture one device call, replay it twice
                ctx.reserve(n, int(ln.sum()))
                out = torch.zeros(n, dtype=torch.int32, device=dev)
                d_off, d_len = u64(off), u64(ln)
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g):
                    ctx.batch_device(d.data_ptr(), d_off, d_len, out, init=d_init, max_len=max_len,
                                     total_bytes=int(ln.sum()), stream=torch.cuda.current_stream())
                out.zero_()
                g.replay()
                g.replay()
                torch.cuda.synchronize()
                got = out.cpu().numpy().view(np.uint32)
                del g  # the graph is gone: its capture set may serve the next capture (kvsep_crc32c_release_captures)
                ctx.release_captures()
            mism = int(np.count_nonzero(np.asarray(got, np.uint32) != exp))
            cases += 1
            blocks += n
            nbytes += int(ln.sum())
            msg = (f"case {cases}: n={n} {kind} hint={hint}({max_len}) piece={piece} kernel={kern} form={form} -> "
                   f"{'ok' if not mism else f'{mism} MISMATCHES'}")
            log(msg)
            if mism:
                raise Mismatch(f"seed {seed}: {msg}")
            continue
        if verify:
            masked = np.array([kvsep.mask(int(x)) for x in exp], dtype=np.uint32)
            bad = rng.random(n) < bad_rate(rng)
            masked[bad] ^= np.uint32(1 << int(rng.integers(0, 32)))
            fb = torch.zeros(1, dtype=torch.int64, device=dev)
            nb = torch.zeros(1, dtype=torch.int64, device=dev)
            ctx.verify_device(d.data_ptr(), u64(off), u64(ln), torch.from_numpy(masked.view(np.int32)).to(dev), out,
                              fb, nb, init=d_init, max_len=max_len, total_bytes=int(ln.sum()))
        else:
            ctx.batch_device(d.data_ptr(), u64(off), u64(ln), out, init=d_init, max_len=max_len,
                             total_bytes=int(ln.sum()))
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        mism = int(np.count_nonzero(got != exp))
        ok = mism == 0
        if verify:
            want_fb = int(np.argmax(bad)) if bad.any() else -1
            ok &= int(nb.item()) == int(bad.sum()) and (int(fb.item()) == want_fb if bad.any() else
                                                         (int(fb.item()) & 0xFFFFFFFFFFFFFFFF) == 0xFFFFFFFFFFFFFFFF)
        cases += 1
        blocks += n
        nbytes += int(ln.sum())
        msg = (f"case {cases}: n={n} {kind} hint={hint}({max_len}) piece={piece} kernel={kern} "
               f"({ctx.kernel_name(n, max_len, int(ln.sum()))}) verify={verify} -> {'ok' if ok else f'{mism} MISMATCHES'}")
        log(msg)
        if not ok:
            raise Mismatch(f"seed {seed}: {msg}")
    for c in ctxs.values():
        c.close()
    group.close()
    return cases, blocks, nbytes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=240)
    ap.add_argument("--seed", type=int, default=int(time.time()) & 0xFFFFFFFF)
    args = ap.parse_args()
    print(f"seed {args.seed}", flush=True)
    try:
        cases, blocks, nbytes = soak(args.seed, seconds=args.seconds, log=lambda m: print(m, flush=True))
    except Mismatch as e:
        print(e, flush=True)
        sys.exit(1)
    print(f"soak ok: {cases} cases, {blocks} blocks, {nbytes / 2**30:.2f} GiB, seed {args.seed}", flush=True)


if __name__ == "__main__":
    main()
