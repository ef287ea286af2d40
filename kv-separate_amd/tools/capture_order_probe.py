#!/usr/bin/env python3
"""Round 6: do captured graphs keep their node order when several are replayed at once on different streams?
Each graph is one batch call of a context (own capture set); every graph is first replayed alone (so every plan array
holds valid values), then rounds of concurrent replays on three streams with the payload REWRITTEN before each round
(new seed): a graph whose nodes ran out of order (a combine before its pieces kernel, a CRC kernel before the plan)
returns last round's CRCs, which the check sees -- without any wild read, since the plan (lengths only) stays valid.
usage: capture_order_probe.py [planned|unplanned|all] [rounds]"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from conftest import load_oracle  # noqa: E402  (the checker)
from kvsep import workloads as W  # noqa: E402

dev = torch.device("cuda:0")
u64 = lambda a: torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)  # noqa: E731
which = sys.argv[1] if len(sys.argv) > 1 else "planned"
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 6
kinds = {"planned": ["planned"] * 6, "unplanned": ["claim", "sorted", "wide", "claim", "sorted", "wide"],
         "all": ["planned", "claim", "sorted", "wide", "planned", "claim"]}[which]


def layout(kind):
    if kind == "claim":
        off, ln = W.uniform_layout(40000, 4096)
        return off, ln, 4096
    if kind == "sorted":
        rng = np.random.default_rng(1)
        ln = rng.integers(1, 4097, 30000).astype(np.uint64)
        off = np.zeros(ln.size, np.uint64)
        off[1:] = np.cumsum(ln[:-1] + np.uint64(3), dtype=np.uint64)
        return off, ln, 4096
    if kind == "wide":
        off, ln = W.uniform_layout(2000, 70_000, 70_013, 5)
        return off, ln, 70_000
    off, ln = W.cfg3_layout(vlog=True, count=24)
    return off, ln, 0


oracle = load_oracle()
ctx = kvsep.Context(0)
cases = []
big = (0, 0)
for i, k in enumerate(kinds):
    off, ln, hint = layout(k)
    span = int(off[-1] + ln[-1])
    cases.append(dict(kind=k, off=off, ln=ln, hint=hint, span=span, d_off=u64(off), d_len=u64(ln),
                      data=torch.empty(span + 64, dtype=torch.uint8, device=dev),
                      out=torch.zeros(off.size, dtype=torch.int32, device=dev)))
    big = (max(big[0], off.size), max(big[1], int(ln.sum())))
ctx.reserve(*big)
ctx.reserve_captures(len(cases))
for c in cases:
    kvsep.fill_splitmix64(c["data"].data_ptr(), c["span"], 1, 0)
torch.cuda.synchronize()
for c in cases:
    c["g"] = torch.cuda.CUDAGraph()
    with torch.cuda.graph(c["g"]):
        ctx.batch_device(c["data"].data_ptr(), c["d_off"], c["d_len"], c["out"], total_bytes=int(c["ln"].sum()),
                         max_len=c["hint"], stream=torch.cuda.current_stream())
for c in cases:
    c["g"].replay()
    torch.cuda.synchronize()
    ok = np.array_equal(c["out"].cpu().numpy().view(np.uint32), oracle.batch(c["data"].cpu().numpy(), c["off"],
                                                                             c["ln"], threads=8))
    print(f"alone {c['kind']}: {'ok' if ok else 'MISMATCH'}", flush=True)
streams = [torch.cuda.Stream() for _ in range(3)]
bad = 0
for r in range(rounds):
    for c in cases:
        kvsep.fill_splitmix64(c["data"].data_ptr(), c["span"], 1000 + r, 0)
    torch.cuda.synchronize()
    for k, c in enumerate(cases):
        with torch.cuda.stream(streams[k % 3]):
            c["g"].replay()
    torch.cuda.synchronize()
    for c in cases:
        exp = oracle.batch(c["data"].cpu().numpy(), c["off"], c["ln"], threads=8)
        got = c["out"].cpu().numpy().view(np.uint32)
        n = int((got != exp).sum())
        bad += n
        print(f"round {r} {c['kind']}: {n} / {exp.size} mismatches", flush=True)
print("TOTAL mismatches", bad, flush=True)
ctx.close()
