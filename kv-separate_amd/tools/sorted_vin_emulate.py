#!/usr/bin/env python3
"""Diag: execute the compiled sorted-window kernel variants in the functional ISA emulator (tools/wave_emu.py) on the
batch of tools/sorted_vin_probe.py (n = 70,000, lengths 0..39, correct stored words), one workgroup of the 256-CU grid.

If the emulator -- which runs the instructions exactly as the ISA defines them, every memory op complete before the next
instruction -- reproduces the hardware's wrong CRCs for a variant, the generated code is wrong (a compiler/logic error
one can trace here); if it computes them right while the hardware does not, the fault is in how the hardware executes
that sequence.  CPU only; needs the .s from a --save-temps build of the KVSEP_DIAG device code.
usage: sorted_vin_emulate.py ASM [--variants 20,24,25,28] [--wg 0]"""
import argparse
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", "..", "tests"))
import numpy as np  # noqa: E402

import wave_emu as E  # noqa: E402
from conftest import load_oracle  # noqa: E402  (the checker)
from kvsep import mask, splitmix64_bytes  # noqa: E402

KVIN = {"20": 0, "24": 1, "25": 2, "26": 3, "27": 4, "28": 5, "29": 6}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("asm")
    ap.add_argument("--variants", default="20,24,25,28")
    ap.add_argument("--wg", type=int, default=0)
    ap.add_argument("--grid", type=int, default=256)
    args = ap.parse_args()

    rng = np.random.default_rng(1)
    n, maxlen = 70000, 39
    ln = rng.integers(0, maxlen + 1, n).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
    span = int(off[-1] + ln[-1])
    host = splitmix64_bytes(span + 4096, 5, 0)
    exp = load_oracle().batch(host, off, ln, None, threads=8)
    stored = np.array([mask(int(x)) for x in exp], dtype=np.uint32)
    tabs = E.dev_tables()
    for v in args.variants.split(","):
        ext = "NS_5ExactE" if KVIN[v] == 0 else "NS_9SortedVInILi%dEEE" % KVIN[v]  # the Ext type (crc32c_diag.inc)
        name = "_ZN5kvsep27crc32c_narrow_sorted_kernelILi4ELb1ELi1024ELb0E%sEEvNS_10PiecesArgsE" % ext
        t0 = time.time()
        # the diag variants read expect / first_bad / nbad themselves (kVerify false, kVIn > 0)
        out, written, fb, nb, steps = E.run_batch_kernel(args.asm, name, 1024, host, off, ln, tabs, wg=args.wg,
                                                         grid=args.grid, hint=maxlen, expect=stored)
        touched = np.nonzero(written)[0]
        bad = touched[out[touched] != exp[touched]]
        print(f"variant {v}: {steps} instructions in {time.time() - t0:.1f}s; blocks written {touched.size}, "
              f"wrong {bad.size}{' first ' + str(bad[:8].tolist()) if bad.size else ''}; first_bad {fb}, nbad {nb}",
              flush=True)


if __name__ == "__main__":
    main()
