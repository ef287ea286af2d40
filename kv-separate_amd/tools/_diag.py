"""Point the kvsep binding at the KVSEP_DIAG tools build (tools/libkvsep_diag.so, `make -C kv-separate_amd diag`).

That build carries the A/B and ablation kernel variants (selected by KVSEP_CRC_VARIANT / KVSEP_NARROW /
KVSEP_CRC_STATIC_RR; the ablation variants give wrong results by design).  The shipped library has none of them and
reads none of those variables.  Import this module before the first kvsep call of a diagnostic tool."""
import os
import subprocess

import kvsep

DIAG = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libkvsep_diag.so")


def use_diag_lib():
    if not os.path.exists(DIAG):
        subprocess.check_call(["make", "-s", "-C", os.path.join(os.path.dirname(DIAG), ".."), "diag"])
    kvsep.LIB_PATH, kvsep._lib = DIAG, None
    return kvsep.lib()


use_diag_lib()
