#!/usr/bin/env python3
"""Run pytest with the kvsep binding pointed at the KVSEP_DIAG tools build (tools/libkvsep_diag.so): its kernels carry
the diagnosis checks of the shipped ones (printf instead of a wild access).  usage: run_with_diag.py <pytest args>"""
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, HERE)
import _diag  # noqa: E402,F401  (kvsep.LIB_PATH -> the diag build)
import pytest  # noqa: E402

sys.exit(pytest.main(sys.argv[1:]))
