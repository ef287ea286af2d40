"""Shared test plumbing.  `-m gpu` tests need a real gfx950 device; everything else runs on CPU."""
import ctypes
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
# arms the library's test-only hooks (csrc/kvsep_testing.h: fault injection); the shipped library ignores them otherwise
os.environ.setdefault("KVSEP_TEST_HOOKS", "1")
sys.path.insert(0, os.path.join(ROOT, "kv-separate_amd"))
sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden", "crc32c_golden.json")
ORACLE_SO = os.path.join(ROOT, "oracle", "_build", "liboracle_crc32c.so")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device")
    config.addinivalue_line("markers", "slow: long-running")


@pytest.fixture(scope="session")
def golden():
    with open(GOLDEN) as f:
        return json.load(f)


class Oracle:
    """ctypes view of oracle/crc32c_oracle.c -- the CHECKER, never the product."""

    def __init__(self, path):
        l = ctypes.CDLL(path)
        l.oracle_crc32c_extend.restype = ctypes.c_uint32
        l.oracle_crc32c_extend.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
        l.oracle_crc32c_mask.restype = ctypes.c_uint32
        l.oracle_crc32c_mask.argtypes = [ctypes.c_uint32]
        l.oracle_crc32c_unmask.restype = ctypes.c_uint32
        l.oracle_crc32c_unmask.argtypes = [ctypes.c_uint32]
        l.oracle_fill_splitmix64.restype = None
        l.oracle_fill_splitmix64.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64]
        l.oracle_crc32c_batch.restype = ctypes.c_int
        l.oracle_crc32c_batch.argtypes = [ctypes.c_void_p] * 5 + [ctypes.c_size_t, ctypes.c_int]
        self.lib = l

    def extend_addr(self, init, addr, n):
        return int(self.lib.oracle_crc32c_extend(init & 0xFFFFFFFF, addr, n))

    def extend(self, init, data):
        import numpy as np
        a = np.frombuffer(bytes(data), dtype=np.uint8).copy() if len(data) else np.zeros(1, np.uint8)
        return self.extend_addr(init, a.ctypes.data, len(data))

    def batch(self, buf, off, length, init=None, threads=1):
        import numpy as np
        off = np.ascontiguousarray(off, dtype=np.uint64)
        length = np.ascontiguousarray(length, dtype=np.uint64)
        out = np.zeros(off.size, dtype=np.uint32)
        ip = None
        if init is not None:
            init = np.ascontiguousarray(init, dtype=np.uint32)
            ip = init.ctypes.data
        rc = self.lib.oracle_crc32c_batch(buf.ctypes.data, off.ctypes.data, length.ctypes.data, ip,
                                          out.ctypes.data, off.size, threads)
        assert rc == 0
        return out


def load_oracle():
    if not os.path.exists(ORACLE_SO):
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle"), "oracle"])
    return Oracle(ORACLE_SO)


@pytest.fixture(scope="session")
def oracle():
    return load_oracle()


def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
