"""The three host legs of Extend (kv-separate_amd/csrc/host_crc.cpp) against the oracle: the
VPCLMULQDQ fold, the SSE4.2 crc32 loop and the portable table-driven leg that any CPU runs, so Extend is total on any
host as util/crc32c.cc's portable path is (/root/reference/util/crc32c.cc:276-377, gated by port/port_stdcxx.h:142-152).

  * every length 0..1023 at every offset 0..15, init 0 and a random init, plus the reference's large-block goldens, on
    each leg (KVSEP_HOST_CRC forces the slower legs, in a child process each: the leg is chosen once per process);
  * the leg the library reports (kvsep_crc32c_host_path) is the one the CPU supports, so a fold sweep cannot pass on
    the crc32 path without saying so;
  * host_crc.cpp built alone with KVSEP_HOST_NO_X86 -- the form a non-x86 host compiles -- contains no x86 CRC
    instruction and is exact.  No GPU."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import kvsep

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "kv-separate_amd", "csrc")

SWEEP = r"""
import json, os, sys
import numpy as np
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
from conftest import load_oracle  # the checker
import kvsep
from kvsep import splitmix64_bytes
oracle = load_oracle()
f = kvsep.lib().kvsep_crc32c_extend_host
data = splitmix64_bytes(1024 + 64, 2024, 0)
rng = np.random.default_rng(5)
bad = []
for o in range(16):
    for n in range(1024):
        for init in (0, int(rng.integers(0, 2**32))):
            if f(init, data.ctypes.data + o, n) != oracle.extend_addr(init, data.ctypes.data + o, n):
                bad.append((o, n, init))
print(json.dumps({"path": kvsep.host_path(), "bad": bad[:10], "nbad": len(bad)}))
"""


def _cpu_flags():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("flags"):
                return set(line.split(":", 1)[1].split())
    except OSError:
        pass
    return set()


def _run(leg):
    env = dict(os.environ)
    env.pop("KVSEP_HOST_CRC", None)
    if leg:
        env["KVSEP_HOST_CRC"] = leg
    r = subprocess.run([sys.executable, "-c", SWEEP, ROOT], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("leg", [None, "sse42", "portable"])
def test_every_length_and_offset_on_each_leg(leg):
    out = _run(leg)
    assert out["nbad"] == 0, out
    flags = _cpu_flags()
    best = ("fold" if {"avx512f", "vpclmulqdq", "pclmulqdq", "sse4_2"} <= flags else
            "sse42" if "sse4_2" in flags else "portable")
    expect = {None: best, "sse42": "sse42" if best != "portable" else "portable", "portable": "portable"}[leg]
    assert out["path"] == expect, (out, best)


def test_large_blocks_on_the_portable_leg():
    """The reference's 4 KiB ... 4 MiB + 1 goldens (tests/golden, computed by the compiled util/crc32c.cc) on the
    portable leg, where the 8-byte table loop carries nearly every byte."""
    from kvsep import workloads as W
    body = r"""
import json, os, sys
sys.path.insert(0, os.path.join(sys.argv[1], "tests"))
from conftest import GOLDEN
import kvsep
from kvsep import splitmix64_bytes
from kvsep import workloads as W
g = json.load(open(GOLDEN))
data = splitmix64_bytes((4 << 20) + 64, W.SEED + 1, 0)
f = kvsep.lib().kvsep_crc32c_extend_host
bad = [c for c in g["large"] if f(c["init"], data.ctypes.data + c["offset"], c["len"]) != c["crc"]]
print(json.dumps({"path": kvsep.host_path(), "n": len(g["large"]), "bad": len(bad)}))
"""
    env = dict(os.environ, KVSEP_HOST_CRC="portable")
    r = subprocess.run([sys.executable, "-c", body, ROOT], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert out["path"] == "portable" and out["n"] >= 10 and out["bad"] == 0, out


def test_portable_only_build_has_no_x86_crc_and_is_exact(tmp_path, oracle):
    so = tmp_path / "libhostcrc_portable.so"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-shared", "-fPIC", "-DKVSEP_HOST_NO_X86", "-I", CSRC,
                           "-o", str(so), os.path.join(CSRC, "host_crc.cpp"),
                           os.path.join(ROOT, "tests", "cpp", "host_crc_only.cc")])
    dis = subprocess.run(["objdump", "-d", str(so)], capture_output=True, text=True).stdout
    assert "crc32" not in dis and "pclmul" not in dis, "x86 CRC instructions in the portable-only build"
    import ctypes
    l = ctypes.CDLL(str(so))
    l.hc_extend.restype = ctypes.c_uint32
    l.hc_extend.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
    l.hc_path.restype = ctypes.c_char_p
    assert l.hc_path() == b"portable"
    data = kvsep.splitmix64_bytes(70000, 31, 0)
    rng = np.random.default_rng(9)
    for o in range(16):
        for n in list(range(0, 300)) + [1023, 4096, 4097, 65536, 69000]:
            init = int(rng.integers(0, 2**32))
            assert l.hc_extend(init, data.ctypes.data + o, n) == oracle.extend_addr(init, data.ctypes.data + o, n)
    assert l.hc_extend(0, b"123456789", 9) == 0xE3069283  # util/crc32c_test.cc / RFC 3720 check value
