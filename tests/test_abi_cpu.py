"""The C-ABI library loads and exports every symbol include/kvsep_crc32c.h declares, and its
host-only legs (SSE4.2 Extend below the offload threshold, Mask/Unmask) are bit-exact.  No GPU."""
import ctypes
import os

import numpy as np
import pytest

import kvsep
from kvsep import splitmix64_bytes
from kvsep import workloads as W


def test_library_exports_every_header_symbol():
    names = kvsep.header_functions()
    assert len(names) >= 20
    l = ctypes.CDLL(kvsep.LIB_PATH)
    missing = [n for n in names if not hasattr(l, n)]
    assert not missing, missing


SHIM = os.path.join(os.path.dirname(kvsep.LIB_PATH), "libkvsep_leveldb_abi.so")


def test_exports_leveldb_extend_cpp_symbol():
    """The link-level boundary: leveldb::crc32c::Extend(uint32_t, const char*, size_t) with C++ linkage
    (util/crc32c.h:17), so a KVDB build keeps its own util/crc32c.h and only swaps util/crc32c.cc for the shim
    libkvsep_leveldb_abi.so (over the engine library)."""
    l = ctypes.CDLL(SHIM)
    f = getattr(l, "_ZN7leveldb6crc32c6ExtendEjPKcm")
    f.restype = ctypes.c_uint32
    f.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_size_t]
    assert f(0, b"123456789", 9) == 0xE3069283
    assert f(0, b"TestCRCBuffer", 13) == 0xDCBC59FA  # util/crc32c.cc:267-274 self-test
    assert f(0x12345678, None, 0) == 0x12345678


def test_engine_library_does_not_export_the_leveldb_symbol():
    """loading the engine (e.g. RTLD_GLOBAL next to a real LevelDB) must not interpose that LevelDB's
    leveldb::crc32c::Extend -- the C++ symbol lives only in the drop-in shim."""
    import subprocess
    syms = subprocess.run(["nm", "-D", "--defined-only", kvsep.LIB_PATH], capture_output=True, text=True).stdout
    assert "_ZN7leveldb6crc32c6ExtendEjPKcm" not in syms
    shim = subprocess.run(["nm", "-D", "--defined-only", SHIM], capture_output=True, text=True).stdout
    assert "_ZN7leveldb6crc32c6ExtendEjPKcm" in shim


def test_abi_version():
    assert kvsep.lib().kvsep_abi_version() == 4
    assert "ABI 4" in kvsep.build_info()


def test_no_environment_variable_reaches_the_kernel_choice():
    """The shipped library reads no variant / kernel-routing variable (those exist only in the KVSEP_DIAG tools
    build): only KVSEP_STRICT_GPU, KVSEP_COPY_THREADS, KVSEP_HOST_CRC (=sse42 / =portable: a slower host leg, for
    A/B), KVSEP_SYSFS_ROOT (where the topology is read: tests fake it) and KVSEP_TEST_HOOKS (=1 arms the test-only
    fault injection of csrc/kvsep_testing.h), none of which can change a CRC."""
    import re
    strings = open(kvsep.LIB_PATH, "rb").read()
    names = set(re.findall(rb"KVSEP_[A-Z_]{3,}", strings))
    assert names <= {b"KVSEP_STRICT_GPU", b"KVSEP_COPY_THREADS", b"KVSEP_HOST_CRC", b"KVSEP_SYSFS_ROOT",
                     b"KVSEP_TEST_HOOKS"}, names


def test_fault_injection_is_not_public_and_needs_the_test_environment():
    """the fault-injection hook is not in the public header, and the library refuses it without
    KVSEP_TEST_HOOKS=1 (checked before any device is touched: a null context is refused either way)."""
    assert "kvsep_crc32c_ctx_inject_failure" not in kvsep.header_functions()
    assert kvsep.lib().kvsep_crc32c_ctx_inject_failure(None) == -1


def test_python_extend_rejects_n_past_buffer():
    with pytest.raises(ValueError):
        kvsep.extend(0, b"abc", 4)
    with pytest.raises(ValueError):
        kvsep.extend_host(0, b"abc", 5)
    assert kvsep.extend(0, b"abc", 3) == kvsep.value(b"abc")


def test_binding_covers_header():
    assert set(kvsep.header_functions()) <= set(kvsep._SIGS), set(kvsep.header_functions()) - set(kvsep._SIGS)


def test_build_info():
    assert "gfx950" in kvsep.build_info()


def test_host_extend_golden_sweep(golden):
    sw = golden["sweep"]
    data = splitmix64_bytes(4096, sw["seed"], 0)
    raw = np.zeros(4096 + 128, np.uint8)
    b = (-raw.ctypes.data) % 64
    raw[b:b + 4096] = data
    base = raw.ctypes.data + b
    f = kvsep.lib().kvsep_crc32c_extend_host
    for o in range(16):
        for n in range(257):
            assert f(0, base + o, n) == sw["crc_init0"][o][n]
            assert f(sw["init"][o][n], base + o, n) == sw["crc_init"][o][n]


def test_host_extend_large(golden):
    data = splitmix64_bytes((4 << 20) + 64, W.SEED + 1, 0)
    f = kvsep.lib().kvsep_crc32c_extend_host
    for c in golden["large"]:
        assert f(c["init"], data.ctypes.data + c["offset"], c["len"]) == c["crc"], c


def test_dropin_extend_below_threshold(golden):
    # crc32c_test.cc semantics through the drop-in entry points (no offload at these sizes)
    assert kvsep.value(bytes(32)) == 0x8A9136AA
    assert kvsep.value(b"hello world") == kvsep.extend(kvsep.value(b"hello "), b"world")
    assert kvsep.lib().kvsep_accelerated_crc32c(0, b"TestCRCBuffer", 13) == 0xDCBC59FA
    assert kvsep.extend(0x12345678, b"", 0) == 0x12345678
    assert kvsep.lib().kvsep_crc32c_extend(0x12345678, None, 0) == 0x12345678
    for k in golden["known"]:
        d = bytes.fromhex(k["hex"]) if k["hex"] is not None else bytes([k["fill"]["byte"]]) * k["fill"]["n"]
        assert kvsep.value(d) == k["value"], k["name"]


def test_mask_unmask(golden):
    for m in golden["mask"]:
        assert kvsep.mask(m["crc"]) == m["masked"]
        assert kvsep.unmask(m["crc"]) == m["unmask_of_crc"]
        assert kvsep.unmask(kvsep.mask(m["crc"])) == m["crc"]


def test_ctx_without_gpu_fails_loudly():
    from conftest import gpu_available
    if gpu_available():
        pytest.skip("GPU present")
    with pytest.raises(kvsep.KvsepError):
        kvsep.Context(0)


def test_partition_byte_balanced():
    """kvsep_crc32c_partition: contiguous, monotone, covers every block, each part within one
    block of its byte share; degenerate inputs."""
    from kvsep import workloads as W

    for count, parts in ((1 << 20, 8), (1000, 3), (5, 8), (1, 1), (0, 4)):
        ln = W.zipf_lengths(count) if count else np.zeros(0, np.uint64)
        b = kvsep.partition(ln, parts)
        assert b[0] == 0 and b[-1] == count and np.all(np.diff(b.astype(np.int64)) >= 0)
        if count:
            pre = np.concatenate([[0], np.cumsum(ln, dtype=np.uint64)])
            share = pre[-1] / parts
            for p in range(parts):
                got = int(pre[b[p + 1]] - pre[b[p]])
                assert abs(got - share) <= int(ln.max()), (count, parts, p, got, share)
    b = kvsep.partition(np.array([10, 0, 0, 10], np.uint64), 2)
    assert b.tolist() in ([0, 1, 4], [0, 2, 4], [0, 3, 4])


def test_host_extend_lane_boundaries(oracle):
    """The host leg's 3-way loop runs lanes of 4 KiB, 1 KiB and 256 B (crc32c_host.cpp host_crc): every length around
    3 L for each L, and a sweep to 13 KB, at eight start offsets and two inits, against the oracle."""
    data = splitmix64_bytes(60000, 77, 0)
    lens = set(range(0, 13000, 37))
    for L in (256, 1024, 4096):
        for k in (1, 2, 3, 4):
            lens.update(range(3 * L * k - 9, 3 * L * k + 10))
    f = kvsep.lib().kvsep_crc32c_extend_host
    for o in range(8):
        for n in sorted(lens):
            for init in (0, 0x9E3779B9):
                b = data[o:o + n].tobytes()
                assert f(init, data.ctypes.data + o, n) == oracle.extend(init, b), (o, n, init)


def test_host_extend_fold_boundaries(oracle):
    """The host leg's VPCLMULQDQ fold (crc32c_host.cpp fold_bulk, from 128 B) takes whole 256-B rounds, then the
    remainder's 64-B and 16-B chunks, and leaves < 16 B to the crc32 loop: every length around 256 k for k = 1..9 at
    64 start offsets (the zmm loads' alignments), and every length 0..1023 (both entries, every remainder) at 8
    offsets, three inits each,
    against the oracle.  On a CPU without AVX-512 VPCLMULQDQ the fold cannot run: the test then says which leg it
    checked instead of passing silently on it."""
    flags = set()
    for line in open("/proc/cpuinfo"):
        if line.startswith("flags"):
            flags = set(line.split(":", 1)[1].split())
            break
    leg = kvsep.host_path()
    if {"avx512f", "vpclmulqdq", "pclmulqdq", "sse4_2"} <= flags and os.environ.get("KVSEP_HOST_CRC") is None:
        assert leg == "fold", leg
    elif os.environ.get("KVSEP_HOST_CRC") is None:
        pytest.skip(f"no AVX-512 VPCLMULQDQ on this CPU: the fold leg cannot run (host leg here: {leg})")
    data = splitmix64_bytes(8192, 91, 0)
    f = kvsep.lib().kvsep_crc32c_extend_host
    lens = sorted({n for k in range(1, 10) for n in range(256 * k - 5, 256 * k + 21)} | {4096, 4097, 4095})
    cases = [(o, n) for o in range(64) for n in lens] + [(o, n) for o in range(0, 64, 9) for n in range(0, 1024)]
    for o, n in cases:
        b = data[o:o + n].tobytes()
        for init in (0, 0xFFFFFFFF, 0x9E3779B9 ^ o):
            assert f(init, data.ctypes.data + o, n) == oracle.extend(init, b), (o, n, init)


def test_host_extend_both_paths_in_subprocess():
    """KVSEP_HOST_CRC=sse42 keeps the crc32 3-way loop (the path of CPUs without AVX-512 VPCLMULQDQ): run the lane
    boundary and fold boundary sweeps in a child process with it set, so that path stays covered on this machine."""
    import os
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    env = dict(os.environ, KVSEP_HOST_CRC="sse42")
    r = subprocess.run([sys.executable, "-m", "pytest", "-q", "-x", "-p", "no:cacheprovider",
                        os.path.join(here, "test_abi_cpu.py") + "::test_host_extend_lane_boundaries",
                        os.path.join(here, "test_abi_cpu.py") + "::test_host_extend_fold_boundaries",
                        os.path.join(here, "test_abi_cpu.py") + "::test_host_extend_large"],
                       env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-2000:]
    assert "3 passed" in r.stdout, r.stdout[-2000:]
