"""The C-ABI library loads and exports every symbol include/kvsep_crc32c.h declares, and its
host-only legs (SSE4.2 Extend below the offload threshold, Mask/Unmask) are bit-exact.  No GPU."""
import ctypes

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
