"""The drop-in and the host forms under concurrent callers (SURVEY.md §8b Threading: Extend is called at once by the
writer, compaction, GC and reader threads).  Eight threads call the scalar drop-in with buffers over a lowered offload
threshold -- so they race for the device's GPU leg, and the busy ones divert to the host leg -- while two more threads
run batched host-span calls on one shared context.  ctypes releases the GIL around every library call, so the calls
really overlap.  Every result is checked against the oracle, and the drop-in's counters must show GPU calls and no
GPU failure."""
import ctypes
import threading

import numpy as np
import pytest

import kvsep
from kvsep import splitmix64_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)


def test_concurrent_dropin_and_host_forms(oracle):
    lib = kvsep.lib()
    data = splitmix64_bytes(24 << 20, 4242, 0)
    base = data.ctypes.data
    g0, h0, f0 = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    lib.kvsep_offload_stats(ctypes.byref(g0), ctypes.byref(h0), ctypes.byref(f0))
    lib.kvsep_set_offload_threshold(1 << 20)
    errors = []
    ctx = kvsep.Context(0)

    def dropin(seed):
        rng = np.random.default_rng(seed)
        try:
            for _ in range(6):
                n = int(rng.integers(1 << 20, 6 << 20))
                o = int(rng.integers(0, data.size - n))
                init = int(rng.integers(0, 2**32))
                got = lib.kvsep_crc32c_extend(init, ctypes.c_void_p(base + o), n) & 0xFFFFFFFF
                exp = oracle.extend(init, data[o:o + n].tobytes())
                if got != exp:
                    errors.append(("dropin", seed, o, n))
        except Exception as e:  # pragma: no cover - reported below
            errors.append(("dropin-exc", seed, repr(e)))

    def span(seed):
        rng = np.random.default_rng(seed)
        try:
            for _ in range(4):
                k = 2000
                ln = rng.integers(0, 9000, k).astype(np.uint64)
                off = rng.integers(0, data.size - 9000, k).astype(np.uint64)
                got = ctx.batch_host_span(data, off, ln)
                exp = oracle.batch(data, off, ln, None, threads=2)
                if not np.array_equal(got, exp):
                    errors.append(("span", seed))
        except Exception as e:  # pragma: no cover
            errors.append(("span-exc", seed, repr(e)))

    try:
        threads = [threading.Thread(target=dropin, args=(s,)) for s in range(8)]
        threads += [threading.Thread(target=span, args=(100 + s,)) for s in range(2)]
        for t in threads:
            t.start()
        for t in threads:
            t.join(timeout=300)
        assert not any(t.is_alive() for t in threads), "a caller hung"
    finally:
        lib.kvsep_set_offload_threshold(64 << 20)
        ctx.close()
    assert not errors, errors[:5]
    g1, h1, f1 = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    lib.kvsep_offload_stats(ctypes.byref(g1), ctypes.byref(h1), ctypes.byref(f1))
    assert g1.value > g0.value, "no drop-in call reached the GPU leg"
    assert f1.value == f0.value, "a drop-in GPU call failed"
