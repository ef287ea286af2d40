"""GPU: the batched entry points captured into a HIP graph (torch.cuda.CUDAGraph on ROCm = hipGraph) and
replayed -- planned (split) batches, the narrow kernel and the verify form.  Each replay re-reads the payload,
so rewriting the data between replays must change the results exactly as the oracle says."""
import numpy as np
import pytest

import kvsep
from kvsep import workloads as W

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda:0")


def u64(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(DEV)


def oracle_batch(oracle, data, off, ln):
    return oracle.batch(data.cpu().numpy(), off, ln, threads=8)


@pytest.mark.parametrize("layout", ["planned", "narrow"])
def test_capture_and_replay(layout, oracle):
    if layout == "planned":
        off, ln = W.cfg3_layout(vlog=True, count=96)  # 1,048,609-B records at odd offsets: 9 pieces each
    else:
        off, ln = W.uniform_layout(20000, 4096, 4099, 3)  # 4 KiB blocks at odd offsets (narrow kernel)
    span = int(off[-1] + ln[-1])
    data = torch.empty(span + 64, dtype=torch.uint8, device=DEV)
    d_off, d_len = u64(off), u64(ln)
    out = torch.zeros(off.size, dtype=torch.int32, device=DEV)
    ctx = kvsep.Context(0)
    try:
        ctx.reserve(off.size, int(ln.sum()))
        assert ctx.kernel_name(off.size, int(ln.max())) == (
            "crc32c_pieces_kernel" if layout == "planned" else "crc32c_narrow_kernel")  # 20,000 x 4 KiB: 16 waves
        kvsep.fill_splitmix64(data.data_ptr(), span, 1, 0)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            ctx.batch_device(data.data_ptr(), d_off, d_len, out, total_bytes=int(ln.sum()), max_len=int(ln.max()),
                             stream=torch.cuda.current_stream())
        for seed in (1, 2, 3):
            kvsep.fill_splitmix64(data.data_ptr(), span, seed, 0)
            g.replay()
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy().view(np.uint32), oracle_batch(oracle, data, off, ln)), seed
    finally:
        ctx.close()


@pytest.mark.parametrize("layout", ["planned", "unplanned", "narrow", "sorted", "claim", "claim16", "coop"])
def test_capture_verify_form(layout, oracle):
    """The verify form captured once and replayed: its verdict words are published by the last workgroup of the
    publishing kernel (the CRC kernel; the combine kernel for a split batch), which also resets the context's
    accumulators, so a verdict never leaks into the next replay: clean -> one bad record -> three bad records spread
    over the batch (several workgroups post) -> clean again, each replayed twice, two calls per replay."""
    kernel = {"planned": "auto", "unplanned": "wide", "narrow": "narrow16", "sorted": "sorted", "claim": "claim",
              "claim16": "claim16", "coop": "coop"}[layout]
    if layout == "planned":
        off, ln = W.cfg3_layout(vlog=True, count=40)  # split blocks: the combine kernel publishes
        hint = 0
    elif layout == "unplanned":
        off, ln = W.uniform_layout(3000, 70_000, 70_013, 5)  # unsplit, the wide kernel publishes
        hint = 70_000
    else:
        rng = np.random.default_rng(5)
        ln = rng.integers(1, 4097, 30000).astype(np.uint64)
        off = np.zeros(ln.size, np.uint64)
        off[1:] = np.cumsum(ln[:-1] + np.uint64(7), dtype=np.uint64)
        hint = 4096
    span = int(off[-1] + ln[-1])
    data = torch.empty(span + 64, dtype=torch.uint8, device=DEV)
    kvsep.fill_splitmix64(data.data_ptr(), span, 9, 0)
    exp = oracle_batch(oracle, data, off, ln)
    masked = np.array([kvsep.mask(int(c)) for c in exp], np.uint32)
    d_exp = torch.from_numpy(masked.view(np.int32)).to(DEV)
    out = torch.zeros(off.size, dtype=torch.int32, device=DEV)
    fb = torch.zeros(2, dtype=torch.int64, device=DEV)
    nb = torch.zeros(2, dtype=torch.int64, device=DEV)
    ctx = kvsep.Context(0)
    try:
        ctx.set_kernel(kernel)
        ctx.reserve(off.size, int(ln.sum()))
        d_off, d_len = u64(off), u64(ln)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for k in range(2):  # two verify calls back to back in one graph, each its own verdict words
                ctx.verify_device(data.data_ptr(), d_off, d_len, d_exp, out, fb[k:], nb[k:], total_bytes=int(ln.sum()),
                                  max_len=hint, stream=torch.cuda.current_stream())
        n = off.size
        bad_sets = [[], [17], [3, n // 2, n - 1], []]
        for bad in bad_sets:
            m = masked.copy()
            m[bad] ^= 0x40
            d_exp.copy_(torch.from_numpy(m.view(np.int32)))
            for _ in range(2):
                fb.fill_(123)
                nb.fill_(123)
                g.replay()
                torch.cuda.synchronize()
                want = (min(bad) if bad else -1, len(bad))
                assert [(int(fb[k]), int(nb[k])) for k in range(2)] == [want, want], (layout, bad)
                assert np.array_equal(out.cpu().numpy().view(np.uint32), exp)
        data[int(off[n // 3]) + 1] ^= 1  # a flipped payload byte: the CRC changes, the stored word does not
        d_exp.copy_(torch.from_numpy(masked.view(np.int32)))
        g.replay()
        torch.cuda.synchronize()
        assert (int(fb[0]), int(nb[0])) == (n // 3, 1)
    finally:
        ctx.close()


def test_verify_empty_batch_sets_the_verdict():
    """count == 0: no kernel runs, the verdict words still read "none" (first_bad = -1, nbad = 0)."""
    ctx = kvsep.Context(0)
    try:
        z = torch.zeros(1, dtype=torch.int64, device=DEV)
        fb = torch.full((1,), 7, dtype=torch.int64, device=DEV)
        nb = torch.full((1,), 7, dtype=torch.int64, device=DEV)
        e = torch.zeros(1, dtype=torch.int32, device=DEV)
        ctx.verify_device(e.data_ptr(), z, z, e, e, fb, nb, count=0, total_bytes=0, max_len=0)
        torch.cuda.synchronize()
        assert (fb.item(), nb.item()) == (-1, 0)
    finally:
        ctx.close()
