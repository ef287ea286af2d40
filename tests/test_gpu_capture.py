"""GPU: captured calls replayed at the same time.  Every graph capture runs on a capture set of
its own (csrc/crc32c_device.hip stream_scratch: plan, work counter, SST arrays, verify verdict slots), so

  * nine verify graphs of one context -- the claim, sorted-window, 16-wave narrow and wide kernels, and planned
    (split) batches with the combine kernel -- each with its own planted mismatches, replayed together on three
    streams, round after round, all give their own exact verdict and CRCs, with eager verify calls in between;
  * one verify graph replayed on two streams at once (its replays overlap themselves) still gives the exact verdict:
    a captured call publishes through verdict slots that every replay overwrites whole, never through shared
    arrival counters;
  * a capture that finds every set held fails at capture time with KVSEP_EINVAL instead of sharing one, and
    kvsep_crc32c_release_captures (once those graphs are gone) makes the sets available again.

The contract is the reader's: a mismatch is Corruption and the scan truncates at the first bad record
(/root/reference/db/value_log_reader.cc:109-122), so a verdict mixed from another call is a wrong truncation point."""
import numpy as np
import pytest

import kvsep
from kvsep import workloads as W

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda:0")
NONE = 2**64 - 1


def u64(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(DEV)


def _layout(kind, seed):
    rng = np.random.default_rng(seed)
    if kind == "claim":  # uniform 4 KiB blocks: the claim kernel (form 10)
        off, ln = W.uniform_layout(40000, 4096)
        return off, ln, 4096
    if kind == "sorted":  # ragged short blocks: the sorted-window kernel
        ln = rng.integers(1, 4097, 30000).astype(np.uint64)
        off = np.zeros(ln.size, np.uint64)
        off[1:] = np.cumsum(ln[:-1] + np.uint64(3), dtype=np.uint64)
        return off, ln, 4096
    if kind == "narrow16":  # 20,000 uniform 4 KiB blocks at odd offsets: the 16-wave narrow kernel
        off, ln = W.uniform_layout(20000, 4096, 4099, 3)
        return off, ln, 4096
    if kind == "wide":  # unsplit 70 KB blocks: the wide kernel publishes
        off, ln = W.uniform_layout(2000, 70_000, 70_013, 5)
        return off, ln, 70_000
    off, ln = W.cfg3_layout(vlog=True, count=24)  # 1,048,609-B records: planned, the combine kernel publishes
    return off, ln, 0


KINDS = ["claim", "sorted", "narrow16", "wide", "planned", "claim", "sorted", "wide", "planned"]


def test_overlapping_verify_graphs_are_exact(oracle):
    ctx = kvsep.Context(0)
    try:
        cases = []
        biggest = (0, 0)
        for i, kind in enumerate(KINDS):
            off, ln, hint = _layout(kind, i)
            span = int(off[-1] + ln[-1])
            data = torch.empty(span + 64, dtype=torch.uint8, device=DEV)
            kvsep.fill_splitmix64(data.data_ptr(), span, 100 + i, 0)
            exp = oracle.batch(data.cpu().numpy(), off, ln, threads=8)
            stored = np.array([kvsep.mask(int(c)) for c in exp], np.uint32)
            n = off.size
            bad = sorted({(i * 7919 + 11) % n, (i * 131 + n // 2) % n, n - 1 - i})[: 1 + i % 3]
            stored[bad] ^= np.uint32(0x20)
            cases.append(dict(kind=kind, off=off, ln=ln, hint=hint, data=data, exp=exp, bad=bad,
                              d_off=u64(off), d_len=u64(ln), d_exp=torch.from_numpy(stored.view(np.int32)).to(DEV),
                              out=torch.zeros(n, dtype=torch.int32, device=DEV),
                              fb=torch.zeros(1, dtype=torch.int64, device=DEV),
                              nb=torch.zeros(1, dtype=torch.int64, device=DEV)))
            biggest = (max(biggest[0], n), max(biggest[1], int(ln.sum())))
        ctx.reserve(*biggest)
        ctx.reserve_captures(len(cases) + 1)
        torch.cuda.synchronize()
        for c in cases:
            c["g"] = torch.cuda.CUDAGraph()
            with torch.cuda.graph(c["g"]):
                ctx.verify_device(c["data"].data_ptr(), c["d_off"], c["d_len"], c["d_exp"], c["out"], c["fb"], c["nb"],
                                  total_bytes=int(c["ln"].sum()), max_len=c["hint"],
                                  stream=torch.cuda.current_stream())
        assert ctx.capture_sets() == (len(cases) + 1, len(cases))  # one set per graph
        for c in cases:  # each graph alone first
            c["g"].replay()
            torch.cuda.synchronize()
            got = (int(c["fb"].item()) & NONE, int(c["nb"].item()))
            assert got == (min(c["bad"]), len(c["bad"])), ("alone", c["kind"], got, c["bad"])
            assert np.array_equal(c["out"].cpu().numpy().view(np.uint32), c["exp"]), ("alone", c["kind"])
        streams = [torch.cuda.Stream() for _ in range(3)]
        for rnd in range(4):
            for c in cases:
                c["fb"].fill_(7)
                c["nb"].fill_(7)
            torch.cuda.synchronize()
            for k, c in enumerate(cases):  # all nine in flight together, three per stream
                with torch.cuda.stream(streams[k % 3]):
                    c["g"].replay()
            if rnd % 2:  # an eager verify call of the same context among them (the context's own scratch)
                c0 = cases[0]
                ofb = torch.zeros(1, dtype=torch.int64, device=DEV)
                onb = torch.zeros(1, dtype=torch.int64, device=DEV)
                oout = torch.zeros(c0["off"].size, dtype=torch.int32, device=DEV)
                ctx.verify_device(c0["data"].data_ptr(), c0["d_off"], c0["d_len"], c0["d_exp"], oout, ofb, onb,
                                  total_bytes=int(c0["ln"].sum()), max_len=c0["hint"])
            torch.cuda.synchronize()
            for c in cases:
                got = (int(c["fb"].item()) & NONE, int(c["nb"].item()))
                assert got == (min(c["bad"]), len(c["bad"])), (rnd, c["kind"], got, c["bad"])
                assert np.array_equal(c["out"].cpu().numpy().view(np.uint32), c["exp"]), (rnd, c["kind"])
            if rnd % 2:
                assert (int(ofb.item()), int(onb.item())) == (min(cases[0]["bad"]), len(cases[0]["bad"]))
    finally:
        ctx.close()


@pytest.mark.parametrize("kind", ["claim", "sorted", "wide"])
def test_one_verify_graph_replayed_over_itself(kind, oracle):
    """One captured verify graph launched on two streams back to back, so its replays may overlap (and a second
    instantiation of the same capture on a third): the verdict slots of its capture set are written whole by each
    replay with the same words, so every verdict is exact."""
    off, ln, hint = _layout(kind, 42)
    span = int(off[-1] + ln[-1])
    data = torch.empty(span + 64, dtype=torch.uint8, device=DEV)
    kvsep.fill_splitmix64(data.data_ptr(), span, 77, 0)
    exp = oracle.batch(data.cpu().numpy(), off, ln, threads=8)
    stored = np.array([kvsep.mask(int(c)) for c in exp], np.uint32)
    n = off.size
    bad = [5, n // 3, n - 2]
    stored[bad] ^= np.uint32(0x1)
    d_off, d_len = u64(off), u64(ln)
    d_exp = torch.from_numpy(stored.view(np.int32)).to(DEV)
    out = torch.zeros(n, dtype=torch.int32, device=DEV)
    fb = torch.zeros(1, dtype=torch.int64, device=DEV)
    nb = torch.zeros(1, dtype=torch.int64, device=DEV)
    ctx = kvsep.Context(0)
    try:
        ctx.reserve(n, int(ln.sum()))
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            ctx.verify_device(data.data_ptr(), d_off, d_len, d_exp, out, fb, nb, total_bytes=int(ln.sum()),
                              max_len=hint, stream=torch.cuda.current_stream())
        g.replay()  # a first launch alone (see test_overlapping_verify_graphs_are_exact)
        torch.cuda.synchronize()
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        for _ in range(6):
            fb.fill_(9)
            nb.fill_(9)
            torch.cuda.synchronize()
            with torch.cuda.stream(s1):
                g.replay()
            with torch.cuda.stream(s2):
                g.replay()
            with torch.cuda.stream(s1):
                g.replay()
            torch.cuda.synchronize()
            assert (int(fb.item()), int(nb.item())) == (5, 3)
            assert np.array_equal(out.cpu().numpy().view(np.uint32), exp)
    finally:
        ctx.close()


def test_capture_sets_run_out_at_capture_time_and_come_back():
    off, ln = W.uniform_layout(40000, 4096)
    n, tb = off.size, int(ln.sum())
    data = torch.zeros(tb + 64, dtype=torch.uint8, device=DEV)
    d_off, d_len = u64(off), u64(ln)
    outs = [torch.zeros(n, dtype=torch.int32, device=DEV) for _ in range(5)]
    ctx = kvsep.Context(0)
    try:
        with pytest.raises(kvsep.KvsepError, match="reserve"):  # no reservation, no capture set
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                ctx.batch_device(data.data_ptr(), d_off, d_len, outs[0], max_len=4096, total_bytes=tb,
                                 stream=torch.cuda.current_stream())
        del g
        ctx.reserve(n, int(ln.sum()))
        assert ctx.capture_sets() == (4, 0)  # the default
        graphs = []
        for k in range(4):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                ctx.batch_device(data.data_ptr(), d_off, d_len, outs[k], max_len=4096, total_bytes=tb,
                                 stream=torch.cuda.current_stream())
            graphs.append(g)
        assert ctx.capture_sets() == (4, 4)
        with pytest.raises(kvsep.KvsepError, match="every capture set"):
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                ctx.batch_device(data.data_ptr(), d_off, d_len, outs[4], max_len=4096, total_bytes=tb,
                                 stream=torch.cuda.current_stream())
        del g
        for g in graphs:
            g.replay()
        torch.cuda.synchronize()
        want = kvsep.extend_host(0, bytes(4096))
        assert all(int(o[0].item()) & 0xffffffff == want for o in outs[:4])
        del graphs
        torch.cuda.synchronize()
        ctx.release_captures()
        assert ctx.capture_sets() == (4, 0)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            ctx.batch_device(data.data_ptr(), d_off, d_len, outs[4], max_len=4096, total_bytes=tb,
                             stream=torch.cuda.current_stream())
        g.replay()
        torch.cuda.synchronize()
        assert int(outs[4][n - 1].item()) & 0xffffffff == want
        assert ctx.capture_sets() == (4, 1)
    finally:
        ctx.close()


def test_fault_injection_needs_the_test_environment(monkeypatch):
    """the test-only hook is inert in a process without KVSEP_TEST_HOOKS=1."""
    ctx = kvsep.Context(0)
    try:
        monkeypatch.delenv("KVSEP_TEST_HOOKS", raising=False)
        with pytest.raises(kvsep.KvsepError, match="KVSEP_TEST_HOOKS"):
            ctx.inject_failure()
    finally:
        ctx.close()
