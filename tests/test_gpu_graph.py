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
            "crc32c_pieces_kernel" if layout == "planned" else "crc32c_narrow_kernel")
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


def test_capture_verify_form(oracle):
    off, ln = W.cfg3_layout(vlog=True, count=40)
    span = int(off[-1] + ln[-1])
    data = torch.empty(span + 64, dtype=torch.uint8, device=DEV)
    kvsep.fill_splitmix64(data.data_ptr(), span, 9, 0)
    exp = oracle_batch(oracle, data, off, ln)
    masked = np.array([kvsep.mask(int(c)) for c in exp], np.uint32)
    d_exp = torch.from_numpy(masked.view(np.int32)).to(DEV)
    out = torch.zeros(off.size, dtype=torch.int32, device=DEV)
    fb = torch.zeros(1, dtype=torch.int64, device=DEV)
    nb = torch.zeros(1, dtype=torch.int64, device=DEV)
    ctx = kvsep.Context(0)
    try:
        ctx.reserve(off.size, int(ln.sum()))
        d_off, d_len = u64(off), u64(ln)
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            ctx.verify_device(data.data_ptr(), d_off, d_len, d_exp, out, fb, nb, total_bytes=int(ln.sum()),
                              max_len=int(ln.max()), stream=torch.cuda.current_stream())
        g.replay()
        torch.cuda.synchronize()
        assert (fb.item(), nb.item()) == (-1, 0)
        data[int(off[17]) + 5] ^= 1  # one flipped bit in record 17
        g.replay()
        torch.cuda.synchronize()
        assert (fb.item(), nb.item()) == (17, 1)
    finally:
        ctx.close()
