"""GPU parity at BASELINE.json's full sizes (configs 3a, 3b, 4 on one MI355X): 64 GiB / 64 GiB / 149.7 GiB.

The oracle cannot recompute a whole batch in test time, so each batch is checked through properties that do
not depend on its size, plus a sample:
  * piece-size invariance: the same batch through 128 KiB pieces (planned, guided schedule), 1 MiB pieces
    and whole blocks (unplanned, static schedule) -- three different work decompositions and combine paths
    -- gives identical results;
  * verify-mode consistency: expected = Mask(results) gives nbad = 0; flipping one stored word gives
    exactly that block as first_bad;
  * 48 blocks spread over the batch, copied to the host, recomputed by the oracle (bit-exact).
"""
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


@pytest.mark.parametrize("cfg", ["3a", "3b", "4"])
def test_full_size_batch(cfg, oracle):
    off, ln = {"3a": W.cfg3_layout, "3b": lambda: W.cfg3_layout(vlog=True), "4": W.cfg4_layout}[cfg]()
    span = int(off[-1] + ln[-1])
    total, max_len = int(ln.sum()), int(ln.max())
    data = torch.empty(span + 64, dtype=torch.uint8, device=DEV)
    kvsep.fill_splitmix64(data.data_ptr(), span, W.SEED + 1, 0)
    d_off, d_len = u64(off), u64(ln)
    ctx = kvsep.Context(0)
    try:
        outs = []
        for piece, hint in ((128 * 1024, max_len), (1 << 20, max_len), (8 << 20, max_len)):
            ctx.set_piece_bytes(piece)
            ctx.reserve(off.size, total)
            o = torch.zeros(off.size, dtype=torch.int32, device=DEV)
            ctx.batch_device(data.data_ptr(), d_off, d_len, o, total_bytes=total, max_len=hint)
            torch.cuda.synchronize()
            outs.append(o)
        for o in outs[1:]:
            assert torch.equal(o, outs[0]), "piece-size decompositions disagree"
        crcs = outs[0].cpu().numpy().view(np.uint32)

        # verify mode over the whole batch
        exp = np.array([kvsep.mask(int(c)) for c in crcs], dtype=np.uint32)
        bad_at = off.size // 3
        exp[bad_at] ^= 0x10
        d_exp = torch.from_numpy(exp.view(np.int32)).to(DEV)
        o = torch.zeros(off.size, dtype=torch.int32, device=DEV)
        fb = torch.zeros(1, dtype=torch.int64, device=DEV)
        nb = torch.zeros(1, dtype=torch.int64, device=DEV)
        ctx.verify_device(data.data_ptr(), d_off, d_len, d_exp, o, fb, nb, total_bytes=total, max_len=max_len)
        torch.cuda.synchronize()
        assert (fb.item(), nb.item()) == (bad_at, 1)
        assert torch.equal(o, outs[0])

        # sampled blocks vs the oracle
        idx = np.unique(np.linspace(0, off.size - 1, 48).astype(np.int64))
        for i in idx:
            h = data[int(off[i]):int(off[i] + ln[i])].cpu().numpy()
            assert int(crcs[i]) == oracle.extend_addr(0, h.ctypes.data, h.size), (cfg, int(i))
    finally:
        ctx.close()
        del data
        torch.cuda.empty_cache()
