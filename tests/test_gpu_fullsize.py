"""GPU parity at BASELINE.json's full sizes, EVERY block against the reference (util/crc32c.cc compiled into
oracle/_ref and run over the same synthetic streams by tests/golden/make_fullsize_golden.py):

  config 2   65,536 x 4 KiB                                   256 MiB   tests/golden/full_cfg2.u32 (rank 0's part)
  config 3a  65,536 x 1 MiB                                   64 GiB    tests/golden/full_cfg3a.u32 (rank 0's part)
  config 3b  65,536 x 1,048,609-B vlog records, odd offsets   64 GiB    slice 0 of full_cfg5.u32
  config 4   1,048,576 Zipf blocks, 32 B - 4 MiB              149.7 GiB tests/golden/full_cfg4.u32
  config 5   the 512 GiB vlog (524,288 records) as 8 distinct 64 GiB slices, each regenerated in HBM at its true
             stream offset and checked block by block                    full_cfg5.u32

Seeds and stream offsets are bench.py's.  On top of the reference check, each batch runs through three work
decompositions (128 KiB pieces planned + guided, 1 MiB pieces, 8 MiB = whole blocks) that must agree, and the verify
mode (fused Mask + compare against the stored words) must report exactly the one flipped word.
"""
import os

import numpy as np
import pytest

import kvsep
from kvsep import workloads as W

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda:0")
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def golden(name):
    return np.fromfile(os.path.join(GOLDEN, name), dtype="<u4")


def u64(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(DEV)


CONFIGS = {  # layout, seed, reference per-block CRCs
    "2": (W.cfg2_layout, W.SEED, lambda: golden("full_cfg2.u32")[:W.CFG2_BLOCKS]),  # rank 0 of the 8-rank files
    "3a": (W.cfg3_layout, W.SEED + 1, lambda: golden("full_cfg3a.u32")[:W.CFG3_BLOCKS]),
    "3b": (lambda: W.cfg3_layout(vlog=True), W.SEED + 1, lambda: golden("full_cfg5.u32")[:W.CFG3_BLOCKS]),
    "4": (W.cfg4_layout, W.SEED + 2, lambda: golden("full_cfg4.u32")),
}


@pytest.mark.parametrize("cfg", ["2", "3a", "3b", "4"])
def test_full_size_batch_every_block_vs_reference(cfg):
    layout, seed, ref = CONFIGS[cfg]
    off, ln = layout()
    span = int(off[-1] + ln[-1])
    total, max_len = int(ln.sum()), int(ln.max())
    exp_all = ref()
    assert exp_all.size == off.size
    data = torch.empty(span + 64, dtype=torch.uint8, device=DEV)
    kvsep.fill_splitmix64(data.data_ptr(), span, seed, 0)
    d_off, d_len = u64(off), u64(ln)
    ctx = kvsep.Context(0)
    try:
        outs = []
        for piece in (128 * 1024, 1 << 20, 8 << 20):
            ctx.set_piece_bytes(piece)
            ctx.reserve(off.size, total)
            o = torch.zeros(off.size, dtype=torch.int32, device=DEV)
            ctx.batch_device(data.data_ptr(), d_off, d_len, o, total_bytes=total, max_len=max_len)
            torch.cuda.synchronize()
            outs.append(o)
        crcs = outs[0].cpu().numpy().view(np.uint32)
        bad = np.flatnonzero(crcs != exp_all)
        assert bad.size == 0, (cfg, bad[:8])
        for o in outs[1:]:
            assert torch.equal(o, outs[0]), "work decompositions disagree"

        # verify mode over the whole batch: the reference's stored words, one flipped
        exp = np.array([kvsep.mask(int(c)) for c in exp_all], dtype=np.uint32)
        bad_at = off.size // 3
        exp[bad_at] ^= 0x10
        o = torch.zeros(off.size, dtype=torch.int32, device=DEV)
        fb = torch.zeros(1, dtype=torch.int64, device=DEV)
        nb = torch.zeros(1, dtype=torch.int64, device=DEV)
        ctx.verify_device(data.data_ptr(), d_off, d_len, torch.from_numpy(exp.view(np.int32)).to(DEV), o, fb, nb,
                          total_bytes=total, max_len=max_len)
        torch.cuda.synchronize()
        assert (fb.item(), nb.item()) == (bad_at, 1)
        assert torch.equal(o, outs[0])
    finally:
        ctx.close()
        del data
        torch.cuda.empty_cache()


def test_config5_512gib_vlog_all_slices_vs_reference():
    """Config 5 on one MI355X: all 512 GiB as 8 distinct 64 GiB slices (slice s regenerated in place at stream offset
    s * span, as bench.py --config 5 does), every record's CRC against the reference, and the recovery-scan verify
    (stored word = Mask(reference CRC), db/value_log_reader.cc:109-122) clean on every slice."""
    off, ln = W.cfg3_layout(vlog=True)
    span = int(off[-1] + ln[-1])
    total, max_len = int(ln.sum()), int(ln.max())
    ref = golden("full_cfg5.u32")
    assert ref.size == 8 * off.size
    data = torch.empty(span + 64, dtype=torch.uint8, device=DEV)
    d_off, d_len = u64(off), u64(ln)
    ctx = kvsep.Context(0)
    ctx.reserve(off.size, total)
    o = torch.zeros(off.size, dtype=torch.int32, device=DEV)
    fb = torch.zeros(1, dtype=torch.int64, device=DEV)
    nb = torch.zeros(1, dtype=torch.int64, device=DEV)
    try:
        for s in range(8):
            kvsep.fill_splitmix64(data.data_ptr(), span, W.SEED + 1, s * span)
            exp = ref[s * off.size:(s + 1) * off.size]
            ctx.batch_device(data.data_ptr(), d_off, d_len, o, total_bytes=total, max_len=max_len)
            torch.cuda.synchronize()
            got = o.cpu().numpy().view(np.uint32)
            assert np.array_equal(got, exp), (s, np.flatnonzero(got != exp)[:8])
            stored = np.array([kvsep.mask(int(c)) for c in exp], dtype=np.uint32)
            ctx.verify_device(data.data_ptr(), d_off, d_len, torch.from_numpy(stored.view(np.int32)).to(DEV), o, fb,
                              nb, total_bytes=total, max_len=max_len)
            torch.cuda.synchronize()
            assert (fb.item(), nb.item()) == (-1, 0), s
    finally:
        ctx.close()
        del data
        torch.cuda.empty_cache()
