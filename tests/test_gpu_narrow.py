"""GPU parity of the narrow kernel (8 lanes per block, 8 blocks per wavefront), which serves unsplit batches
of many short blocks (SST blocks, WAL fragments; routing rule use_narrow() in crc32c_device.hip), forced here
for every batch whose max_len hint is <= 64 KiB.  Bit-exact vs the oracle restatement and
vs the wide kernel (set_kernel("wide") context), on ragged lengths, any alignment, non-zero init, partial
8-block groups and verify mode."""

import numpy as np
import pytest

import kvsep
from kvsep import splitmix64_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda:0")
NARROW_MAX = 64 * 1024


@pytest.fixture(scope="module")
def ctxs():
    narrow = kvsep.Context(0)
    narrow.set_kernel("narrow")  # narrow kernel whenever max_len <= 64 KiB (the default routes by count)
    wide = kvsep.Context(0)
    wide.set_kernel("wide")
    yield narrow, wide
    narrow.close()
    wide.close()


def dev_u64(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(DEV)


def dev_u32(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint32).view(np.int32)).to(DEV)


def run(ctx, d, off, ln, init=None, max_len=None):
    out = torch.zeros(len(off), dtype=torch.int32, device=DEV)
    ml = int(ln.max()) if max_len is None and len(ln) else (max_len or 0)
    ctx.batch_device(d.data_ptr(), dev_u64(off), dev_u64(ln), out, init=None if init is None else dev_u32(init),
                     max_len=ml, total_bytes=int(np.sum(ln, dtype=np.uint64)))
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


@pytest.fixture(scope="module")
def pool():
    data = splitmix64_bytes(8 << 20, 1234, 0)
    t = torch.zeros(data.size + 64, dtype=torch.uint8, device=DEV)
    t[:data.size] = torch.from_numpy(data).to(DEV)
    return data, t


@pytest.mark.parametrize("count", [1, 7, 8, 9, 63, 64, 65, 1000, 4099])
def test_ragged_any_alignment(ctxs, oracle, pool, count):
    narrow, wide = ctxs
    data, d = pool
    rng = np.random.default_rng(count)
    ln = rng.integers(0, NARROW_MAX + 1, count).astype(np.uint64)
    short = rng.random(count) < 0.4
    ln[short] = rng.integers(0, 300, int(short.sum()))
    off = rng.integers(0, data.size - NARROW_MAX - 1, count).astype(np.uint64)
    init = rng.integers(0, 2**32, count, dtype=np.uint64).astype(np.uint32)
    exp = oracle.batch(data, off, ln, init, threads=8)
    got = run(narrow, d, off, ln, init)
    assert np.array_equal(got, exp)
    assert np.array_equal(run(wide, d, off, ln, init), exp)
    assert np.array_equal(run(narrow, d, off, ln), oracle.batch(data, off, ln, threads=8))


@pytest.mark.parametrize("blen", [16, 127, 128, 129, 4096, 4097, 16384, 65535, 65536])
def test_uniform_lengths_packed(ctxs, oracle, pool, blen):
    narrow, _ = ctxs
    data, d = pool
    count = min(2048, (data.size - 64) // blen)
    for shift in (0, 1, 8, 15):
        off = (np.arange(count, dtype=np.uint64) * np.uint64(blen) + np.uint64(shift))
        ln = np.full(count, blen, np.uint64)
        assert np.array_equal(run(narrow, d, off, ln), oracle.batch(data, off, ln, threads=8)), shift


def test_mixed_slot_lengths_in_one_group(ctxs, oracle, pool):
    """The 8 blocks of a group differ in length (divergent row counts, empty slots, head-only slots)."""
    narrow, _ = ctxs
    data, d = pool
    ln = np.array([0, 1, 15, 16, 17, 65536, 4096, 3, 128, 129, 255, 0, 0, 0, 40000, 7], np.uint64)
    off = np.array([5, 6, 7, 16, 31, 100, 4096 * 3 + 9, 1, 2, 3, 4, 5, 6, 7, 8, 9], np.uint64) * np.uint64(97)
    init = np.arange(ln.size, dtype=np.uint32) * np.uint32(0x9E3779B1)
    assert np.array_equal(run(narrow, d, off, ln, init), oracle.batch(data, off, ln, init, threads=4))


def test_verify_mode_narrow(ctxs, oracle, pool):
    narrow, _ = ctxs
    data, d = pool
    count = 2000  # 8,192,000 B of the 8 MiB pool
    off = np.arange(count, dtype=np.uint64) * np.uint64(4096)
    ln = np.full(count, 4096, np.uint64)
    crc = oracle.batch(data, off, ln, threads=8)
    masked = np.array([oracle.lib.oracle_crc32c_mask(int(c)) for c in crc], np.uint32)
    for b in (17, 1500, 1999):
        masked[b] ^= 1
    out = torch.zeros(count, dtype=torch.int32, device=DEV)
    fb = torch.zeros(1, dtype=torch.int64, device=DEV)
    nb = torch.zeros(1, dtype=torch.int64, device=DEV)
    narrow.verify_device(d.data_ptr(), dev_u64(off), dev_u64(ln), dev_u32(masked), out, fb, nb,
                         total_bytes=int(ln.sum()), max_len=4096)
    torch.cuda.synchronize()
    assert fb.item() == 17 and nb.item() == 3
    assert np.array_equal(out.cpu().numpy().view(np.uint32), crc)


@pytest.mark.parametrize("count", [1, 63, 64, 65, 200, 5000])
def test_sorted_windows_ragged(oracle, pool, count):
    """The sorted-window form (crc32c_narrow_sorted_kernel): Zipf-like lengths, partial windows, empty blocks, blocks
    over the hint (deferred), any alignment, random inits; batch and verify forms; and that auto routing picks it
    for a ragged batch and keeps the plain narrow kernel for a uniform one."""
    data, d = pool
    rng = np.random.default_rng(count + 7)
    ln = np.minimum((32 * 2.0 ** rng.integers(0, 11, count)) * rng.random(count), 40000).astype(np.uint64)
    ln[rng.random(count) < 0.05] = 0
    off = rng.integers(0, data.size - 40001, count).astype(np.uint64)
    init = rng.integers(0, 2**32, count, dtype=np.uint64).astype(np.uint32)
    exp = oracle.batch(data, off, ln, init, threads=8)
    ctx = kvsep.Context(0)
    try:
        ctx.set_kernel("sorted")
        assert np.array_equal(run(ctx, d, off, ln, init), exp)
        assert np.array_equal(run(ctx, d, off, ln, init, max_len=2048), exp)  # longer blocks deferred
        masked = np.array([oracle.lib.oracle_crc32c_mask(int(c)) for c in exp], np.uint32)
        bad = sorted({0, count // 2, count - 1})
        masked[bad] ^= 4
        out = torch.zeros(count, dtype=torch.int32, device=DEV)
        fb = torch.zeros(1, dtype=torch.int64, device=DEV)
        nb = torch.zeros(1, dtype=torch.int64, device=DEV)
        ctx.verify_device(d.data_ptr(), dev_u64(off), dev_u64(ln), dev_u32(masked), out, fb, nb, init=dev_u32(init),
                          total_bytes=int(ln.sum()), max_len=int(ln.max()))
        torch.cuda.synchronize()
        assert (fb.item(), nb.item()) == (bad[0], len(bad))
        assert np.array_equal(out.cpu().numpy().view(np.uint32), exp)
        ctx.set_kernel("auto")
        n = 40000  # enough blocks for the narrow kernels (use_narrow); ragged -> sorted, uniform -> plain
        assert ctx.kernel_name(n, 32768, n * 2000) == "crc32c_narrow_sorted_kernel"
        assert ctx.kernel_name(n, 4096, n * 4096) == "crc32c_narrow_claim_kernel"  # uniform, < 256 Ki blocks
        assert ctx.kernel_name(n, 4096) == "crc32c_narrow_claim_kernel"  # total_bytes unknown: not ragged
        assert ctx.kernel_name(3 << 17, 4096, (3 << 17) * 4096) == "crc32c_narrow_claim_kernel"  # 1.5 GiB
        assert ctx.kernel_name(1 << 19, 4096, (1 << 19) * 4096) == "crc32c_narrow_kernel"  # 2 GiB and up: 8-wave
        assert ctx.kernel_name(n, 16384, n * 16384) == "crc32c_narrow_kernel"  # blocks over 12 KiB
        # 16-lane claim kernel (claim16_route): uniform 8-12 KiB blocks, >= 4 Ki of them, <= 512 MiB
        assert ctx.kernel_name(6000, 10240, 6000 * 10240) == "crc32c_narrow_claim_kernel"  # was the wide kernel
        assert ctx.kernel_name(3000, 10240, 3000 * 10240) == "crc32c_pieces_kernel"  # too few blocks
        assert ctx.kernel_name(1 << 17, 8192, (1 << 17) * 8192) == "crc32c_narrow_kernel"  # 1 GiB
        assert ctx.kernel_name(6000, 10240, 6000 * 4000) == "crc32c_pieces_kernel"  # ragged, too few for sorted
    finally:
        ctx.close()


@pytest.mark.parametrize("kernel", ["narrow16", "narrow8", "sorted", "claim", "claim16", "coop"])
@pytest.mark.parametrize("count", [70000, 200000])
def test_verify_several_groups_per_wave(oracle, pool, kernel, count):
    """Verify form with several 8-block groups per wave (3 and 7 per 64-block window at these counts): the sorted
    kernel once returned wrong CRCs from the third group of a window on in this form only (tools/soak.py); the
    compare now runs after the kernel (verify_finish_kernel).  Random offsets (overlapping), ragged short lengths,
    planted mismatches."""
    data, d = pool
    rng = np.random.default_rng(count)
    ln = rng.integers(0, 201, count).astype(np.uint64)
    off = rng.integers(0, data.size - 256, count).astype(np.uint64)
    exp = oracle.batch(data, off, ln, threads=8)
    masked = np.array([oracle.lib.oracle_crc32c_mask(int(c)) for c in exp], np.uint32)
    bad = sorted({5, count // 3, count - 2})
    masked[bad] ^= 0x100
    ctx = kvsep.Context(0)
    try:
        ctx.set_kernel(kernel)
        out = torch.zeros(count, dtype=torch.int32, device=DEV)
        fb = torch.zeros(1, dtype=torch.int64, device=DEV)
        nb = torch.zeros(1, dtype=torch.int64, device=DEV)
        ctx.verify_device(d.data_ptr(), dev_u64(off), dev_u64(ln), dev_u32(masked), out, fb, nb,
                          total_bytes=int(ln.sum()), max_len=int(ln.max()))
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy().view(np.uint32), exp)
        assert (fb.item(), nb.item()) == (bad[0], len(bad))
        assert np.array_equal(run(ctx, d, off, ln), exp)
    finally:
        ctx.close()


@pytest.mark.parametrize("kernel", ["narrow16", "narrow8", "sorted", "claim", "claim16", "coop"])
def test_every_end_geometry(oracle, pool, kernel):
    """Every case of the slot's end path: m = 0..7 whole 16-B chunks between the 128-B grid and the 16-B end (m = 7
    uses all of lanes 0..6 of the tail load), each with head and tail bytes 0..15, with and without body rows.  The
    16-lane slots (claim16) have 256-B rows: m = 0..15 on the 256-B grid."""
    data, d = pool
    ctx = kvsep.Context(0)
    ctx.set_kernel(kernel)
    row = 256 if kernel == "claim16" else 128
    ps, pe = [], []
    for rows in (-1, 0, 1, 3):  # -1: no row on the grid (a1 = h0 + 16 m)
        for m in range(row // 16):
            for head in range(16):
                for tail in (0, 1, 7, 15):
                    start = 6 * row * len(ps) + 16 + row - head  # ps % 16 == (16 - head) % 16: `head` head bytes
                    h0 = start + head
                    a1 = h0 + 16 * m if rows < 0 else ((h0 + row - 1) // row + rows) * row + 16 * m
                    ps.append(start)
                    pe.append(a1 + tail)
    off = np.array(ps, np.uint64)
    ln = np.array(pe, np.uint64) - off
    assert int(off[-1] + ln[-1]) < data.size
    init = np.arange(off.size, dtype=np.uint32) * np.uint32(2654435761)
    got = run(ctx, d, off, ln, init=init)
    ctx.close()
    assert np.array_equal(got, oracle.batch(data, off, ln, init))


@pytest.mark.parametrize("kernel", ["narrow16", "narrow8", "sorted", "claim", "claim16", "coop"])
def test_verify_mismatch_on_deferred_block(oracle, pool, kernel):
    """Verify form under an understated max_len: blocks longer than the hint leave their 8-block group and
    are checksummed by the deferred walk, whose compare is verify_uniform over the wave-uniform stored word.  Mismatches
    planted on deferred blocks (and one on an in-group block) must give the exact first_bad / nbad and CRCs."""
    data, d = pool
    rng = np.random.default_rng(4242)
    count = 3000
    ln = rng.integers(0, 2049, count).astype(np.uint64)
    long_ix = rng.choice(count, 40, replace=False)
    ln[long_ix] = rng.integers(2049, 40000, long_ix.size)  # over the 2048-B hint: deferred
    off = rng.integers(0, data.size - 40001, count).astype(np.uint64)
    init = rng.integers(0, 2**32, count, dtype=np.uint64).astype(np.uint32)
    exp = oracle.batch(data, off, ln, init, threads=8)
    deferred = sorted(int(i) for i in long_ix[:3])
    short_bad = int(np.flatnonzero(ln <= 2048)[count // 2 % 100])
    bad = sorted(set(deferred + [short_bad]))
    ctx = kvsep.Context(0)
    try:
        ctx.set_kernel(kernel)
        for planted in ([deferred[-1]], bad):  # a deferred block alone, then mixed with an in-group one
            m = np.array([oracle.lib.oracle_crc32c_mask(int(c)) for c in exp], np.uint32)
            m[planted] ^= 0x20
            out = torch.zeros(count, dtype=torch.int32, device=DEV)
            fb = torch.zeros(1, dtype=torch.int64, device=DEV)
            nb = torch.zeros(1, dtype=torch.int64, device=DEV)
            ctx.verify_device(d.data_ptr(), dev_u64(off), dev_u64(ln), dev_u32(m), out, fb, nb, init=dev_u32(init),
                              total_bytes=int(ln.sum()), max_len=2048)
            torch.cuda.synchronize()
            assert np.array_equal(out.cpu().numpy().view(np.uint32), exp)
            assert (fb.item(), nb.item()) == (min(planted), len(planted)), planted
    finally:
        ctx.close()
