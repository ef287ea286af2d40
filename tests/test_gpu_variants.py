"""GPU parity of every kernel configuration the shipped library can run -- the wide kernel under each schedule
(static contiguous, static round-robin, guided) and piece size, and the narrow kernel at both workgroup sizes
(kvsep_crc32c_ctx_set_kernel) -- against the oracle, bit-exact: ragged blocks at every start offset mod 128
(every head length and row-grid phase relative to a cache line), random inits.  Also: the max_len hint is a
performance hint only -- a hint that understates the longest block still gives exact results on every kernel.
The A/B and ablation variants live only in the KVSEP_DIAG tools build (tools/libkvsep_diag.so) and are not
shipped."""
import numpy as np
import pytest

import kvsep
from kvsep import splitmix64_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda:0")


def u64(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(DEV)


def run(ctx, d, off, ln, init, max_len, base=None):
    out = torch.zeros(off.size, dtype=torch.int32, device=DEV)
    ctx.batch_device(d.data_ptr() if base is None else base, u64(off), u64(ln), out,
                     init=None if init is None else torch.from_numpy(init.view(np.int32)).to(DEV), max_len=max_len,
                     total_bytes=int(ln.sum()))
    torch.cuda.synchronize()
    return out.cpu().numpy().view(np.uint32)


@pytest.fixture(scope="module")
def ragged(oracle):
    rng = np.random.default_rng(20261016)
    n = 3000
    host = splitmix64_bytes(8 << 20, 99, 0)
    ln = np.concatenate([rng.integers(0, 40000, n - 40), np.arange(1000, 1040) * 16 + 7]).astype(np.uint64)
    off = (rng.integers(0, (host.size - 40000) // 128, n) * 128 + np.arange(n) % 128).astype(np.uint64)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    exp = oracle.batch(host, off, ln, init, threads=8)
    d = torch.from_numpy(host).to(DEV)
    return d, off, ln, init, exp


@pytest.mark.parametrize("sched", [None, False, True, "rr"])
def test_wide_schedules_ragged(ragged, sched):
    d, off, ln, init, exp = ragged
    ctx = kvsep.Context(0)
    try:
        ctx.set_kernel("wide")
        ctx.set_schedule(sched)
        for piece in (1024, 4096, 128 * 1024):
            ctx.set_piece_bytes(piece)
            got = run(ctx, d, off, ln, init, max_len=0)  # planned: pieces of long blocks
            assert np.array_equal(got, exp), (piece, sched, np.flatnonzero(got != exp)[:8])
        ctx.set_piece_bytes(64 * 1024)
        keep = ln <= 64 * 1024
        got = run(ctx, d, off[keep], ln[keep], init[keep], max_len=64 * 1024 + 1)  # unplanned, wide kernel
        assert np.array_equal(got, exp[keep])
    finally:
        ctx.close()


@pytest.mark.parametrize("kernel", ["narrow", "narrow16", "narrow8", "sorted", "claim", "claim16", "coop"])
def test_narrow_workgroups_ragged(ragged, kernel):
    d, off, ln, init, exp = ragged
    ctx = kvsep.Context(0)
    try:
        ctx.set_kernel(kernel)
        keep = ln <= 64 * 1024
        got = run(ctx, d, off[keep], ln[keep], init[keep], max_len=64 * 1024)
        assert np.array_equal(got, exp[keep])
    finally:
        ctx.close()


@pytest.mark.parametrize("kernel", ["auto", "wide", "narrow16", "narrow8", "sorted", "claim", "claim16", "coop"])
def test_understated_hint_is_exact(ragged, kernel):
    """max_len = 4 KiB although blocks run to 40 KB: blocks over the hint are deferred (narrow) or whole (wide)."""
    d, off, ln, init, exp = ragged
    ctx = kvsep.Context(0)
    try:
        ctx.set_kernel(kernel)
        got = run(ctx, d, off, ln, init, max_len=4096)
        assert np.array_equal(got, exp), np.flatnonzero(got != exp)[:8]
        got = run(ctx, d, off, ln, None, max_len=1)
        assert np.array_equal(got[ln == 0], np.zeros(int((ln == 0).sum()), np.uint32))
    finally:
        ctx.close()


@pytest.mark.parametrize("n,kernel", [((1 << 32) + 77, "narrow16"), ((9 << 30) + 5, "narrow16"),
                                      ((1 << 32) + 77, "sorted")])
def test_understated_hint_block_over_4gib(oracle, n, kernel):
    """A 2^32 + 77-byte block among 4 KiB blocks under a 4 KiB hint, on the narrow kernel: its length does not fit
    the narrow kernel's 32-bit staging, so it must take the deferred path with its full 64-bit length.  At 9 GiB + 5
    the deferred path cuts it into 10 parts of <= 1 GiB, two rounds of 8 slots."""
    buf = torch.empty(n + 4096 * 64 + 64, dtype=torch.uint8, device=DEV)
    kvsep.fill_splitmix64(buf.data_ptr(), buf.numel(), 4242, 0)
    ctx = kvsep.Context(0)
    try:
        ctx.set_kernel(kernel)
        off = np.concatenate([np.arange(64, dtype=np.uint64) * np.uint64(4096), [np.uint64(4096 * 64 + 3)]])
        ln = np.concatenate([np.full(64, 4096, np.uint64), [np.uint64(n)]])
        got = run(ctx, buf, off, ln, None, max_len=4096, base=buf.data_ptr())
        # the long block through the library's own planned path (checked against the oracle in test_gpu_parity)
        planned = run(kvsep.Context(0), buf, off[-1:], ln[-1:], None, max_len=0, base=buf.data_ptr())
        head = buf[:4096 * 64].cpu().numpy()
        assert np.array_equal(got[:64], oracle.batch(head, off[:64], ln[:64], threads=8))
        assert got[64] == planned[0]
    finally:
        ctx.close()
        del buf
        torch.cuda.empty_cache()
