"""GPU parity of every wide-kernel build variant (KVSEP_CRC_VARIANT, launch_pieces_v in crc32c_device.hip)
and every narrow-kernel variant (KVSEP_NARROW) against the oracle, bit-exact: ragged blocks at every start
offset mod 128 (every head length and row-grid phase relative to a cache line), random inits, several piece
sizes, both schedules.  The default variant is covered by test_gpu_parity.py as well."""
import os

import numpy as np
import pytest

import kvsep
from kvsep import splitmix64_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda:0")
WIDE = ["0", "1", "2", "3", "5", "6", "7"]


def make_ctx(variant, narrow="1"):
    old = os.environ.get("KVSEP_CRC_VARIANT"), os.environ.get("KVSEP_NARROW")
    os.environ["KVSEP_CRC_VARIANT"], os.environ["KVSEP_NARROW"] = variant, narrow
    try:
        return kvsep.Context(0)
    finally:
        for k, v in zip(("KVSEP_CRC_VARIANT", "KVSEP_NARROW"), old):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def u64(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(DEV)


def run(ctx, d, off, ln, init, max_len):
    out = torch.zeros(off.size, dtype=torch.int32, device=DEV)
    ctx.batch_device(d.data_ptr(), u64(off), u64(ln), out,
                     init=torch.from_numpy(init.view(np.int32)).to(DEV), max_len=max_len,
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


@pytest.mark.parametrize("variant", WIDE)
def test_wide_variant_ragged(ragged, variant):
    d, off, ln, init, exp = ragged
    ctx = make_ctx(variant)
    try:
        for piece in (1024, 4096, 128 * 1024):
            ctx.set_piece_bytes(piece)
            for dyn in (None, False, True):
                ctx.set_schedule(dyn)
                got = run(ctx, d, off, ln, init, max_len=0)  # planned: pieces of long blocks
                assert np.array_equal(got, exp), (variant, piece, dyn, np.flatnonzero(got != exp)[:8])
        ctx.set_piece_bytes(64 * 1024)
        ctx.set_schedule(None)
        keep = ln <= 64 * 1024
        got = run(ctx, d, off[keep], ln[keep], init[keep], max_len=64 * 1024 + 1)  # unplanned, wide kernel
        assert np.array_equal(got, exp[keep])
    finally:
        ctx.close()


@pytest.mark.parametrize("narrow", ["1", "2", "3", "4", "5", "6", "7", "9"])
def test_narrow_variant_ragged(ragged, narrow):
    d, off, ln, init, exp = ragged
    ctx = make_ctx("1", narrow)
    try:
        keep = ln <= 64 * 1024
        got = run(ctx, d, off[keep], ln[keep], init[keep], max_len=64 * 1024)
        assert np.array_equal(got, exp[keep])
    finally:
        ctx.close()
