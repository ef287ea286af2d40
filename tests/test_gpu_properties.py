"""GPU property-based parity (hypothesis): random batches -- block counts, ragged lengths, any offsets,
overlaps, inits, piece sizes, max_len hints (which pick the split / unsplit / narrow paths) -- through the HIP
path, each bit-exact against the oracle on the same bytes."""
import numpy as np
import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

import kvsep
from kvsep import splitmix64_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

DEV = torch.device("cuda:0")
POOL = 4 << 20


@pytest.fixture(scope="module")
def pool():
    host = splitmix64_bytes(POOL + 64, 31337, 0)
    return host, torch.from_numpy(host).to(DEV)


@pytest.fixture(scope="module")
def ctxs():
    cs = {}
    for piece in (None, 1024, 4096, 64 * 1024):
        c = kvsep.Context(0)
        if piece:
            c.set_piece_bytes(piece)
        cs[piece] = c
    yield cs
    for c in cs.values():
        c.close()


def u64(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(DEV)


@settings(max_examples=60, deadline=None, suppress_health_check=[HealthCheck.function_scoped_fixture])
@given(data=st.data())
def test_random_batches_vs_oracle(pool, ctxs, oracle, data):
    host, dev = pool
    n = data.draw(st.integers(min_value=1, max_value=400), label="blocks")
    big = data.draw(st.sampled_from([64, 4096, 70000, 1 << 20]), label="length scale")
    rng = np.random.default_rng(data.draw(st.integers(min_value=0, max_value=2**32 - 1), label="seed"))
    ln = rng.integers(0, big + 1, n).astype(np.uint64)
    off = (rng.integers(0, POOL + 1, n).astype(np.uint64) % (np.uint64(POOL + 1) - ln)).astype(np.uint64)
    init = rng.integers(0, 2**32, n, dtype=np.uint64).astype(np.uint32)
    piece = data.draw(st.sampled_from([None, 1024, 4096, 64 * 1024]), label="piece")
    hint = data.draw(st.sampled_from(["none", "exact", "loose"]), label="max_len hint")
    max_len = 0 if hint == "none" else int(ln.max()) if hint == "exact" else int(ln.max()) * 2 + 1
    out = torch.zeros(n, dtype=torch.int32, device=DEV)
    ctxs[piece].batch_device(dev.data_ptr(), u64(off), u64(ln), out,
                             init=torch.from_numpy(init.view(np.int32)).to(DEV), max_len=max_len,
                             total_bytes=int(ln.sum()))
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    exp = oracle.batch(host, off, ln, init, threads=8)
    assert np.array_equal(got, exp), np.flatnonzero(got != exp)[:8]
