"""Property-based checks (hypothesis) of the library's host leg and host logic against the oracle, no GPU:
the SSE4.2 host CRC (the drop-in's small-input leg) on arbitrary bytes / inits / splits, the affine structure of
CRC-32C that the kernels' combine relies on, Mask/Unmask, and the framing walkers on arbitrary bytes."""
import numpy as np
from hypothesis import given, settings
from hypothesis import strategies as st

import kvsep
from framing_builders import vlog_image

BYTES = st.binary(min_size=0, max_size=5000)
U32 = st.integers(min_value=0, max_value=2**32 - 1)


@settings(max_examples=300, deadline=None)
@given(data=BYTES, init=U32)
def test_host_extend_matches_oracle(oracle, data, init):
    assert kvsep.extend_host(init, data) == oracle.extend(init, data)


@settings(max_examples=200, deadline=None)
@given(a=BYTES, b=BYTES, init=U32)
def test_extend_split_invariance(a, b, init):
    """util/crc32c_test.cc:43-45 generalised: Extend(Extend(i, a), b) == Extend(i, a || b)."""
    assert kvsep.extend_host(kvsep.extend_host(init, a), b) == kvsep.extend_host(init, a + b)


@settings(max_examples=200, deadline=None)
@given(st.data())
def test_crc_is_affine(data):
    """R(x ^ y) = R(x) ^ R(y) ^ R(0) for equal lengths: the linearity behind the piece / lane combine."""
    n = data.draw(st.integers(min_value=0, max_value=3000))
    x = np.frombuffer(data.draw(st.binary(min_size=n, max_size=n)), np.uint8)
    y = np.frombuffer(data.draw(st.binary(min_size=n, max_size=n)), np.uint8)
    z = bytes(n)
    lhs = kvsep.extend_host(0, (x ^ y).tobytes())
    assert lhs == kvsep.extend_host(0, x.tobytes()) ^ kvsep.extend_host(0, y.tobytes()) ^ kvsep.extend_host(0, z)


@settings(max_examples=300, deadline=None)
@given(c=U32)
def test_mask_roundtrip(oracle, c):
    m = kvsep.mask(c)
    assert m == oracle.lib.oracle_crc32c_mask(c)
    assert kvsep.unmask(m) == c and kvsep.unmask(kvsep.mask(m)) == m  # util/crc32c_test.cc:47-53


@settings(max_examples=100, deadline=None)
@given(payloads=st.lists(st.binary(max_size=700), max_size=12), cut=st.integers(min_value=0, max_value=10**6))
def test_vlog_walk_prefixes(oracle, payloads, cut):
    """Every prefix of a framed vlog walks to exactly the records that are complete in it (reader eof rule)."""
    img = vlog_image(payloads, oracle)
    cut = cut % (len(img) + 1)
    off, ln, st_, used = kvsep.vlog_walk(img[:cut])
    ends = np.cumsum([8 + len(p) for p in payloads]) if payloads else np.zeros(0)
    assert off.size == int(np.sum(ends <= cut)) and used == (int(ends[off.size - 1]) if off.size else 0)
    for k in range(off.size):
        assert int(ln[k]) == len(payloads[k]) and kvsep.unmask(int(st_[k])) == oracle.extend(0, payloads[k])


@settings(max_examples=100, deadline=None)
@given(junk=st.binary(max_size=70000))
def test_log_walk_arbitrary_bytes(junk):
    """The MANIFEST walker on arbitrary bytes: records stay inside the image and inside their 32 KiB block."""
    off, ln, _, _ = kvsep.log_walk(junk)
    for o, n in zip(off.tolist(), ln.tolist()):
        hdr = o - 6
        assert o + n <= len(junk) and hdr // 32768 == (o + n - 1) // 32768
