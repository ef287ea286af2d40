"""Host header walkers of the vlog and log/MANIFEST framings (no GPU)."""
import numpy as np

import kvsep
from kvsep import splitmix64_bytes
from framing_builders import log_image, vlog_image


def _payloads(n, seed, maxlen):
    rng = np.random.default_rng(seed)
    lens = rng.integers(0, maxlen, n)
    data = splitmix64_bytes(int(lens.sum()) + 1, seed, 0)
    out, p = [], 0
    for l in lens:
        out.append(data[p:p + l].tobytes())
        p += l
    return out


def test_vlog_walk_matches_writer(oracle):
    pl = _payloads(200, 1, 5000) + [b""]
    img = vlog_image(pl, oracle)
    off, ln, st, used = kvsep.vlog_walk(img)
    assert off.size == len(pl) and used == len(img)
    exp_off = np.cumsum([0] + [8 + len(p) for p in pl[:-1]]) + 8
    assert np.array_equal(off, exp_off) and ln.tolist() == [len(p) for p in pl]
    assert st.tolist() == [oracle.lib.oracle_crc32c_mask(oracle.extend(0, p)) for p in pl]


def test_vlog_walk_truncation_is_eof(oracle):
    pl = _payloads(10, 2, 3000)
    img = vlog_image(pl, oracle)
    full = kvsep.vlog_walk(img)[0].size
    assert kvsep.vlog_walk(img[:-1])[0].size == full - 1          # payload short by one byte
    last_hdr = len(img) - 8 - len(pl[-1])
    assert kvsep.vlog_walk(img[:last_hdr + 5])[0].size == full - 1  # header cut
    assert kvsep.vlog_walk(b"")[0].size == 0


def test_log_walk_matches_writer_fragments(oracle):
    recs = _payloads(40, 3, 90000) + [b"", b"x" * 32761, b"y" * 32762]
    img, phys = log_image(recs, oracle)
    off, ln, st, ty = kvsep.log_walk(img)
    assert off.size == len(phys)
    assert off.tolist() == [h + 6 for h, _, _ in phys]
    assert ln.tolist() == [1 + l for _, _, l in phys]
    assert ty.tolist() == [t for _, t, _ in phys]
    assert {2, 3, 4} <= set(ty.tolist())  # FIRST / MIDDLE / LAST fragments present


def test_log_accept_checksum_mismatch_like_log_test(oracle):
    """db/log_test.cc:413-418 ChecksumMismatch: one 3-byte record with a bad checksum -> nothing returned and
    10 bytes (7-byte header + payload) reported dropped."""
    img, phys = log_image([b"foo"], oracle)
    off = kvsep.log_walk(img)[0]
    acc, dropped = kvsep.log_accept(off, [0], len(img))
    assert acc.tolist() == [0] and dropped == 10
    acc, dropped = kvsep.log_accept(off, [1], len(img))
    assert acc.tolist() == [1] and dropped == 0


def test_log_accept_drops_rest_of_block_only(oracle):
    recs = _payloads(80, 5, 3000)
    img, phys = log_image(recs, oracle)
    off = kvsep.log_walk(img)[0]
    blk = (off - 6) // 32768
    ok = np.ones(off.size, np.uint8)
    bad = int(np.flatnonzero(blk == 1)[2])   # third record of block 1
    ok[bad] = 0
    acc, dropped = kvsep.log_accept(off, ok, len(img))
    expect = np.ones(off.size, np.uint8)
    expect[bad:] = 0
    expect[blk > 1] = 1                      # the reader resumes with the next block
    assert np.array_equal(acc, expect)
    assert dropped == 2 * 32768 - int(off[bad] - 6)


def test_log_walk_stops_at_zero_padding_and_bad_length(oracle):
    img, phys = log_image([b"abc" * 10], oracle)
    padded = img + b"\x00" * 100                       # preallocated zeros (db/log_reader.cc:243-249)
    assert kvsep.log_walk(padded)[0].size == 1
    bad = bytearray(img)
    bad[4] = 0xFF                                      # length beyond the block (:229-241)
    assert kvsep.log_walk(bytes(bad))[0].size == 0
