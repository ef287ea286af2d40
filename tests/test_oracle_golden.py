"""The oracle (oracle/crc32c_oracle.c) pinned against golden vectors captured from the compiled
reference util/crc32c.cc, and util/crc32c_test.cc restated (config 1).  CPU only."""
import numpy as np

from kvsep import splitmix64_bytes
from kvsep import workloads as W


def _known_bytes(k):
    if k["hex"] is not None:
        return bytes.fromhex(k["hex"])
    return bytes([k["fill"]["byte"]]) * k["fill"]["n"]


def test_crc32c_test_cc_standard_results(oracle):
    # util/crc32c_test.cc:12-39 (RFC 3720 B.4)
    assert oracle.extend(0, bytes(32)) == 0x8A9136AA
    assert oracle.extend(0, b"\xff" * 32) == 0x62A8AB43
    assert oracle.extend(0, bytes(range(32))) == 0x46DD794E
    assert oracle.extend(0, bytes(range(31, -1, -1))) == 0x113FDB5C
    iscsi = bytes([0x01, 0xC0] + [0] * 14 + [0x14, 0, 0, 0, 0, 0, 0x04, 0, 0, 0, 0, 0x14, 0, 0, 0, 0x18, 0x28]
                  + [0] * 7 + [0x02] + [0] * 7)
    assert len(iscsi) == 48 and oracle.extend(0, iscsi) == 0xD9963A56


def test_crc32c_test_cc_values_extend_mask(oracle):
    # util/crc32c_test.cc:41-53
    assert oracle.extend(0, b"a") != oracle.extend(0, b"foo")
    assert oracle.extend(0, b"hello world") == oracle.extend(oracle.extend(0, b"hello "), b"world")
    crc = oracle.extend(0, b"foo")
    m = oracle.lib.oracle_crc32c_mask
    u = oracle.lib.oracle_crc32c_unmask
    assert crc != m(crc) and crc != m(m(crc))
    assert crc == u(m(crc)) and crc == u(u(m(m(crc))))


def test_self_test_buffer(oracle):
    # util/crc32c.cc:267-274: the accelerated backend must give 0xdcbc59fa for "TestCRCBuffer"
    assert oracle.extend(0, b"TestCRCBuffer") == 0xDCBC59FA


def test_known_vectors(oracle, golden):
    for k in golden["known"]:
        assert oracle.extend(0, _known_bytes(k)) == k["value"], k["name"]
    ke = golden["known_extend"]
    assert oracle.extend(ke["init"], ke["data"].encode()) == ke["value"]


def test_sweep_all_offsets_lengths(oracle, golden):
    sw = golden["sweep"]
    data = splitmix64_bytes(4096, sw["seed"], sw["stream_offset"])
    raw = np.zeros(4096 + 128, np.uint8)
    b = (-raw.ctypes.data) % 64
    raw[b:b + 4096] = data
    base = raw.ctypes.data + b
    for o in range(16):
        for n in range(257):
            assert oracle.extend_addr(0, base + o, n) == sw["crc_init0"][o][n], (o, n)
            assert oracle.extend_addr(sw["init"][o][n], base + o, n) == sw["crc_init"][o][n], (o, n)


def test_large(oracle, golden):
    data = splitmix64_bytes((4 << 20) + 64, W.SEED + 1, 0)
    for c in golden["large"]:
        assert oracle.extend_addr(c["init"], data.ctypes.data + c["offset"], c["len"]) == c["crc"], c


def test_cfg4_prefix(oracle, golden):
    g = golden["cfg4"]
    off, ln = W.cfg4_layout(g["count"])
    assert ln.tolist() == g["len"]
    data = splitmix64_bytes(int(off[-1] + ln[-1]), g["seed"], 0)
    got = oracle.batch(data, off, ln, threads=4)
    assert got.tolist() == g["crc"]


def test_mask_pairs(oracle, golden):
    for m in golden["mask"]:
        assert oracle.lib.oracle_crc32c_mask(m["crc"]) == m["masked"]
        assert oracle.lib.oracle_crc32c_unmask(m["crc"]) == m["unmask_of_crc"]


def test_oracle_splitmix_matches_numpy(oracle):
    for so, n in ((0, 100), (3, 77), (4093, 300)):
        a = np.zeros(n, np.uint8)
        oracle.lib.oracle_fill_splitmix64(a.ctypes.data, n, W.SEED, so)
        assert np.array_equal(a, splitmix64_bytes(n, W.SEED, so))


def test_oracle_batch_threads_agree(oracle):
    off, ln = W.cfg4_layout(2000)
    data = splitmix64_bytes(int(off[-1] + ln[-1]), 7, 0)
    assert np.array_equal(oracle.batch(data, off, ln, threads=1), oracle.batch(data, off, ln, threads=8))


# ---------------------------------------------------------------- full-size reference files (make_fullsize_golden.py)
import os  # noqa: E402

_GOLDEN_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _full(name):
    return np.fromfile(os.path.join(_GOLDEN_DIR, name), dtype="<u4")


def test_fullsize_files_agree_with_the_small_fixtures(golden):
    c2, c5, c4, c3a = _full("full_cfg2.u32"), _full("full_cfg5.u32"), _full("full_cfg4.u32"), _full("full_cfg3a.u32")
    assert (c2.size, c3a.size, c5.size, c4.size) == (8 * 65536, 8 * 65536, 8 * 65536, 1 << 20)  # 8-rank batches
    g2 = golden["cfg2"]
    assert c2[:256].tolist() == g2["first"]
    r0 = c2[:65536]  # rank 0's part is config 2 itself
    assert int(np.bitwise_xor.reduce(r0)) == g2["xor"] and int(r0.astype(np.uint64).sum()) == g2["sum"]
    assert c5[:32].tolist() == golden["cfg3b"]["crc"]          # slice 0 of config 5 is config 3b
    assert c4[:512].tolist() == golden["cfg4"]["crc"]


def _oracle_blocks(oracle, seed, base, off, ln, idx):
    out = []
    for i in idx:
        d = splitmix64_bytes(int(ln[i]), seed, base + int(off[i]))
        out.append(oracle.extend_addr(0, d.ctypes.data, d.size))
    return out


def test_oracle_matches_fullsize_reference_samples(oracle):
    """The restatement against the reference's whole-batch outputs, on blocks spread over each batch (config 5:
    every slice, i.e. stream offsets up to 448 GiB)."""
    rng = np.random.default_rng(7)
    off, ln = W.cfg3_layout()
    span = int(off[-1] + ln[-1])
    c3a = _full("full_cfg3a.u32")
    for r in (0, 3, 7):  # rank r's blocks: stream bytes r * span + off[i], entry r * 65,536 + i
        idx = rng.integers(0, off.size, 2)
        assert _oracle_blocks(oracle, W.SEED + 1, r * span, off, ln, idx) == c3a[r * off.size + idx].tolist(), r
    off, ln = W.cfg3_layout(vlog=True)
    span = int(off[-1] + ln[-1])
    c5 = _full("full_cfg5.u32")
    for s in range(8):
        idx = rng.integers(0, off.size, 2)
        assert _oracle_blocks(oracle, W.SEED + 1, s * span, off, ln, idx) == c5[s * off.size + idx].tolist(), s
    off, ln = W.cfg4_layout()
    idx = np.concatenate([rng.integers(0, off.size, 24), [off.size - 1]])
    assert _oracle_blocks(oracle, W.SEED + 2, 0, off, ln, idx) == _full("full_cfg4.u32")[idx].tolist()
    off, ln = W.cfg2_layout()
    span = int(off[-1] + ln[-1])
    c2 = _full("full_cfg2.u32")
    for r in range(8):
        idx = rng.integers(0, off.size, 8)
        assert _oracle_blocks(oracle, W.SEED, r * span, off, ln, idx) == c2[r * off.size + idx].tolist(), r
