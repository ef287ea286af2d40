"""Workload layouts match SURVEY.md §8(d)."""
import numpy as np

from kvsep import workloads as W


def test_cfg2():
    off, ln = W.cfg2_layout()
    assert off.size == 65536 and (ln == 4096).all() and int(off[-1]) == 65535 * 4096


def test_cfg3_variants():
    off, ln = W.cfg3_layout()
    assert int(ln.sum()) == 64 << 30
    off, ln = W.cfg3_layout(vlog=True)
    assert int(off[0]) == 8 and int(off[1]) == 8 + 8 + W.VLOG_PAYLOAD
    assert (off[1::2] % 2 == 1).all()  # odd records start at odd byte offsets
    assert (off % 16 != 0).mean() > 0.9  # almost no payload is 16-B aligned


def test_cfg4_stats():
    off, ln = W.cfg4_layout()
    assert ln.size == 1 << 20 and ln.min() >= 32 and ln.max() <= 4 << 20
    assert 140 << 30 < int(ln.sum()) < 160 << 30
    assert (ln <= 4096).mean() > 0.7
    assert np.array_equal(off[1:], np.cumsum(ln[:-1]))
