"""Synthetic workload layouts of BASELINE.json's configs, shared by tests and bench.

Data bytes always come from the splitmix64 byte stream (kvsep.splitmix64_bytes on the host,
kvsep_fill_splitmix64_device on the GPU, oracle_fill_splitmix64 in the oracle): byte i of stream
`seed` is byte (i & 7) of word mix(seed + ((i >> 3) + 1) * 0x9E3779B97F4A7C15).
"""
from __future__ import annotations

import numpy as np

SEED = 0x6B76736570617261  # "kvsepara" 
GAMMA = 0x9E3779B97F4A7C15
MASK64 = (1 << 64) - 1

CFG2_BLOCKS, CFG2_LEN = 65536, 4096
CFG3_BLOCKS, CFG3_LEN = 65536, 1 << 20
VLOG_PAYLOAD = 1_048_609          # 12-B WriteBatch header + tag + varint key + 16-B key + varint + 1 MiB value
VLOG_HEADER = 8                   # [masked crc LE32][len LE32], db/log_format.h:40, db/value_log_writer.cc:59-60
CFG4_BLOCKS = 1 << 20
CFG4_LEN_SEED = 42
ZIPF_S = 1.1
ZIPF_CLASSES = 18                 # k in [0, 17]: len ~ U[32*2^k, min(32*2^(k+1), 4 MiB + 1))
MAX_LEN = (4 << 20) + 1


def splitmix_words(seed: int, j: np.ndarray) -> np.ndarray:
    j = np.asarray(j, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = np.uint64(seed & MASK64) + (j + np.uint64(1)) * np.uint64(GAMMA)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def uniform_layout(count: int, length: int, stride: int | None = None, first: int = 0):
    """Blocks of `length` bytes at first + i*stride (stride defaults to length: packed)."""
    stride = length if stride is None else stride
    off = first + np.arange(count, dtype=np.uint64) * np.uint64(stride)
    return off, np.full(count, length, dtype=np.uint64)


def cfg2_layout():
    return uniform_layout(CFG2_BLOCKS, CFG2_LEN)


def cfg3_layout(vlog: bool = False, count: int = CFG3_BLOCKS):
    """Variant A: aligned 1 MiB blocks.  Variant B: vlog records, payload at 8 + i*(8+len) (odd offsets)."""
    if vlog:
        return uniform_layout(count, VLOG_PAYLOAD, VLOG_PAYLOAD + VLOG_HEADER, VLOG_HEADER)
    return uniform_layout(count, CFG3_LEN)


def zipf_lengths(count: int = CFG4_BLOCKS, seed: int = CFG4_LEN_SEED) -> np.ndarray:
    """Config 4 ragged lengths: class k with P(k) ~ (k+1)^-1.1, len uniform inside the class."""
    k = np.arange(ZIPF_CLASSES, dtype=np.float64)
    w = (k + 1.0) ** (-ZIPF_S)
    cdf = np.cumsum(w) / w.sum()
    i = np.arange(count, dtype=np.uint64)
    u = (splitmix_words(seed, 2 * i) >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    cls = np.minimum(np.searchsorted(cdf, u, side="right"), ZIPF_CLASSES - 1).astype(np.uint64)
    lo = np.uint64(32) << cls
    hi = np.minimum(np.uint64(32) << (cls + np.uint64(1)), np.uint64(MAX_LEN))
    r = splitmix_words(seed, 2 * i + 1)
    return lo + r % (hi - lo)


def cfg4_layout(count: int = CFG4_BLOCKS):
    length = zipf_lengths(count)
    off = np.zeros(count, dtype=np.uint64)
    if count > 1:
        off[1:] = np.cumsum(length[:-1], dtype=np.uint64)
    return off, length
