#!/usr/bin/env python3
"""Generate tests/golden/crc32c_golden.json from the REAL reference implementation.

Runs only where /root/reference exists (this container): `make -C oracle ref` compiles
/root/reference/util/crc32c.cc (+ oracle/ref_shim.cc) into oracle/_ref/libref_crc32c.so, and this
script calls it through ctypes on synthetic inputs (splitmix64 stream, kvsep/workloads.py).  Only the
resulting numbers -- inputs are regenerable from (seed, offset, length) -- are committed.

Fixture groups
  known      util/crc32c_test.cc:12-53 inputs (+ "123456789", db_bench's 4 KiB of 'x',
             benchmarks/db_bench.cc:693-710, and the self-test buffer of util/crc32c.cc:267-274)
  sweep      every length 0..256 at every start offset 0..15 of a 16-B aligned buffer, init 0 and a
             random init per case
  large      4 KiB .. 4 MiB+1 at offsets {0,1,3,7,8,15}, init 0 and random
  cfg2       65,536 x 4 KiB packed blocks (config 2): XOR / sum / CRC-of-CRCs digests + first 256
  cfg3b      first 32 vlog records of config 3 variant B (1,048,609 B at 8 + i*(8+len))
  cfg4       first 512 blocks of the config-4 Zipf layout
  mask       Mask/Unmask pairs (util/crc32c.h:22-38)
"""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(ROOT, "kv-separate_amd"))
from kvsep import workloads as W  # noqa: E402
from kvsep import splitmix64_bytes  # noqa: E402

REF_SO = os.path.join(ROOT, "oracle", "_ref", "libref_crc32c.so")


def load_ref():
    if not os.path.exists(REF_SO):
        subprocess.check_call(["make", "-C", os.path.join(ROOT, "oracle"), "ref"])
    r = ctypes.CDLL(REF_SO)
    r.ref_crc32c_extend.restype = ctypes.c_uint32
    r.ref_crc32c_extend.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t]
    r.ref_crc32c_mask.restype = ctypes.c_uint32
    r.ref_crc32c_mask.argtypes = [ctypes.c_uint32]
    r.ref_crc32c_unmask.restype = ctypes.c_uint32
    r.ref_crc32c_unmask.argtypes = [ctypes.c_uint32]
    return r


def aligned_buffer(data: np.ndarray, align: int = 64) -> tuple[np.ndarray, int]:
    raw = np.zeros(data.size + 2 * align, dtype=np.uint8)
    base = (-raw.ctypes.data) % align
    raw[base:base + data.size] = data
    return raw, raw.ctypes.data + base


def main():
    r = load_ref()

    def ext(init, addr, n):
        return int(r.ref_crc32c_extend(init, addr, n))

    def ext_bytes(init, b: bytes):
        a = np.frombuffer(b, dtype=np.uint8).copy() if b else np.zeros(1, np.uint8)
        return ext(init, a.ctypes.data, len(b))

    rng = np.random.Generator(np.random.PCG64(20261015))
    out = {"generator": "tests/golden/make_golden.py", "reference": "util/crc32c.cc (compiled, portable path)"}

    iscsi = bytes([0x01, 0xc0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0x14, 0, 0, 0, 0, 0, 0x04, 0,
                   0, 0, 0, 0x14, 0, 0, 0, 0x18, 0x28, 0, 0, 0, 0, 0, 0, 0, 0x02, 0, 0, 0, 0, 0, 0, 0])
    known = [
        ("zeros32", bytes(32)), ("ones32", b"\xff" * 32), ("inc32", bytes(range(32))),
        ("dec32", bytes(range(31, -1, -1))), ("iscsi48", iscsi), ("a", b"a"), ("foo", b"foo"),
        ("hello_world", b"hello world"), ("hello_", b"hello "), ("digits", b"123456789"),
        ("TestCRCBuffer", b"TestCRCBuffer"), ("x4096", b"x" * 4096), ("zeros1MiB", bytes(1 << 20)), ("empty", b""),
    ]
    out["known"] = [{"name": n, "hex": b.hex() if len(b) <= 64 else None,
                     "fill": None if len(b) <= 64 else {"byte": b[0], "n": len(b)},
                     "value": ext_bytes(0, b)} for n, b in known]
    out["known_extend"] = {"init": ext_bytes(0, b"hello "), "data": "world",
                           "value": ext_bytes(ext_bytes(0, b"hello "), b"world")}

    # sweep: stream SEED from stream offset 0, placed at a 64-B aligned address
    sw = splitmix64_bytes(4096, W.SEED, 0)
    raw, base = aligned_buffer(sw)
    inits = rng.integers(0, 2**32, size=(16, 257), dtype=np.uint64).astype(np.uint32)
    crc0 = [[ext(0, base + o, n) for n in range(257)] for o in range(16)]
    crci = [[ext(int(inits[o, n]), base + o, n) for n in range(257)] for o in range(16)]
    out["sweep"] = {"seed": W.SEED, "stream_offset": 0, "init": inits.tolist(), "crc_init0": crc0, "crc_init": crci}

    # large: stream SEED+1, block at buffer offset `o`
    lg = []
    big = splitmix64_bytes((4 << 20) + 64, W.SEED + 1, 0)
    raw2, base2 = aligned_buffer(big)
    for n in (4096, 65536, 1 << 20, W.VLOG_PAYLOAD, 4 << 20, (4 << 20) + 1):
        for o in (0, 1, 3, 7, 8, 15):
            if o + n > big.size:
                continue
            init = int(rng.integers(0, 2**32))
            lg.append({"seed": W.SEED + 1, "offset": o, "len": n, "init": 0, "crc": ext(0, base2 + o, n)})
            lg.append({"seed": W.SEED + 1, "offset": o, "len": n, "init": init, "crc": ext(init, base2 + o, n)})
    out["large"] = lg

    # config 2: 65,536 x 4 KiB packed, stream SEED from 0
    off, ln = W.cfg2_layout()
    d2 = splitmix64_bytes(int(ln.sum()), W.SEED, 0)
    raw3, base3 = aligned_buffer(d2)
    c2 = np.array([ext(0, base3 + int(off[i]), int(ln[i])) for i in range(off.size)], dtype=np.uint32)
    out["cfg2"] = {"seed": W.SEED, "count": int(off.size), "len": int(ln[0]), "first": c2[:256].tolist(),
                   "xor": int(np.bitwise_xor.reduce(c2)), "sum": int(c2.astype(np.uint64).sum()),
                   "crc_of_crcs": ext(0, c2.ctypes.data, c2.nbytes)}
    del d2, raw3

    # config 3 variant B: first 32 vlog records, stream SEED+1
    off, ln = W.cfg3_layout(vlog=True, count=32)
    span = int(off[-1] + ln[-1])
    d3 = splitmix64_bytes(span, W.SEED + 1, 0)
    raw4, base4 = aligned_buffer(d3)
    out["cfg3b"] = {"seed": W.SEED + 1, "count": 32,
                    "crc": [ext(0, base4 + int(off[i]), int(ln[i])) for i in range(32)]}
    del d3, raw4

    # config 4: first 512 Zipf blocks, stream SEED+2
    off, ln = W.cfg4_layout(512)
    span = int(off[-1] + ln[-1])
    d4 = splitmix64_bytes(span, W.SEED + 2, 0)
    raw5, base5 = aligned_buffer(d4)
    out["cfg4"] = {"seed": W.SEED + 2, "count": 512, "len": ln.tolist(),
                   "crc": [ext(0, base5 + int(off[i]), int(ln[i])) for i in range(512)]}

    vals = [0, 1, 0xFFFFFFFF, 0x8A9136AA, ext_bytes(0, b"foo")] + [int(x) for x in rng.integers(0, 2**32, 27)]
    out["mask"] = [{"crc": v, "masked": int(r.ref_crc32c_mask(v)), "unmask_of_crc": int(r.ref_crc32c_unmask(v))}
                   for v in vals]

    path = os.path.join(os.path.dirname(__file__), "crc32c_golden.json")
    with open(path, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print(f"wrote {path} ({os.path.getsize(path)} bytes)")


if __name__ == "__main__":
    main()
