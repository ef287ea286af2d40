#!/usr/bin/env python3
"""Throughput of the four framing call sites on one MI355X, each checked against
the oracle on the same bytes.  Prints one JSON object per row and, with --out, writes them as a JSON list.

  vlog_verify   db/value_log_reader.cc:86-138  recovery / GC scan of a whole pageable vlog image:
                host header walk + one batched GPU checksum + compare (PCIe-inclusive)
  vlog_frame    db/value_log_writer.cc:46-76   group-commit framing of pageable payloads (PCIe-inclusive)
  log_frame     db/log_writer.cc:35-115        WAL/MANIFEST AddRecord fragmenting + one batched checksum
  log_verify    db/log_reader.cc:189-272       walk of the 32 KiB-block framing + batched verify
  sst_trailers  table/table_builder.cc:209-232 trailer words of device-resident 4 KiB blocks (kernel time)
  sst_verify    table/format.cc:99-108         read check of a device-resident file image (kernel time)

usage: python framing_bench.py [--vlog-gib 4] [--log-gib 1] [--out profiles/round1/framing_bench.json]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "..", "tests"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import kvsep  # noqa: E402
from kvsep import workloads as W  # noqa: E402

GIB = float(1 << 30)
DEV = torch.device("cuda:0")


def load_oracle():
    from conftest import load_oracle as _lo  # test infrastructure: the checker only
    return _lo()


def host_random(nbytes, seed):
    """Random bytes made on the device (fast), copied to pageable host memory."""
    t = torch.empty(nbytes + 16, dtype=torch.uint8, device=DEV)
    kvsep.fill_splitmix64(t.data_ptr(), t.numel(), seed, 0)
    torch.cuda.synchronize()
    return t.cpu().numpy()[:nbytes]


def timed(fn, reps):
    fn()  # warm (first-pass effects, pinned slot allocation)
    best = float("inf")
    for _ in range(reps):
        t0 = time.perf_counter()
        r = fn()
        best = min(best, time.perf_counter() - t0)
    return best, r


def row(name, ref, nbytes, seconds, parity, note):
    r = {"row": name, "reference": ref, "bytes": int(nbytes), "seconds": round(seconds, 6),
         "GiBps": round(nbytes / GIB / seconds, 3), "parity": bool(parity), "note": note}
    print(json.dumps(r), flush=True)
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--vlog-gib", type=float, default=4.0)
    ap.add_argument("--log-gib", type=float, default=1.0)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--out", default=None)
    ap.add_argument("--lib", default=None, help="another build of libkvsep_crc32c.so (A/B runs)")
    args = ap.parse_args()
    if args.lib:
        kvsep.LIB_PATH, kvsep._lib = args.lib, None
    oracle = load_oracle()
    ctx = kvsep.Context(0)
    rows = []
    rng = np.random.default_rng(7)

    # ---- vlog: group-commit framing (write side) then the recovery scan (read side) of the same image
    plen = W.VLOG_PAYLOAD
    k = max(2, int(args.vlog_gib * GIB) // (plen + 8))
    src = host_random(k * plen, 101)
    addrs = src.ctypes.data + np.arange(k, dtype=np.uint64) * np.uint64(plen)
    plens = np.full(k, plen, dtype=np.uint64)
    img = np.empty(k * (plen + 8), dtype=np.uint8)  # the writer's output buffer (touched by the warm rep)
    dt, wrote = timed(lambda: ctx.frame_raw("vlog", addrs, plens, img), args.reps)
    pick = rng.choice(k, 16, replace=False)
    ok = all(int.from_bytes(img[i * (plen + 8):i * (plen + 8) + 4].tobytes(), "little") ==
             oracle.lib.oracle_crc32c_mask(oracle.extend(0, src[i * plen:(i + 1) * plen])) for i in pick)
    rows.append(row("vlog_frame", "db/value_log_writer.cc:46-76", k * plen, dt, ok and wrote == img.size,
                    f"{k} pageable payloads of {plen} B (config 3b records) framed into a caller buffer (the C-ABI call on "
                    "prebuilt pointer arrays): gather through the copier pool, H2D, batched kernel, D2H of the CRCs, "
                    "headers, parallel payload copy into the image"))
    dt, (n, good, gb) = timed(lambda: ctx.vlog_verify(img), args.reps)
    bad = img.copy()
    flip = int(k // 2)
    bad[flip * (plen + 8) + 8 + plen // 3] ^= 0x40
    n2, good2, _ = ctx.vlog_verify(bad)
    rows.append(row("vlog_verify", "db/value_log_reader.cc:86-138", img.size, dt,
                    n == good == k and gb == img.size and (n2, good2) == (k, flip),
                    f"pageable {img.size / GIB:.2f} GiB vlog image: header walk + batched GPU checksum + compare; "
                    f"parity: all {k} good, a flipped byte in record {flip} stops the scan there"))
    del src, img, bad

    # ---- WAL / MANIFEST: AddRecord framing, then the reader's walk + verify of the result
    lens = rng.integers(100, 65536, max(1, int(args.log_gib * GIB) // 32868))
    src = host_random(int(lens.sum()), 202)
    starts = np.concatenate([[0], np.cumsum(lens)[:-1]])
    addrs = src.ctypes.data + starts.astype(np.uint64)
    img = np.empty(int(lens.sum()) + 7 * (int(lens.sum()) // 32761 + 2 * lens.size) + 64, dtype=np.uint8)
    dt, wrote = timed(lambda: ctx.frame_raw("log", addrs, lens, img), args.reps)
    img = img[:wrote]
    off, ln, stored, types = kvsep.log_walk(img)
    pick = rng.choice(off.size, 32, replace=False)
    tcrc = {t: oracle.extend(0, bytes([t])) for t in (1, 2, 3, 4)}
    ok = all(int(stored[i]) == oracle.lib.oracle_crc32c_mask(
        oracle.extend(tcrc[int(types[i])], img[int(off[i]) + 1:int(off[i] + ln[i])])) for i in pick)
    rows.append(row("log_frame", "db/log_writer.cc:35-115", int(lens.sum()), dt, ok and off.size > 0,
                    f"{lens.size} records of U[100, 65536) B ({lens.sum() / GIB:.2f} GiB) appended to an empty log: "
                    f"{off.size} physical records over 32 KiB blocks, one batched checksum"))
    dt, okv = timed(lambda: ctx.log_verify(img), args.reps)
    rows.append(row("log_verify", "db/log_reader.cc:189-272", img.size, dt, okv.size == off.size and okv.all(),
                    f"{img.size / GIB:.2f} GiB log image: walk of the block framing + batched verify of "
                    f"{off.size} physical records"))
    del src, img

    # ---- SST trailers and the read check, device-resident (config 2 geometry: 65,536 x 4 KiB blocks)
    count, blen = 65536, 4096
    file_stride = blen + 5
    span = count * file_stride
    fimg = torch.empty(span + 64, dtype=torch.uint8, device=DEV)
    kvsep.fill_splitmix64(fimg.data_ptr(), fimg.numel(), 303, 0)
    off = np.arange(count, dtype=np.uint64) * np.uint64(file_stride)
    lens = np.full(count, blen, dtype=np.uint64)
    d_off = torch.from_numpy(off.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lens.view(np.int64)).to(DEV)
    types = torch.from_numpy(rng.integers(0, 2, count).astype(np.uint8)).to(DEV)
    masked = torch.zeros(count, dtype=torch.int32, device=DEV)
    ctx.reserve(count, count * blen)

    def kernel_time(fn, reps=20):
        fn()
        torch.cuda.synchronize()
        ctx.get_timing()
        ctx.set_timing(True)
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        ctx.set_timing(False)
        ms, nl = ctx.get_timing()
        return ms * 1e-3 / max(1, nl)

    trail = lambda: ctx.sst_trailers_device(fimg.data_ptr(), d_off, d_len, types, masked,  # noqa: E731
                                            total_bytes=count * blen, max_len=blen)
    dt = kernel_time(trail)
    torch.cuda.synchronize()
    host_img = fimg.cpu().numpy()
    mk = masked.cpu().numpy().view(np.uint32)
    ty = types.cpu().numpy()
    pick = rng.choice(count, 32, replace=False)
    ok = all(int(mk[i]) == oracle.lib.oracle_crc32c_mask(
        oracle.extend(oracle.extend(0, host_img[int(off[i]):int(off[i]) + blen]), bytes([int(ty[i])])))
        for i in pick)
    rows.append(row("sst_trailers", "table/table_builder.cc:209-232", count * blen, dt, ok,
                    f"{count} x {blen} B device-resident blocks -> Mask(Extend(Value(block), type)); kernel time by "
                    "HIP events (the ~5 us event floor is inside a 50 us batch)"))
    # write the trailers into the image ([type][masked LE32] after each block), then the read check
    t8 = fimg[:span].view(count, file_stride)
    t8[:, blen] = types
    t8[:, blen + 1:blen + 5] = masked.view(torch.uint8).view(count, 4)
    out = torch.zeros(count, dtype=torch.int32, device=DEV)
    first_bad = torch.zeros(1, dtype=torch.int64, device=DEV)
    nbad = torch.zeros(1, dtype=torch.int64, device=DEV)
    ver = lambda: ctx.sst_verify_device(fimg.data_ptr(), d_off, d_len, out, first_bad, nbad,  # noqa: E731
                                        total_bytes=count * (blen + 1), max_len=blen + 1)
    dt = kernel_time(ver)
    torch.cuda.synchronize()
    clean = int(nbad.item()) == 0
    t8[count // 3, 100] ^= 1
    ver()
    torch.cuda.synchronize()
    caught = int(nbad.item()) == 1 and int(first_bad.item()) == count // 3
    rows.append(row("sst_verify", "table/format.cc:99-108", count * (blen + 1), dt, clean and caught,
                    f"{count} blocks + type bytes of a device-resident file image: Value(block, n+1) vs Unmask(stored); "
                    f"parity: clean image passes, one flipped bit is reported at block {count // 3}"))

    # ---- the same two call sites for host-resident blocks (kvsep_sst_trailers_host / kvsep_sst_verify_host): the way
    # TableBuilder::WriteRawBlock and ReadBlock hold them, through the pinned staging pipeline (PCIe-inclusive)
    t8[count // 3, 100] ^= 1  # intact again
    ver()
    torch.cuda.synchronize()
    dout = out.cpu().numpy().view(np.uint32).copy()  # the device form's words on the intact image
    himg = fimg[:span].cpu().numpy()  # pageable host copy of the file image (blocks + trailers)
    addrs = np.uint64(himg.ctypes.data) + off  # the blocks where TableBuilder holds them: prebuilt pointers
    hty = ty.copy()
    words = np.zeros(count, np.uint32)
    dt, _ = timed(lambda: ctx.sst_trailers_raw(addrs, lens, hty, words), 3)
    okh = np.array_equal(words, mk)
    views = [memoryview(himg)[int(o):int(o) + blen] for o in off[:64]]  # the per-block Python form agrees too
    okh = okh and np.array_equal(ctx.sst_trailers(views, hty[:64]), mk[:64])
    rows.append(row("sst_trailers_host", "table/table_builder.cc:209-232", count * blen, dt, okh,
                    f"{count} x {blen} B pageable host blocks (one pointer per block) -> trailer words, H2D + kernel + "
                    "D2H; parity: equal to the device form's words"))
    res = None

    def hver():
        nonlocal res
        res = ctx.sst_verify(himg, off, lens)

    dt, _ = timed(hver, 3)
    hout, hfb, hnb = res
    okv = hfb == -1 and hnb == 0 and np.array_equal(hout, dout)
    himg[int(off[count // 5]) + 7] ^= 4
    _, hfb2, hnb2 = ctx.sst_verify(himg, off, lens)
    okv = okv and hfb2 == count // 5 and hnb2 == 1
    rows.append(row("sst_verify_host", "table/format.cc:73-108", count * (blen + 1), dt, okv,
                    f"a pageable {span >> 20} MiB host file image with {count} block handles -> Value(block, n+1) vs "
                    f"Unmask(stored), H2D + kernel + D2H; parity: clean image passes with the device form's words, one "
                    f"flipped bit is reported at block {count // 5}"))
    ctx.close()
    if args.out:
        with open(args.out, "w") as f:
            json.dump(rows, f, indent=1)
    if not all(r["parity"] for r in rows):
        sys.exit(1)


if __name__ == "__main__":
    main()
