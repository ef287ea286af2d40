"""The batched framing entry points against files WRITTEN BY THE REFERENCE and verdicts of the REFERENCE READERS
(tests/golden/ref_framing.json, ref_manifest.log, ref_table.sst; tests/golden/make_framing_golden.py runs the
reference's own db/value_log_writer.cc, db/log_writer.cc, table/table_builder.cc and readers, compiled from
/root/reference):

  vlog   kvsep_vlog_frame_host reproduces the reference vlog byte for byte (SHA-256); kvsep_vlog_verify_host stops
         where VlogReader stops (db/value_log_reader.cc:86-138) and reports the same "checksum mismatch" bytes.
  log    kvsep_log_frame_host, fresh and reopened at dest_length, reproduces the reference MANIFEST log byte for
         byte; kvsep_log_walk + kvsep_log_verify_host + kvsep_log_accept, assembled into logical records as
         log::Reader::ReadRecord does (db/log_reader.cc:58-153), give the records the reference reader returned on
         every corrupted copy, and the bytes it reported as "checksum mismatch".
  SST    kvsep_sst_trailers_device gives the reference TableBuilder's trailer words (table/table_builder.cc:222-227);
         kvsep_sst_verify_device flags exactly the blocks the reference ReadBlock rejects (table/format.cc:99-108).
"""
import hashlib
import json
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
HERE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def gold():
    with open(os.path.join(HERE, "ref_framing.json")) as f:
        return json.load(f)


@pytest.fixture(scope="module")
def ctx():
    c = kvsep.Context(0)
    yield c
    c.close()


def fnv64(b: bytes) -> str:
    h = 0xCBF29CE484222325
    for x in b:
        h = ((h ^ x) * 0x100000001B3) & 0xFFFFFFFFFFFFFFFF
    return "%016x" % h


def payloads(seed, lens):
    data = splitmix64_bytes(int(sum(lens)) + 1, seed, 0)
    out, p = [], 0
    for n in lens:
        out.append(data[p:p + n].tobytes())
        p += n
    return out


def flipped(img: bytes, case) -> bytes:
    b = bytearray(img)
    if case.get("cut"):
        del b[case["cut"]:]
    else:
        b[case["flip"]] ^= 0x80
    return bytes(b)


def mismatch_bytes(drops):
    return sum(n for n, why in drops if why == "Corruption: checksum mismatch")


# ------------------------------------------------------------------ vlog
@pytest.fixture(scope="module")
def vlog_image(ctx, gold):
    v = gold["vlog"]
    img = ctx.vlog_frame(payloads(v["seed"], v["lens"]))
    return img


def test_vlog_frame_matches_reference_writer(vlog_image, gold):
    v = gold["vlog"]
    assert len(vlog_image) == v["size"]
    assert hashlib.sha256(vlog_image).hexdigest() == gold["sha256"]["vlog.bin"]
    p = 0
    for n, h in zip(v["lens"], v["headers"]):
        assert vlog_image[p:p + 8].hex() == h
        p += 8 + n


@pytest.mark.parametrize("name", ["intact", "payload_r11", "crc_r3", "len_r9", "torn_tail"])
def test_vlog_verify_matches_reference_reader(ctx, vlog_image, gold, name):
    v = gold["vlog"]
    if name == "intact":
        img, reader = vlog_image, v["intact"]
    else:
        case = next(c for c in v["cases"] if c["name"] == name)
        img, reader = flipped(vlog_image, case), case["reader"]
    n, good, good_bytes, drop = ctx.vlog_verify(img, with_drop=True)
    assert good == len(reader["records"])
    assert drop == mismatch_bytes(reader["drops"])
    off, ln, _, _ = kvsep.vlog_walk(img)
    got = [[int(ln[i]) + 8, fnv64(img[int(off[i]) - 8:int(off[i] + ln[i])])] for i in range(good)]
    assert got == reader["records"]  # header + payload, as VlogReader::ReadRecord returns them


# ------------------------------------------------------------------ log / MANIFEST
@pytest.fixture(scope="module")
def manifest():
    with open(os.path.join(HERE, "ref_manifest.log"), "rb") as f:
        return f.read()


def test_log_frame_matches_reference_writer(ctx, gold, manifest):
    lg = gold["log"]
    pl = payloads(lg["seed"], lg["lens"])
    first = [p for p, w in zip(pl, lg["writer"]) if w == 0]
    second = [p for p, w in zip(pl, lg["writer"]) if w == 1]
    a = ctx.log_frame(first, dest_length=0)
    assert len(a) == lg["reopen_at"]
    b = ctx.log_frame(second, dest_length=len(a))  # log::Writer(dest, dest_length), db/log_writer.cc:25-28
    assert a + b == manifest
    assert hashlib.sha256(a + b).hexdigest() == gold["sha256"]["manifest.log"]


def assemble(img, off, ln, ty, accept):
    """log::Reader::ReadRecord (db/log_reader.cc:58-153) over the physical records: FULL returns, FIRST/MIDDLE/LAST
    assemble, a dropped record (kBadRecord) abandons a record in progress."""
    out, scratch, infrag = [], b"", False
    for o, n, t, a in zip(off, ln, ty, accept):
        frag = img[int(o) + 1:int(o) + int(n)]  # off points at the type byte, len = 1 + payload
        if not a:
            infrag, scratch = False, b""
        elif t == 1:
            infrag, scratch = False, b""
            out.append(frag)
        elif t == 2:
            scratch, infrag = frag, True
        elif t == 3:
            if infrag:
                scratch += frag
        elif t == 4:
            if infrag:
                out.append(scratch + frag)
                infrag, scratch = False, b""
    return [[len(r), fnv64(r)] for r in out]


@pytest.mark.parametrize("name", ["intact", "full_payload", "first_payload", "middle_payload", "last_payload",
                                  "type_byte", "length_field", "crc_after_reopen"])
def test_log_verify_matches_reference_reader(ctx, gold, manifest, name):
    lg = gold["log"]
    if name == "intact":
        img, reader = manifest, lg["intact"]
    else:
        case = next(c for c in lg["cases"] if c["name"] == name)
        img, reader = flipped(manifest, case), case["reader"]
    off, ln, _, ty = kvsep.log_walk(img)
    if name == "intact":
        assert off.size == lg["physical_records"]
    ok = ctx.log_verify(img)
    accept, dropped = kvsep.log_accept(off, ok, len(img))
    assert dropped == mismatch_bytes(reader["drops"])
    assert assemble(img, off, ln, ty, accept) == reader["records"]


# ------------------------------------------------------------------ SST
@pytest.fixture(scope="module")
def sst():
    with open(os.path.join(HERE, "ref_table.sst"), "rb") as f:
        return f.read()


def dev_u64(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(DEV)


def test_sst_trailers_match_reference_builder(ctx, gold, sst):
    blocks = gold["sst"]["blocks"]
    off = np.array([b[0] for b in blocks], np.uint64)
    ln = np.array([b[1] for b in blocks], np.uint64)
    types = torch.tensor([b[2] for b in blocks], dtype=torch.uint8, device=DEV)
    d = torch.frombuffer(bytearray(sst), dtype=torch.uint8).to(DEV)
    masked = torch.zeros(len(blocks), dtype=torch.int32, device=DEV)
    ctx.sst_trailers_device(d.data_ptr(), dev_u64(off), dev_u64(ln), types, masked, max_len=int(ln.max()))
    torch.cuda.synchronize()
    got = ["%08x" % x for x in masked.cpu().numpy().view(np.uint32)]
    want = ["%08x" % int.from_bytes(bytes.fromhex(b[3]), "little") for b in blocks]
    assert got == want


@pytest.mark.parametrize("name", ["intact", "data_block_5", "trailer_crc_9", "type_byte_2", "last_block"])
def test_sst_verify_matches_reference_readblock(ctx, gold, sst, name):
    s = gold["sst"]
    if name == "intact":
        img, ok_ref = sst, s["intact_ok"]
    else:
        case = next(c for c in s["cases"] if c["name"] == name)
        img, ok_ref = flipped(sst, case), case["ok"]
    blocks = s["blocks"]
    off = np.array([b[0] for b in blocks], np.uint64)
    ln = np.array([b[1] for b in blocks], np.uint64)
    d = torch.frombuffer(bytearray(img), dtype=torch.uint8).to(DEV)
    out = torch.zeros(len(blocks), dtype=torch.int32, device=DEV)
    fb = torch.zeros(1, dtype=torch.int64, device=DEV)
    nb = torch.zeros(1, dtype=torch.int64, device=DEV)
    ctx.sst_verify_device(d.data_ptr(), dev_u64(off), dev_u64(ln), out, fb, nb, max_len=int(ln.max()))
    torch.cuda.synchronize()
    bad_ref = [i for i, k in enumerate(ok_ref) if not k]
    assert nb.item() == len(bad_ref)
    assert fb.item() == (bad_ref[0] if bad_ref else -1)
    crc = out.cpu().numpy().view(np.uint32)
    stored = [int.from_bytes(img[int(o + n + 1):int(o + n + 5)], "little") for o, n in zip(off, ln)]
    ours = [1 if kvsep.mask(int(c)) == w else 0 for c, w in zip(crc, stored)]
    assert ours == ok_ref


def test_sst_trailers_host_match_reference_builder(ctx, gold, sst):
    # the host-resident form (kvsep_sst_trailers_host): blocks as TableBuilder::WriteRawBlock holds them, in host
    # memory (table/table_builder.cc:209-232), one pointer per block
    blocks = gold["sst"]["blocks"]
    img = bytes(sst)
    views = [img[b[0]:b[0] + b[1]] for b in blocks]
    got = ["%08x" % x for x in ctx.sst_trailers(views, [b[2] for b in blocks])]
    want = ["%08x" % int.from_bytes(bytes.fromhex(b[3]), "little") for b in blocks]
    assert got == want


@pytest.mark.parametrize("name", ["intact", "data_block_5", "trailer_crc_9", "type_byte_2", "last_block"])
def test_sst_verify_host_matches_reference_readblock(ctx, gold, sst, name):
    # the host-resident read check (kvsep_sst_verify_host) over a host SST file image, as ReadBlock reads it
    # (table/format.cc:73-108): first_bad / nbad and the per-block verdicts equal the reference reader's
    s = gold["sst"]
    if name == "intact":
        img, ok_ref = sst, s["intact_ok"]
    else:
        case = next(c for c in s["cases"] if c["name"] == name)
        img, ok_ref = flipped(sst, case), case["ok"]
    blocks = s["blocks"]
    off = np.array([b[0] for b in blocks], np.uint64)
    ln = np.array([b[1] for b in blocks], np.uint64)
    out, fb, nb = ctx.sst_verify(bytes(img), off, ln)
    bad_ref = [i for i, k in enumerate(ok_ref) if not k]
    assert nb == len(bad_ref)
    assert fb == (bad_ref[0] if bad_ref else -1)
    stored = [int.from_bytes(img[int(o + n + 1):int(o + n + 5)], "little") for o, n in zip(off, ln)]
    assert [1 if kvsep.mask(int(c)) == w else 0 for c, w in zip(out, stored)] == ok_ref


def test_sst_host_forms_reject_short_handles(ctx, gold, sst):
    # a handle whose 5-byte trailer would run past the file is refused (format.cc:84-87 "truncated block read")
    blocks = gold["sst"]["blocks"]
    o, n = blocks[-1][0], blocks[-1][1]
    with pytest.raises(kvsep.KvsepError):
        ctx.sst_verify(bytes(sst)[:o + n + 4], np.array([o], np.uint64), np.array([n], np.uint64))


def test_sst_host_forms_large_batch_match_oracle(ctx, oracle):
    # many 4 KiB-ish blocks (config-2-shaped, ragged) in one host file image, planted bad trailers: the verdicts equal
    # the oracle's recompute, and trailers built by the host trailer form verify clean
    rng = np.random.default_rng(7)
    k = 20000
    ln = rng.integers(1, 8192, k).astype(np.uint64)
    types = rng.integers(0, 2, k).astype(np.uint8)
    off = np.zeros(k, np.uint64)
    off[1:] = np.cumsum(ln[:-1] + 5, dtype=np.uint64)
    n = int(off[-1] + ln[-1] + 5)
    img = bytearray(kvsep.splitmix64_bytes(n, 99, 0).tobytes())
    views = [bytes(img[int(o):int(o + l)]) for o, l in zip(off, ln)]
    words = ctx.sst_trailers(views, types)
    for i in range(k):
        o, l = int(off[i]), int(ln[i])
        img[o + l] = int(types[i])
        img[o + l + 1:o + l + 5] = int(words[i]).to_bytes(4, "little")
    for i in (3, 1777, 19999):  # oracle check of the trailer word itself
        o, l = int(off[i]), int(ln[i])
        assert kvsep.mask(oracle.extend(0, bytes(img[o:o + l + 1]))) == int(words[i])
    out, fb, nb = ctx.sst_verify(bytes(img), off, ln)
    assert (fb, nb) == (-1, 0)
    bad = [5, 4096, 12345]
    for i in bad:
        img[int(off[i]) + 7 % int(ln[i])] ^= 0x20
    out, fb, nb = ctx.sst_verify(bytes(img), off, ln)
    assert (fb, nb) == (bad[0], len(bad))
