"""GPU: the batched framing entry points against independently framed images (oracle checksums)."""
import numpy as np
import pytest

import kvsep
from kvsep import splitmix64_bytes
from framing_builders import log_image, sst_image, vlog_image

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def ctx():
    c = kvsep.Context(0)
    yield c
    c.close()


def _payloads(n, seed, maxlen, minlen=0):
    rng = np.random.default_rng(seed)
    lens = rng.integers(minlen, maxlen, n)
    data = splitmix64_bytes(int(lens.sum()) + 1, seed, 0)
    out, p = [], 0
    for l in lens:
        out.append(data[p:p + l].tobytes())
        p += l
    return out


def test_vlog_recovery_scan(ctx, oracle):
    pl = _payloads(300, 11, 300000) + [b"", bytes(1048609)]
    img = vlog_image(pl, oracle)
    n, good, gb = ctx.vlog_verify(img)
    assert n == good == len(pl) and gb == len(img)
    bad = bytearray(img)
    off, ln, _, _ = kvsep.vlog_walk(img)
    bad[int(off[123]) + int(ln[123]) // 2] ^= 0x80        # corruption_test.cc-style flip in record 123
    n, good, gb, drop = ctx.vlog_verify(bytes(bad), with_drop=True)
    assert (n, good) == (len(pl), 123) and gb == int(off[122] + ln[122])
    assert drop == int(ln[123])  # VlogReader's drop_size for "checksum mismatch" (db/value_log_reader.cc:117-120)
    assert ctx.vlog_verify(img, with_drop=True)[3] == 0
    n, good, gb = ctx.vlog_verify(img[:-5])              # torn tail: the last record is eof, not corrupt
    assert n == good == len(pl) - 1


def test_vlog_group_commit_framing(ctx, oracle):
    pl = _payloads(500, 12, 70000) + [b""]
    ref = vlog_image(pl, oracle)
    assert ctx.vlog_frame(pl) == ref
    out = np.full(len(ref) + 100, 0xEE, dtype=np.uint8)  # into a caller buffer; nothing past the image touched
    assert ctx.vlog_frame(pl, out=out) == len(ref)
    assert out[:len(ref)].tobytes() == ref and (out[len(ref):] == 0xEE).all()


def test_log_manifest_verify(ctx, oracle):
    recs = _payloads(60, 13, 100000)
    img, phys = log_image(recs, oracle)
    ok = ctx.log_verify(img)
    assert ok.size == len(phys) and ok.all()
    bad = bytearray(img)
    h = phys[17][0]
    bad[h + 7] ^= 1                                      # payload byte of physical record 17
    ok = ctx.log_verify(bytes(bad))
    assert not ok[17] and ok.sum() == len(phys) - 1
    # what log::Reader returns: record 17 and the rest of its 32 KiB block are dropped (db/log_reader.cc:250-258)
    off = kvsep.log_walk(bytes(bad))[0]
    acc, dropped = kvsep.log_accept(off, ok, len(bad))
    blk = (off - 6) // 32768
    same = blk == blk[17]
    assert not acc[same & (np.arange(off.size) >= 17)].any() and acc[~same | (np.arange(off.size) < 17)].all()
    assert dropped == min(int(blk[17] + 1) * 32768, len(bad)) - h


def test_log_manifest_write_side(ctx, oracle):
    """log::Writer::AddRecord batched: identical bytes to an independently framed image, also when appending to
    a log that already ends mid-block (block_offset_ = dest_length % 32 KiB) and with trailers < 7 bytes."""
    recs = _payloads(70, 15, 90000) + [b"", b"x" * 32761, b"y" * 32755, b"z" * 40000]
    img, _ = log_image(recs, oracle)
    assert ctx.log_frame(recs) == img
    head, _ = log_image(recs[:23], oracle)
    assert head + ctx.log_frame(recs[23:], dest_length=len(head)) == img
    assert (ctx.log_verify(img) == 1).all()
    out = np.full(len(img) + 50, 0xEE, dtype=np.uint8)  # a dirty caller buffer: trailers must come out zero
    assert ctx.log_frame(recs, out=out) == len(img)
    assert out[:len(img)].tobytes() == img and (out[len(img):] == 0xEE).all()


def test_sst_trailers_and_verify(ctx, oracle):
    blocks = _payloads(2000, 14, 8192, minlen=1)
    types = np.random.default_rng(1).integers(0, 2, len(blocks)).astype(np.uint8)  # kNoCompression / kSnappy
    img, offs, words = sst_image(blocks, types, oracle)
    d = torch.zeros(len(img) + 64, dtype=torch.uint8, device=DEV)
    d[:len(img)] = torch.frombuffer(bytearray(img), dtype=torch.uint8).to(DEV)
    lens = np.array([len(b) for b in blocks], np.uint64)
    d_off = torch.from_numpy(offs.view(np.int64)).to(DEV)
    d_len = torch.from_numpy(lens.view(np.int64)).to(DEV)
    # write side: trailer words computed from the blocks (type bytes passed separately)
    masked = torch.zeros(len(blocks), dtype=torch.int32, device=DEV)
    ctx.sst_trailers_device(d.data_ptr(), d_off, d_len, torch.from_numpy(types).to(DEV), masked)
    torch.cuda.synchronize()
    assert np.array_equal(masked.cpu().numpy().view(np.uint32), words)
    # read side (table/format.cc:99-106)
    out = torch.zeros(len(blocks), dtype=torch.int32, device=DEV)
    fb = torch.zeros(1, dtype=torch.int64, device=DEV)
    nb = torch.zeros(1, dtype=torch.int64, device=DEV)
    ctx.sst_verify_device(d.data_ptr(), d_off, d_len, out, fb, nb)
    torch.cuda.synchronize()
    assert fb.item() == -1 and nb.item() == 0
    assert np.array_equal(out.cpu().numpy().view(np.uint32), [kvsep.unmask(int(w)) for w in words])
    d[int(offs[1500]) + 3] ^= 0x80
    d[int(offs[1700]) + int(lens[1700]) + 2] ^= 0x01     # damage a stored trailer word
    ctx.sst_verify_device(d.data_ptr(), d_off, d_len, out, fb, nb)
    torch.cuda.synchronize()
    assert fb.item() == 1500 and nb.item() == 2
