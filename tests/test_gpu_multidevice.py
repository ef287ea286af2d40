"""Multi-GPU paths on the one-GPU box, each checked against the reference's outputs:

  * the library's group C-ABI (kvsep_crc32c_group_*: one process, several contexts) over the device list [0, 0] --
    two independent contexts on the same GPU exercise the byte-balanced partition, the per-member host threads
    and staging, the merge into one result array and the first_bad / nbad reductions;
  * bench.py's multi-rank path: two torchrun ranks on cuda:0 (KVSEP_BENCH_SAME_DEVICE, gloo for the collectives,
    RCCL on a real multi-GPU node), config 5 -- the 512 GiB vlog as 8 distinct regenerated slices, 4 per rank --
    with the u32 results of both ranks all-gathered and EVERY record checked against the reference
    (tests/golden/full_cfg5.u32); and config 2 at two ranks.
"""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

import kvsep
from kvsep import splitmix64_bytes
from kvsep import workloads as W

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
DEV = torch.device("cuda:0")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def u64(a, dev=DEV):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(dev)


@pytest.fixture(scope="module")
def group():
    g = kvsep.Group([0, 0])
    yield g
    g.close()


def test_group_host_span_ragged_vs_oracle(group, oracle):
    rng = np.random.default_rng(11)
    ln = np.minimum(W.zipf_lengths(6000), 300_000).astype(np.uint64)
    off = np.zeros(ln.size, np.uint64)
    off[1:] = np.cumsum(ln[:-1] + np.uint64(3), dtype=np.uint64)  # 3-byte gaps: odd alignments
    buf = splitmix64_bytes(int(off[-1] + ln[-1]) + 64, 1717, 0)
    init = rng.integers(0, 2**32, ln.size, dtype=np.uint64).astype(np.uint32)
    exp = oracle.batch(buf, off, ln, init, threads=8)
    assert group.size() == 2
    assert np.array_equal(group.batch_host_span(buf, off, ln, init=init), exp)
    stored = np.array([kvsep.mask(int(c)) for c in exp], np.uint32)
    stored[[4500, 4501, 5999]] ^= 1  # in the second member's part
    out, fb, nb = group.batch_host_span(buf, off, ln, init=init, expected_masked=stored)
    assert np.array_equal(out, exp) and (fb, nb) == (4500, 3)
    stored[17] ^= 1  # and one in the first member's part: the global minimum wins
    assert group.batch_host_span(buf, off, ln, init=init, expected_masked=stored)[1:] == (17, 4)


def test_group_vlog_scan_like_gc(group, oracle):
    """A whole vlog image (config-5 records) scanned by the group, as GC would scan one vlog file
    (db/db_impl.cc:880-951 over db/value_log_reader.cc:86-138)."""
    off, ln = W.cfg3_layout(vlog=True, count=96)
    span = int(off[-1] + ln[-1])
    img = splitmix64_bytes(span, W.SEED + 1, 0)
    crc = np.fromfile(os.path.join(GOLDEN, "full_cfg5.u32"), dtype="<u4")[:96]  # the reference's CRCs
    for i in range(96):  # the stored headers a VlogWriter writes (db/value_log_writer.cc:57-60)
        h = int(off[i]) - 8
        img[h:h + 4] = np.frombuffer(kvsep.mask(int(crc[i])).to_bytes(4, "little"), np.uint8)
        img[h + 4:h + 8] = np.frombuffer(int(ln[i]).to_bytes(4, "little"), np.uint8)
    assert group.vlog_verify(img) == (96, 96, span, 0)
    img[int(off[70]) + 5] ^= 0x80
    assert group.vlog_verify(img) == (96, 70, int(off[69] + ln[69]), int(ln[70]))


def test_group_device_shards_vs_reference(group):
    """Device-resident shards of config 2 (the reference's full-batch CRCs): one shard per member."""
    off, ln = W.cfg2_layout()
    ref = np.fromfile(os.path.join(GOLDEN, "full_cfg2.u32"), dtype="<u4")
    data = torch.empty(int(ln.sum()) + 64, dtype=torch.uint8, device=DEV)
    kvsep.fill_splitmix64(data.data_ptr(), int(ln.sum()), W.SEED, 0)
    b = kvsep.partition(ln, 2)
    shards, outs, exps = [], [], []
    for i in range(2):
        lo, hi = int(b[i]), int(b[i + 1])
        o = torch.zeros(hi - lo, dtype=torch.int32, device=DEV)
        outs.append(o)
        shards.append({"base": data.data_ptr() + int(off[lo]), "off": u64(off[lo:hi] - off[lo]), "len": u64(ln[lo:hi]),
                       "out": o, "total_bytes": int(ln[lo:hi].sum()), "max_len": 4096})
        e = np.array([kvsep.mask(int(c)) for c in ref[lo:hi]], np.uint32)
        exps.append(e)
    group.batch_device(shards)
    got = np.concatenate([o.cpu().numpy().view(np.uint32) for o in outs])
    assert np.array_equal(got, ref)
    exps[1][100] ^= 4
    d_exps = [torch.from_numpy(e.view(np.int32)).to(DEV) for e in exps]
    fb, nb = group.batch_device(shards, expected_masked=d_exps, index_base=[int(b[0]), int(b[1])])
    assert (fb, nb) == (int(b[1]) + 100, 1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _torchrun_bench(nproc, *bench_args, timeout=900):
    env = dict(os.environ, KVSEP_BENCH_SAME_DEVICE="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={nproc}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(nproc), "--no-cpu", "--roundtrip-gib", "0", *bench_args]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def test_two_ranks_config5_all_records_vs_reference():
    line = _torchrun_bench(2, "--config", "5", "--steps", "1", "--warmup", "0")
    assert line["n_gpus"] == 2 and line["scaling"] == "strong"
    assert line["config"]["total_bytes"] == 524288 * W.VLOG_PAYLOAD
    p = line["parity"]
    assert p["blocks_checked_vs_reference"] == 524288 and p["mismatches"] == 0, p


def test_two_ranks_config2_gathered_results():
    line = _torchrun_bench(2, "--config", "2", "--steps", "4", "--warmup", "1")
    p = line["parity"]
    assert p["blocks_checked_vs_reference"] == 65536 and p["blocks_sampled_vs_oracle"] == 16
    assert p["mismatches"] == 0 and len(line["digests"]) == 2
