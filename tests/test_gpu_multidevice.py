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
    ref = np.fromfile(os.path.join(GOLDEN, "full_cfg2.u32"), dtype="<u4")[:W.CFG2_BLOCKS]
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


@pytest.fixture(scope="module")
def group8():
    # eight members: the 8-way byte-balanced partition, eight member host threads / staging
    # pipelines / streams, and the first_bad / nbad reduction over eight parts -- on the one-GPU box as eight
    # independent contexts on device 0
    g = kvsep.Group([0] * 8)
    yield g
    g.close()


def test_group8_vlog_scan_bad_record_in_last_member(group8):
    """A config-5 vlog slice image (the reference's CRCs as the stored headers, db/value_log_writer.cc:57-60) scanned
    by the 8-member group as GC / recovery scan a whole vlog (db/db_impl.cc:880-951 / :485-571), then with one bad
    record inside the last member's range: the reader verdict (records kept, bytes dropped) is the reference reader's."""
    n = 160
    off, ln = W.cfg3_layout(vlog=True, count=n)
    span = int(off[-1] + ln[-1])
    img = splitmix64_bytes(span, W.SEED + 1, 0)
    crc = np.fromfile(os.path.join(GOLDEN, "full_cfg5.u32"), dtype="<u4")[:n]
    for i in range(n):
        h = int(off[i]) - 8
        img[h:h + 4] = np.frombuffer(kvsep.mask(int(crc[i])).to_bytes(4, "little"), np.uint8)
        img[h + 4:h + 8] = np.frombuffer(int(ln[i]).to_bytes(4, "little"), np.uint8)
    assert group8.size() == 8
    assert group8.vlog_verify(img) == (n, n, span, 0)
    b = kvsep.partition(ln, 8)
    bad = int(b[7]) + 3  # inside member 7's part
    assert bad < n
    img[int(off[bad]) + 1000] ^= 0x01
    assert group8.vlog_verify(img) == (n, bad, int(off[bad - 1] + ln[bad - 1]), int(ln[bad]))


def test_group8_device_shards_index_base_vs_reference(group8):
    """All of config 2 (the reference's whole-batch CRCs) as eight device shards with index_base: results, and the
    global first_bad / nbad of stored words corrupted in members 2, 5 and 7."""
    off, ln = W.cfg2_layout()
    ref = np.fromfile(os.path.join(GOLDEN, "full_cfg2.u32"), dtype="<u4")[:W.CFG2_BLOCKS]
    data = torch.empty(int(ln.sum()) + 64, dtype=torch.uint8, device=DEV)
    kvsep.fill_splitmix64(data.data_ptr(), int(ln.sum()), W.SEED, 0)
    b = kvsep.partition(ln, 8)
    assert all(int(b[i + 1]) - int(b[i]) == 8192 for i in range(8))  # equal lengths: an exact byte split
    shards, outs, exps = [], [], []
    for i in range(8):
        lo, hi = int(b[i]), int(b[i + 1])
        o = torch.zeros(hi - lo, dtype=torch.int32, device=DEV)
        outs.append(o)
        shards.append({"base": data.data_ptr() + int(off[lo]), "off": u64(off[lo:hi] - off[lo]), "len": u64(ln[lo:hi]),
                       "out": o, "total_bytes": int(ln[lo:hi].sum()), "max_len": 4096})
        exps.append(np.array([kvsep.mask(int(c)) for c in ref[lo:hi]], np.uint32))
    group8.batch_device(shards)
    assert np.array_equal(np.concatenate([o.cpu().numpy().view(np.uint32) for o in outs]), ref)
    ib = [int(b[i]) for i in range(8)]
    d_exps = [torch.from_numpy(e.view(np.int32)).to(DEV) for e in exps]
    assert group8.batch_device(shards, expected_masked=d_exps, index_base=ib) == (~0 & (2**64 - 1), 0)
    for m, k in ((7, 8191), (5, 17), (2, 4000)):
        exps[m][k] ^= 0x100
    d_exps = [torch.from_numpy(e.view(np.int32)).to(DEV) for e in exps]
    assert group8.batch_device(shards, expected_masked=d_exps, index_base=ib) == (ib[2] + 4000, 3)


def test_group8_ragged_host_span_with_init_vs_oracle(group8, oracle):
    """A ragged config-4-shaped host batch (Zipf lengths, capped so the test stays small) with per-block init words,
    odd alignments: the 8-way partition by bytes, results and the verify reduction against the oracle."""
    rng = np.random.default_rng(88)
    ln = np.minimum(W.zipf_lengths(12000), 400_000).astype(np.uint64)
    off = np.zeros(ln.size, np.uint64)
    off[1:] = np.cumsum(ln[:-1] + np.uint64(5), dtype=np.uint64)
    buf = splitmix64_bytes(int(off[-1] + ln[-1]) + 64, 8888, 0)
    init = rng.integers(0, 2**32, ln.size, dtype=np.uint64).astype(np.uint32)
    exp = oracle.batch(buf, off, ln, init, threads=8)
    assert np.array_equal(group8.batch_host_span(buf, off, ln, init=init), exp)
    b = kvsep.partition(ln, 8)
    share = [int(ln[int(b[i]):int(b[i + 1])].sum()) for i in range(8)]
    assert max(share) - min(share) <= 2 * int(ln.max())  # within a block or two of its byte share
    stored = np.array([kvsep.mask(int(c)) for c in exp], np.uint32)
    out, fb, nb = group8.batch_host_span(buf, off, ln, init=init, expected_masked=stored)
    assert np.array_equal(out, exp) and (fb, nb) == (2**64 - 1, 0)
    plant = [int(b[7]) + 1, int(b[3]) + 2, int(b[3]) + 3]
    stored[plant] ^= 0x8
    assert group8.batch_host_span(buf, off, ln, init=init, expected_masked=stored)[1:] == (min(plant), 3)


@pytest.mark.skipif(torch.cuda.device_count() < 2, reason="needs two GPUs (ADVICE r2: distinct-device group path)")
def test_group_distinct_devices_vs_reference(oracle):
    """The group over distinct devices: per-member DeviceGuard switching, scratch on each member's device, member
    streams on different devices.  Runs only where two or more GPUs are visible (not on the one-GPU box)."""
    ndev = min(torch.cuda.device_count(), 8)
    g = kvsep.Group(list(range(ndev)))
    try:
        rng = np.random.default_rng(5)
        ln = rng.integers(0, 200_000, 3000).astype(np.uint64)
        off = np.zeros(ln.size, np.uint64)
        off[1:] = np.cumsum(ln[:-1], dtype=np.uint64)
        buf = splitmix64_bytes(int(off[-1] + ln[-1]) + 64, 5150, 0)
        exp = oracle.batch(buf, off, ln, None, threads=8)
        assert np.array_equal(g.batch_host_span(buf, off, ln), exp)
        b = kvsep.partition(ln, ndev)
        shards, outs = [], []
        for i in range(ndev):
            lo, hi = int(b[i]), int(b[i + 1])
            dv = torch.device("cuda", i)
            d = torch.from_numpy(buf[int(off[lo]):int(off[hi - 1] + ln[hi - 1])].copy()).to(dv)
            o = torch.zeros(hi - lo, dtype=torch.int32, device=dv)
            outs.append(o)
            shards.append({"base": d, "off": u64(off[lo:hi] - off[lo], dv), "len": u64(ln[lo:hi], dv), "out": o,
                           "total_bytes": int(ln[lo:hi].sum()), "max_len": int(ln[lo:hi].max())})
        g.batch_device(shards)
        assert np.array_equal(np.concatenate([o.cpu().numpy().view(np.uint32) for o in outs]), exp)
    finally:
        g.close()


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
    assert p["blocks_checked_vs_reference"] == 2 * 65536 and p["blocks_sampled_vs_oracle"] == 0
    assert p["every_block_checked"] and p["mismatches"] == 0 and len(line["digests"]) == 2


def test_bench_self_launch_two_ranks_config2():
    """`python3 bench.py --gpus 2` with no launcher: bench.py starts both ranks itself (here both
    on cuda:0 with gloo for the results, KVSEP_BENCH_SAME_DEVICE), and the line says n_gpus 2 / world_size 2 with every
    block of the global batch checked against the reference."""
    env = dict(os.environ, KVSEP_BENCH_SAME_DEVICE="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--config", "2", "--steps", "3", "--warmup",
           "1", "--no-cpu", "--roundtrip-gib", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2 and line["world_size"] == 2 and line["backend"] == "gloo", line
    p = line["parity"]
    assert p["blocks_checked_vs_reference"] == 2 * 65536 and p["mismatches"] == 0, p


def test_bench_self_launch_eight_ranks_config2_every_block():
    """`python3 bench.py --gpus 8 --config 2` self-launched: eight ranks x 256 MiB, all on cuda:0
    (KVSEP_BENCH_SAME_DEVICE, gloo for the results), and EVERY one of the 524,288 blocks of the 8-rank global batch is
    checked against the reference's CRCs (tests/golden/full_cfg2.u32), none sampled."""
    env = dict(os.environ, KVSEP_BENCH_SAME_DEVICE="1")
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--config", "2", "--steps", "3", "--warmup",
           "1", "--no-cpu", "--roundtrip-gib", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 8 and line["world_size"] == 8 and len(line["digests"]) == 8, line
    p = line["parity"]
    assert p["blocks_checked_vs_reference"] == 524288 and p["blocks_sampled_vs_oracle"] == 0, p
    assert p["every_block_checked"] and p["mismatches"] == 0, p
    # eight per-rank records; all eight ran on the one GPU here, and the line says so
    pr = line["per_rank"]
    assert [r["rank"] for r in pr] == list(range(8)) and len({r["pid"] for r in pr}) == 8, pr
    assert len({r["pci_bus_id"] for r in pr}) == 1 and pr[0]["pci_bus_id"], pr
    assert all(r["kernel_avg_ms"] > 0 and r["GiBps"] > 0 and r["elapsed_s"] > 0 for r in pr), pr
    sm = line["per_rank_summary"]
    assert sm["ranks"] == 8 and sm["same_device_rehearsal"] and not sm["distinct_devices"], sm
    assert sm["GiBps_min"] <= sm["GiBps_max"] and 0 <= sm["GiBps_skew"] < 1 and sm["slowest_rank"] in range(8), sm


def test_two_ranks_host_round_trip_per_rank_records():
    """Two torchrun ranks on the one GPU with the host round trip on: each rank's record carries its own round-trip
    rate and the NUMA node of its pinned image (the node of the rank's GPU, where the rank bound itself), and the
    line's aggregate is the sum over ranks / the slowest rank."""
    env = dict(os.environ, KVSEP_BENCH_SAME_DEVICE="1", MASTER_ADDR="127.0.0.1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "2", "--no-cpu",
           "--config", "2", "--steps", "3", "--warmup", "1", "--roundtrip-gib", "0.25"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["host_roundtrip_parity"] is True and line["host_roundtrip_ranks"] == 2, line
    pr = line["per_rank"]
    assert len(pr) == 2 and all(x["roundtrip_GiBps"] > 0 for x in pr), pr
    node = pr[0]["numa_node"]
    if node is not None and node >= 0:
        assert all(x["roundtrip_image_numa_node"] == node for x in pr), pr
        assert all(x["staging"]["device_node"] == node for x in pr), pr
    assert line["host_roundtrip_GiBps"] <= sum(x["roundtrip_GiBps"] for x in pr) * 1.01, line


@pytest.mark.parametrize("config", ["2", "3a"])
def test_two_ranks_verify_form_reduction(config):
    """`bench.py --form verify` at two ranks: every rank verifies its shard against the reference's words, two planted
    mismatches per rank, and the global first_bad / nbad after the cross-rank reduction.  (Config 4 is 150 GiB per
    rank: two ranks do not fit one GPU; its verify form runs at one rank below.)"""
    line = _torchrun_bench(2, "--config", config, "--steps", "2", "--warmup", "1", "--form", "verify")
    v = line["verify"]
    assert v["ok"] and v["nbad"] == 4 and v["first_bad"] == 13, v
    assert line["parity"]["mismatches"] == 0 and line["parity"]["mismatching_digest_ranges"] == 0, line["parity"]


def test_verify_form_config4_one_rank():
    """Config 4's verify form (ragged Zipf blocks: the planned wide kernel, the combine kernel publishing the verdict)
    against the reference's words for its 2^20 blocks."""
    env = dict(os.environ)
    for k in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "KVSEP_BENCH_SAME_DEVICE"):
        env.pop(k, None)
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "4", "--steps", "2", "--warmup", "1",
           "--no-cpu", "--roundtrip-gib", "0", "--pmc-live", "off", "--form", "verify"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=900, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    v = line["verify"]
    assert v["ok"] and v["nbad"] == 2 and v["first_bad"] == 13, v
    assert line["parity"]["mismatches"] == 0 and line["parity"]["every_block_checked"], line["parity"]
