"""The RCCL path of bench.py / kvsep.shard executed on the one-GPU box: a ONE-rank `nccl` process
group is a real RCCL communicator, and with it the same code runs as at eight ranks -- `dist.init_process_group("nccl",
device_id=...)` as bench.py makes it, and every shard.py collective on device tensors with bench's dtypes and ops:
int64 and int32 all_gather (gather_results), float64 all_reduce MAX / MIN / SUM (max/min/sum_over_ranks).

  * test_shard_collectives_one_rank_rccl: the collectives directly, in a child process, against known answers;
  * test_bench_torchrun_one_rank_rccl: `torchrun --nproc-per-node 1 bench.py --gpus 1` -- bench.py's own RCCL init,
    barriers, max-over-ranks time, byte sum, result gather and the host round trip's min/max reductions -- with
    every block of config 2 checked against the reference.
"""
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env():
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()))
    env.pop("KVSEP_BENCH_SAME_DEVICE", None)
    return env


CHILD = textwrap.dedent(r"""
    import json, os, sys
    import numpy as np
    import torch
    import torch.distributed as dist
    sys.path.insert(0, os.path.join(sys.argv[1], "kv-separate_amd"))
    from kvsep import shard
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    dist.init_process_group("nccl", device_id=dev, rank=0, world_size=1)   # bench.py's init
    assert dist.get_backend() == "nccl" and dist.get_world_size() == 1
    out = {}
    crcs = (np.arange(70_001, dtype=np.uint64) * 2654435761 % 2**32).astype(np.uint32)
    g = shard.gather_results(crcs, dist, dev)                              # int64 sizes + int32 payload all_gather
    out["gather"] = len(g) == 1 and np.array_equal(g[0], crcs)
    e = shard.gather_results(np.zeros(0, np.uint32), dist, dev)           # an empty shard (a rank with no blocks)
    out["gather_empty"] = len(e) == 1 and e[0].size == 0
    out["max"] = shard.max_over_ranks(1.25, dist, dev) == 1.25            # float64 all_reduce MAX
    out["min"] = shard.min_over_ranks(-3.5, dist, dev) == -3.5            # MIN
    out["sum"] = shard.sum_over_ranks(float(2**40 + 7), dist, dev) == float(2**40 + 7)   # SUM (byte totals)
    dist.barrier()
    out["digest"] = shard.crc_of_crcs(crcs, __import__("kvsep").extend_host)
    dist.destroy_process_group()
    print(json.dumps(out), flush=True)
""")


def test_shard_collectives_one_rank_rccl():
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True, timeout=300, env=_env(),
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert all(out[k] for k in ("gather", "gather_empty", "max", "min", "sum")), out


def test_bench_torchrun_one_rank_rccl():
    env = _env()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", env["MASTER_PORT"], os.path.join(ROOT, "bench.py"), "--gpus", "1", "--config",
           "2", "--steps", "4", "--warmup", "1", "--no-cpu", "--pmc-live", "off", "--roundtrip-gib", "0.25"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["backend"] == "nccl" and line["n_gpus"] == 1 and line["world_size"] == 1, line
    p = line["parity"]
    assert p["every_block_checked"] and p["blocks_checked_vs_reference"] == 65536 and p["mismatches"] == 0, p
    assert line["host_roundtrip_parity"] is True and line["host_roundtrip_GiBps"] > 0, line
    # the rank's own record, gathered over RCCL, names the physical GPU and where its host legs ran
    import re
    pr = line["per_rank"]
    assert len(pr) == 1 and pr[0]["rank"] == 0 and pr[0]["local_rank"] == 0, pr
    bdf = pr[0]["pci_bus_id"]
    assert re.fullmatch(r"[0-9a-f]{4}:[0-9a-f]{2}:[0-9a-f]{2}\.[0-7]", bdf or ""), pr
    node_path = f"/sys/bus/pci/devices/{bdf}/numa_node"
    sys_node = int(open(node_path).read()) if os.path.exists(node_path) else -1
    assert pr[0]["numa_node"] == sys_node, (pr, sys_node)
    assert pr[0]["kernel_avg_ms"] > 0 and pr[0]["GiBps"] > 0 and pr[0]["roundtrip_GiBps"] > 0, pr
    sm = line["per_rank_summary"]
    assert sm["ranks"] == 1 and sm["distinct_devices"] and sm["pci_bus_ids"] == [bdf], sm


def test_bench_verify_form_one_rank_rccl():
    """`--form verify` through bench's RCCL path: each step is the verify form against the reference's stored words
    with two planted mismatches, and the verdict goes through the all-reduce MIN / SUM of SURVEY.md §8e."""
    env = _env()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1", "--master-addr",
           "127.0.0.1", "--master-port", env["MASTER_PORT"], os.path.join(ROOT, "bench.py"), "--gpus", "1", "--config",
           "2", "--steps", "4", "--warmup", "1", "--no-cpu", "--pmc-live", "off", "--roundtrip-gib", "0",
           "--form", "verify"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    v = line["verify"]
    assert line["form"] == "verify" and v["ok"] and v["nbad"] == 2 and v["first_bad"] == 13, v
    assert line["parity"]["mismatches"] == 0 and line["parity"]["every_block_checked"], line["parity"]


def test_bench_wrong_result_exits_nonzero():
    """one gathered result word corrupted (test hook KVSEP_BENCH_CORRUPT_RESULT=<rank>) makes the
    reference check fail -- bench.py still prints the line, with the reason in `failures`, and exits non-zero, so a
    driver reading rc never records it as a clean number."""
    env = _env()
    env["KVSEP_BENCH_CORRUPT_RESULT"] = "0"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--config", "2", "--steps", "2", "--warmup", "1", "--no-cpu",
           "--pmc-live", "off", "--roundtrip-gib", "0"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=env, cwd=ROOT)
    assert r.returncode == 1, (r.returncode, r.stderr[-3000:])
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["parity"]["all_blocks_match"] is False and line["parity"]["mismatches"] == 1, line["parity"]
    assert len(line["failures"]) == 1 and line["failures"][0].startswith("parity"), line["failures"]
    assert line["value"] > 0  # the measurement itself is still reported
