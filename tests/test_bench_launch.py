"""bench.py's rank launcher: `bench.py --gpus N` with no WORLD_SIZE starts N ranks itself, and a
WORLD_SIZE that disagrees with --gpus is refused -- so a scaling run can never silently measure one rank.  CPU only
(--dry-run: the ranks join a gloo group and agree on the world size; no GPU is touched)."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


BUS_IDS = "0000:05:00.0,0000:15:00.0,0000:65:00.0,0000:75:00.0"


@pytest.mark.parametrize("n", [1, 2, 3])
def test_gpus_n_launches_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run"], env=_env(KVSEP_BENCH_DRYRUN_BUS_IDS=BUS_IDS),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 alone prints
    line = json.loads(lines[0])
    assert line["n_gpus"] == n and line["world_size"] == n
    assert line["backend"] == ("gloo" if n > 1 else None)
    # every rank's record reaches rank 0 through the process group (gloo here, RCCL on the GPUs)
    pr = line["per_rank"]
    assert [r["rank"] for r in pr] == list(range(n)) and len({r["pid"] for r in pr}) == n, pr
    assert all(r["cpu_affinity"] and r["GiBps"] == 1.0 for r in pr), pr
    sm = line["per_rank_summary"]
    assert sm["ranks"] == n and sm["start_skew_ms"] is not None and sm["GiBps_skew"] == 0.0, sm
    assert sm["distinct_devices"] is True and sm["same_device_rehearsal"] is False, sm
    assert line["failures"] == []


def _dry(n, **kw):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run"], env=_env(**kw), capture_output=True,
                       text=True, timeout=300)
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, (r.stdout, r.stderr[-2000:])  # the line is printed whatever the verdict
    return r, json.loads(lines[0])


@pytest.mark.parametrize("ids", [None, "0000:05:00.0,0000:05:00.0"], ids=["no_bus_ids", "one_gpu_twice"])
def test_ranks_on_one_device_fail_the_run(ids):
    """N > 1 ranks that are not on distinct GPUs (no bus ID, or two ranks on one) print the line
    with the reason and exit non-zero, so a driver's N-GPU run cannot record a one-GPU number as N."""
    kw = {"KVSEP_BENCH_DRYRUN_BUS_IDS": ids} if ids else {}
    r, line = _dry(2, **kw)
    assert r.returncode == 1, r.stderr[-2000:]
    assert line["per_rank_summary"]["distinct_devices"] is False
    assert len(line["failures"]) == 1 and "not on distinct devices" in line["failures"][0]
    assert "not a clean measurement" in r.stderr


def test_same_device_rehearsal_is_allowed():
    r, line = _dry(2, KVSEP_BENCH_SAME_DEVICE="1")
    assert r.returncode == 0, r.stderr[-2000:]
    assert line["per_rank_summary"]["same_device_rehearsal"] is True and line["failures"] == []


def test_line_failures_rules():
    """The rule set itself, on hand-made lines: parity, the verify verdict, the host round trip, a missing rank record
    and the distinct-device rule each fail the line; a clean line passes."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", BENCH)
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    rec = lambda r, bus: {"rank": r, "pci_bus_id": bus}  # noqa: E731
    clean = {"parity": {"all_blocks_match": True, "mismatches": 0, "mismatching_digest_ranges": 0},
             "verify": {"ok": True}, "host_roundtrip_parity": True,
             "per_rank": [rec(0, "a"), rec(1, "b")], "per_rank_summary": {"distinct_devices": True}}
    assert bench.line_failures(clean, 2, False) == []
    for key, val, word in (("parity", {"all_blocks_match": False, "mismatches": 1, "mismatching_digest_ranges": 0},
                            "parity"),
                           ("verify", {"ok": False, "first_bad": 3, "nbad": 1}, "verify"),
                           ("host_roundtrip_parity", False, "round trip"),
                           ("per_rank", [rec(0, "a")], "per-rank records"),
                           ("per_rank_summary", {"distinct_devices": False}, "distinct devices")):
        bad = dict(clean, **{key: val})
        f = bench.line_failures(bad, 2, False)
        assert len(f) == 1 and word in f[0], (key, f)
    assert bench.line_failures(dict(clean, per_rank_summary={"distinct_devices": False}), 2, True) == []
    assert bench.line_failures(dict(clean, parity=None, verify=None, host_roundtrip_parity=None), 2, False) == []


def test_world_size_mismatch_is_refused():
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4", "--dry-run"],
                       env=_env(WORLD_SIZE="2", RANK="0", LOCAL_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT="29555"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode != 0
    assert "WORLD_SIZE=2" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_failing_rank_fails_the_launch():
    # rank 1 dies before joining the group: the launcher stops rank 0 (blocked in the rendezvous) and exits non-zero
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run"], env=_env(KVSEP_BENCH_DRYRUN_FAIL_RANK="1"),
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 3, r.stderr[-2000:]
    assert "rank 1 exited 3" in r.stderr
