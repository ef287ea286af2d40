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


@pytest.mark.parametrize("n", [1, 2, 3])
def test_gpus_n_launches_n_ranks(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run"], env=_env(), capture_output=True,
                       text=True, timeout=300)
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
    assert sm["distinct_devices"] is False and sm["same_device_rehearsal"] is False  # no device: not distinct


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
