"""Host placement next to a GPU on a faked topology, no GPU: sysfs is read under
$KVSEP_SYSFS_ROOT, so a fake tree -- node0 = CPUs 0-3, node1 = 4-5,7, PCI function 0000:aa:00.0 on node 1,
0000:bb:00.0 with numa_node -1 -- drives the same code the GPU box runs:

  * the C-ABI topology calls (kvsep_pci_numa_node, kvsep_numa_node_cpus) and the CPU-list mapping;
  * kvsep_bind_process_numa, as bench.py calls it per rank: EVERY thread of the process (one started before the call
    too) lands on the node's CPUs; an unknown node changes nothing;
  * numa.h's ScopedBind (the group members' threads, the staging allocation) and the copier pool's binding
    (tests/cpp/numa_test.cc): bound for the scope, restored after; the copiers run on the node's CPUs."""
import os
import subprocess
import sys

import pytest

import kvsep

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "kv-separate_amd", "csrc")

pytestmark = pytest.mark.skipif(not hasattr(os, "sched_getaffinity") or os.sched_getaffinity(0) != set(range(8)),
                                reason="the fake topology assumes this process may run on CPUs 0-7")


@pytest.fixture
def fake_sysfs(tmp_path):
    for n, cl in ((0, "0-3"), (1, "4-5,7")):
        d = tmp_path / "devices" / "system" / "node" / f"node{n}"
        d.mkdir(parents=True)
        (d / "cpulist").write_text(cl + "\n")
    for bdf, node in (("0000:aa:00.0", "1"), ("0000:bb:00.0", "-1")):
        d = tmp_path / "bus" / "pci" / "devices" / bdf
        d.mkdir(parents=True)
        (d / "numa_node").write_text(node + "\n")
    return str(tmp_path)


CHILD = r"""
import json, os, sys, threading, time
sys.path.insert(0, os.path.join(sys.argv[1], "kv-separate_amd"))
import kvsep
out = {"aa": kvsep.pci_numa_node("0000:AA:00.0"), "bb": kvsep.pci_numa_node("0000:bb:00.0"),
       "cc": kvsep.pci_numa_node("0000:cc:00.0"), "cpus1": kvsep.numa_node_cpus(1), "cpus9": kvsep.numa_node_cpus(9)}
stop = threading.Event()
early = threading.Thread(target=stop.wait)  # a thread that exists before the binding (as the HIP runtime's do)
early.start()
out["unknown"] = kvsep.bind_process_numa(9)
out["after_unknown"] = sorted(os.sched_getaffinity(0))
out["bound"] = kvsep.bind_process_numa(out["aa"])
out["main"] = sorted(os.sched_getaffinity(0))
out["early"] = sorted(os.sched_getaffinity(early.native_id))
late = threading.Thread(target=lambda: out.__setitem__("late", sorted(os.sched_getaffinity(0))))
late.start(); late.join()
out["tasks"] = {}
for t in os.listdir("/proc/self/task"):
    try:
        out["tasks"][t] = kvsep.format_cpulist(os.sched_getaffinity(int(t)))
    except ProcessLookupError:  # a thread that ended since the listing
        pass
stop.set(); early.join()
print(json.dumps(out))
"""


def test_topology_and_process_binding(fake_sysfs):
    import json
    env = dict(os.environ, KVSEP_SYSFS_ROOT=fake_sysfs)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    assert (out["aa"], out["bb"], out["cc"]) == (1, -1, -1), out
    assert out["cpus1"] == [4, 5, 7] and out["cpus9"] == [], out
    assert out["unknown"] == 0 and out["after_unknown"] == list(range(8)), out
    assert out["bound"] == 3 and out["main"] == [4, 5, 7], out
    assert out["early"] == [4, 5, 7] and out["late"] == [4, 5, 7], out
    assert set(out["tasks"].values()) == {"4-5,7"}, out["tasks"]


def test_format_cpulist():
    assert kvsep.format_cpulist([0, 1, 2, 3, 8, 10, 11]) == "0-3,8,10-11"
    assert kvsep.format_cpulist([]) == ""
    assert kvsep.format_cpulist({7, 5, 4}) == "4-5,7"


def test_scoped_bind_and_copier_pool(tmp_path, fake_sysfs):
    exe = tmp_path / "numa_test"
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-pthread", "-I", CSRC, "-o", str(exe),
                           os.path.join(ROOT, "tests", "cpp", "numa_test.cc")])
    r = subprocess.run([str(exe)], env=dict(os.environ, KVSEP_SYSFS_ROOT=fake_sysfs), capture_output=True, text=True,
                       timeout=60)
    assert r.returncode == 0 and "numa_test ok" in r.stdout, r.stdout + r.stderr
