"""Host placement next to the GPU, on the GPU box, and the verify accumulators after a failed
call:

  * the device's PCI bus ID and NUMA node equal what sysfs says for it;
  * a context's pinned staging is allocated on, and its copier threads run on, that node -- the binding equals
    sysfs (its CPUs this process may use), checked from the outside through /proc (threads named kvsep-copy);
  * a group's members place theirs the same way; a context told set_host_node(-1) places nothing;
  * bench.py's per-rank binding (kvsep_bind_process_numa after selecting the device): every thread on the node, and a
    pinned torch buffer allocated afterwards on it;
  * a verify call that fails after its CRC kernel posted mismatches (kvsep_crc32c_ctx_inject_failure) does not leak
    them into the next verdict -- planned, unsplit-narrow and graph-captured calls.
"""
import json
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import kvsep
from kvsep import splitmix64_bytes

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")
if not torch.cuda.is_available():  # pragma: no cover
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
DEV = torch.device("cuda:0")


def _sys_node(bdf):
    p = f"/sys/bus/pci/devices/{bdf}/numa_node"
    return int(open(p).read()) if os.path.exists(p) else -1


def _node_cpus_allowed(node, allowed):
    p = f"/sys/devices/system/node/node{node}/cpulist"
    if node < 0 or not os.path.exists(p):
        return []
    cpus = set()
    for part in open(p).read().strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            cpus.update(range(int(a), int(b) + 1))
        elif part:
            cpus.add(int(part))
    return sorted(cpus & set(allowed))


def _copier_affinities():
    out = []
    for t in os.listdir("/proc/self/task"):
        try:
            if open(f"/proc/self/task/{t}/comm").read().strip() == "kvsep-copy":
                out.append(sorted(os.sched_getaffinity(int(t))))
        except (OSError, ProcessLookupError):
            pass
    return out


def test_device_bus_id_and_node_match_sysfs():
    bdf = kvsep.pci_bus_id(0)
    assert re.fullmatch(r"[0-9a-f]{4}:[0-9a-f]{2}:[0-9a-f]{2}\.[0-7]", bdf), bdf
    assert kvsep.device_numa_node(0) == _sys_node(bdf) == kvsep.pci_numa_node(bdf.upper())
    print(json.dumps({"pci_bus_id": bdf, "numa_node": _sys_node(bdf),
                      "node_cpus": kvsep.format_cpulist(kvsep.numa_node_cpus(max(0, _sys_node(bdf))))}))


def test_context_staging_and_copiers_on_the_device_node(oracle):
    node = kvsep.device_numa_node(0)
    want = _node_cpus_allowed(node, os.sched_getaffinity(0))
    ctx = kvsep.Context(0)
    try:
        buf = splitmix64_bytes(96 << 20, 5, 0)  # pageable: the copiers gather it into the pinned slots
        off = np.arange(0, 96 << 20, 1 << 20, dtype=np.uint64)
        ln = np.full(off.size, 1 << 20, np.uint64)
        assert np.array_equal(ctx.batch_host_span(buf, off, ln), oracle.batch(buf, off, ln, threads=8))
        pl = ctx.host_placement()
        assert pl["device_node"] == node, pl
        assert pl["copier_cpus"] == want, (pl, want)
        if want:
            assert pl["staging_node"] == node, pl
            aff = _copier_affinities()
            assert aff and all(a == want for a in aff), aff
        print(json.dumps({"placement": {**pl, "copier_cpus": kvsep.format_cpulist(pl["copier_cpus"])}}))
    finally:
        ctx.close()


def test_context_without_placement():
    ctx = kvsep.Context(0)
    try:
        ctx.set_host_node(-1)
        buf = splitmix64_bytes(8 << 20, 6, 0)
        ctx.batch_host_span(buf, np.array([0], np.uint64), np.array([8 << 20], np.uint64))
        pl = ctx.host_placement()
        assert pl["device_node"] == -1 and pl["copier_cpus"] == [], pl
    finally:
        ctx.close()


def test_group_members_on_their_device_node(oracle):
    import ctypes
    node = kvsep.device_numa_node(0)
    want = _node_cpus_allowed(node, os.sched_getaffinity(0))
    before = os.sched_getaffinity(0)
    g = kvsep.Group([0, 0])
    try:
        ln = np.full(200, 300_000, np.uint64)
        off = np.arange(200, dtype=np.uint64) * np.uint64(300_007)
        buf = splitmix64_bytes(int(off[-1] + ln[-1]) + 64, 77, 0)
        assert np.array_equal(g.batch_host_span(buf, off, ln), oracle.batch(buf, off, ln, threads=8))
        assert os.sched_getaffinity(0) == before  # member 0 ran on this thread: its binding was undone
        lib = kvsep.lib()
        for i in range(2):
            c = lib.kvsep_crc32c_group_ctx(g._h, i)
            dn, sn = ctypes.c_int(), ctypes.c_int()
            cpus = (ctypes.c_int * 4096)()
            n = lib.kvsep_crc32c_ctx_host_placement(c, ctypes.byref(dn), ctypes.byref(sn), cpus, 4096)
            assert dn.value == node and list(cpus[:n]) == want, (i, dn.value, list(cpus[:n]), want)
            if want:
                assert sn.value == node
    finally:
        g.close()


BIND_CHILD = r"""
import json, os, sys
import torch
sys.path.insert(0, os.path.join(sys.argv[1], "kv-separate_amd"))
import kvsep
torch.cuda.set_device(0)
torch.zeros(1, device="cuda")  # the HIP runtime's threads exist now
node = kvsep.device_numa_node(0)
allowed = sorted(os.sched_getaffinity(0))
n = kvsep.bind_process_numa(node)
buf = torch.empty(64 << 20, dtype=torch.uint8, pin_memory=True)
buf.fill_(1)
tasks = {}
for t in os.listdir("/proc/self/task"):
    try:
        tasks[t] = sorted(os.sched_getaffinity(int(t)))
    except ProcessLookupError:  # a thread that ended since the listing
        pass
print(json.dumps({"node": node, "allowed": allowed, "bound": n, "tasks": tasks,
                  "pinned_node": kvsep.host_page_node(buf.data_ptr()),
                  "pinned_node_end": kvsep.host_page_node(buf.data_ptr() + (64 << 20) - 1)}))
"""


def test_bench_rank_binding_every_thread_and_pinned_memory():
    r = subprocess.run([sys.executable, "-c", BIND_CHILD, ROOT], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    out = json.loads(r.stdout.strip().splitlines()[-1])
    want = _node_cpus_allowed(out["node"], out["allowed"])
    assert out["bound"] == len(want), out
    if want:
        assert all(v == want for v in out["tasks"].values()), out["tasks"]
        assert out["pinned_node"] == out["node"] and out["pinned_node_end"] == out["node"], out
    print(json.dumps({k: out[k] for k in ("node", "bound", "pinned_node", "pinned_node_end")}))


# ---------------------------------------------------------------- verify accumulators after a failed call
def _mixed_batch(seed):
    """Alternating 1 MiB blocks (split into pieces: the combine kernel compares them) and 1,000-B blocks (whole-block
    items: the CRC kernel itself compares and posts them) -- a planned batch whose CRC kernel posts mismatches."""
    n = 64
    ln = np.where(np.arange(n) % 2 == 0, 1 << 20, 1000).astype(np.uint64)
    off = np.zeros(n, np.uint64)
    off[1:] = np.cumsum(ln[:-1] + np.uint64(16), dtype=np.uint64)
    buf = splitmix64_bytes(int(off[-1] + ln[-1]) + 64, seed, 0)
    return buf, off, ln


def _u64(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint64).view(np.int64)).to(DEV)


def _verify(ctx, d, off, ln, stored, max_len, stream=None):
    out = torch.zeros(off.numel(), dtype=torch.int32, device=DEV)
    fb = torch.zeros(1, dtype=torch.int64, device=DEV)
    nb = torch.zeros(1, dtype=torch.int64, device=DEV)
    ctx.verify_device(d, off, ln, stored, out, fb, nb, max_len=max_len, stream=stream)
    torch.cuda.synchronize()
    return int(fb.item()) & (2**64 - 1), int(nb.item())


@pytest.mark.parametrize("max_len", [0, 1 << 20], ids=["planned", "planned_hint"])
def test_failed_verify_does_not_leak_into_the_next_verdict(oracle, max_len):
    buf, off, ln = _mixed_batch(404)
    exp = oracle.batch(buf, off, ln, threads=8)
    good = np.array([kvsep.mask(int(c)) for c in exp], np.uint32)
    bad = good.copy()
    bad[[1, 7, 33]] ^= 0x10  # three short (whole-block) records: posted by the CRC kernel itself
    d = torch.from_numpy(buf).to(DEV)
    doff, dln = _u64(off), _u64(ln)
    dgood = torch.from_numpy(good.view(np.int32)).to(DEV)
    dbad = torch.from_numpy(bad.view(np.int32)).to(DEV)
    ctx = kvsep.Context(0)
    try:
        assert _verify(ctx, d, doff, dln, dbad, max_len) == (1, 3)
        ctx.inject_failure()
        with pytest.raises(kvsep.KvsepError, match="injected"):
            _verify(ctx, d, doff, dln, dbad, max_len)
        torch.cuda.synchronize()  # the failed call's CRC kernel ran and posted its three mismatches
        assert _verify(ctx, d, doff, dln, dgood, max_len) == (2**64 - 1, 0)  # not (1, 3): the posts were reset
        assert _verify(ctx, d, doff, dln, dbad, max_len) == (1, 3)
        assert _verify(ctx, d, doff, dln, dgood, max_len) == (2**64 - 1, 0)
    finally:
        ctx.close()


def test_failed_narrow_verify_then_exact():
    """The unsplit (narrow kernel) form publishes from the CRC kernel itself; a failure reported after it still
    leaves the next verdicts exact."""
    n = 40000
    ln = np.full(n, 4096, np.uint64)
    off = np.arange(n, dtype=np.uint64) * np.uint64(4096)
    buf = splitmix64_bytes(n * 4096, 77, 0)
    exp = np.array([kvsep.extend_host(0, buf[i * 4096:(i + 1) * 4096]) for i in range(n)], np.uint32)
    good = np.array([kvsep.mask(int(c)) for c in exp], np.uint32)
    bad = good.copy()
    bad[[5, 39999]] ^= 1
    d = torch.from_numpy(buf).to(DEV)
    doff, dln = _u64(off), _u64(ln)
    dgood = torch.from_numpy(good.view(np.int32)).to(DEV)
    dbad = torch.from_numpy(bad.view(np.int32)).to(DEV)
    ctx = kvsep.Context(0)
    try:
        ctx.inject_failure()
        with pytest.raises(kvsep.KvsepError):
            _verify(ctx, d, doff, dln, dbad, 4096)
        torch.cuda.synchronize()
        assert _verify(ctx, d, doff, dln, dgood, 4096) == (2**64 - 1, 0)
        assert _verify(ctx, d, doff, dln, dbad, 4096) == (5, 2)
    finally:
        ctx.close()


def test_captured_verify_calls_use_their_own_accumulators():
    """Two graphs, each one captured verify call of the same context (accumulator sets 1 and 2), replayed on two
    streams at once, and an eager call (set 0) after them: every verdict is its own.  Unplanned
    batches (4 KiB blocks, the claim kernel): they use no scratch but the accumulators, so their replays may overlap."""
    n = 40000
    ln = np.full(n, 4096, np.uint64)
    off = np.arange(n, dtype=np.uint64) * np.uint64(4096)
    buf = splitmix64_bytes(n * 4096, 505, 0)
    exp = np.array([kvsep.extend_host(0, buf[i * 4096:(i + 1) * 4096]) for i in range(n)], np.uint32)
    good = np.array([kvsep.mask(int(c)) for c in exp], np.uint32)
    bad = good.copy()
    bad[[3, 9]] ^= 0x4
    d = torch.from_numpy(buf).to(DEV)
    doff, dln = _u64(off), _u64(ln)
    dgood = torch.from_numpy(good.view(np.int32)).to(DEV)
    dbad = torch.from_numpy(bad.view(np.int32)).to(DEV)
    ctx = kvsep.Context(0)
    try:
        ctx.reserve(n, int(ln.sum()))
        res, graphs = [], []
        for ex in (dgood, dbad):
            out = torch.zeros(n, dtype=torch.int32, device=DEV)
            fb = torch.zeros(1, dtype=torch.int64, device=DEV)
            nb = torch.zeros(1, dtype=torch.int64, device=DEV)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                ctx.verify_device(d, doff, dln, ex, out, fb, nb, total_bytes=n * 4096, max_len=4096)
            graphs.append(g)
            res.append((fb, nb))
        torch.cuda.synchronize()
        s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
        for _ in range(8):
            with torch.cuda.stream(s1):
                graphs[0].replay()
            with torch.cuda.stream(s2):
                graphs[1].replay()
            torch.cuda.synchronize()
            assert (int(res[0][0].item()) & (2**64 - 1), int(res[0][1].item())) == (2**64 - 1, 0)
            assert (int(res[1][0].item()), int(res[1][1].item())) == (3, 2)
            assert _verify(ctx, d, doff, dln, dbad, 4096) == (3, 2)
            assert _verify(ctx, d, doff, dln, dgood, 4096) == (2**64 - 1, 0)
    finally:
        ctx.close()
