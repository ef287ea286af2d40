"""The link-level drop-in, exercised through the reference's OWN call sites.

oracle/_ref/ref_framing_kvsep is the reference's db/value_log_writer.cc, db/value_log_reader.cc, db/log_writer.cc,
db/log_reader.cc, table/table_builder.cc and table/format.cc (compiled unchanged, with the reference's unchanged
util/crc32c.h) linked against libkvsep_crc32c.so INSTEAD of util/crc32c.cc: every crc32c::Extend / Value of those
files resolves to the library's exported leveldb::crc32c::Extend (util/crc32c.h:17).  It writes a vlog, a
MANIFEST log and an SST and reads intact and corrupted copies back with the reference readers.  The same driver
linked with the real util/crc32c.cc produced tests/golden/ref_framing.json (tests/golden/make_framing_golden.py):
the files must be byte-identical (SHA-256) and every reader verdict -- records returned, bytes reported dropped
and why -- identical.

CPU: the drop-in's host leg (every call below the offload threshold), on each of its three legs.  GPU: threshold 0, so every Extend -- down to
log_writer.cc's 1-byte InitTypeCrc calls -- runs through the GPU, and the driver fails if any call finished on
the host."""
import hashlib
import json
import os
import subprocess

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
DRIVER = os.path.join(ROOT, "oracle", "_ref", "ref_framing_kvsep")
GOLD = os.path.join(ROOT, "tests", "golden", "ref_framing.json")


def _gold():
    with open(GOLD) as f:
        return json.load(f)


def _run(tmp_path, gpu, host_leg=None):
    args = [DRIVER, str(tmp_path)] + (["gpu"] if gpu else [])
    env = dict(os.environ)
    env.pop("KVSEP_HOST_CRC", None)
    if host_leg:
        env["KVSEP_HOST_CRC"] = host_leg
    r = subprocess.run(args, capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, (r.returncode, r.stderr[-2000:])
    return json.loads(r.stdout), r.stderr


def _check(j, tmp_path):
    g = _gold()
    for section in ("vlog", "log", "sst"):
        assert j[section] == g[section], section
    for name, sha in g["sha256"].items():
        with open(os.path.join(tmp_path, name), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == sha, name


@pytest.mark.skipif(not os.path.exists(DRIVER), reason="oracle/_ref not built here (needs /root/reference)")
@pytest.mark.parametrize("host_leg", [None, "sse42", "portable"])
def test_reference_callsites_on_engine_host_leg(tmp_path, host_leg):
    """On each host leg (round 5: the portable leg that non-x86 hosts and x86 CPUs without SSE4.2 run, too)."""
    j, err = _run(tmp_path, gpu=False, host_leg=host_leg)
    _check(j, tmp_path)
    assert "0 gpu calls" in err


@pytest.mark.gpu
def test_reference_callsites_on_engine_gpu(tmp_path):
    assert os.path.exists(DRIVER), "oracle/_ref/ref_framing_kvsep must be built in the dev container (build())"
    j, err = _run(tmp_path, gpu=True)
    _check(j, tmp_path)
    assert " 0 host calls, 0 gpu failures" in err, err
