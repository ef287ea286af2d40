"""C++ end-to-end: vlog file on disk -> pinned buffer -> batched GPU verify (tests/cpp/vlog_recover_demo.cc)."""
import os
import shutil
import subprocess

import pytest

import kvsep

pytestmark = pytest.mark.gpu
ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_cpp_vlog_recovery_demo(tmp_path):
    libdir = os.path.dirname(kvsep.LIB_PATH)
    exe = tmp_path / "vlog_recover_demo"
    subprocess.check_call(["g++", "-std=c++11", "-O2", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "vlog_recover_demo.cc"), "-L", libdir,
                           "-lkvsep_crc32c", f"-Wl,-rpath,{libdir}", "-o", str(exe)])
    r = subprocess.run([str(exe), str(tmp_path)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_cpp_sst_whole_table_verify_demo(tmp_path):
    """tests/cpp/sst_verify_demo.cc on the SST the reference TableBuilder wrote: the handles its footer/index decode
    finds are the reference's own blocks (tests/golden/ref_framing.json), one batched read check passes them all, and a
    flipped byte is named at exactly its block."""
    import json

    libdir = os.path.dirname(kvsep.LIB_PATH)
    exe = tmp_path / "sst_verify_demo"
    subprocess.check_call(["g++", "-std=c++11", "-O2", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "sst_verify_demo.cc"), "-L", libdir,
                           "-lkvsep_crc32c", f"-Wl,-rpath,{libdir}", "-o", str(exe)])
    r = subprocess.run([str(exe), os.path.join(ROOT, "tests", "golden", "ref_table.sst")], capture_output=True,
                       text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout
    found = [tuple(int(x) for x in l.split()[2:4]) for l in r.stdout.splitlines() if l.startswith("handle ")]
    with open(os.path.join(ROOT, "tests", "golden", "ref_framing.json")) as f:
        ref = [(b[0], b[1]) for b in json.load(f)["sst"]["blocks"]]
    assert sorted(found) == sorted(ref)
