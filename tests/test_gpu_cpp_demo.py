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
