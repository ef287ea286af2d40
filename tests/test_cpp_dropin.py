"""The C++ drop-in header compiles against the reference's call pattern and passes
util/crc32c_test.cc's assertions when linked to libkvsep_leveldb_abi.so + libkvsep_crc32c.so (host leg; no GPU
needed)."""
import os
import shutil
import subprocess

import pytest

import kvsep

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_cpp_dropin(tmp_path):
    libdir = os.path.dirname(kvsep.LIB_PATH)
    exe = tmp_path / "crc32c_dropin_test"
    subprocess.check_call(["g++", "-std=c++11", "-O2", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "crc32c_dropin_test.cc"), "-L", libdir,
                           "-lkvsep_leveldb_abi", "-lkvsep_crc32c", f"-Wl,-rpath,{libdir}", "-o", str(exe)])
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "PASS" in r.stdout
