"""The staging pipeline's host copiers (csrc/copy_pool.h) under ThreadSanitizer and AddressSanitizer, no GPU: the pool
claims runs of chunks from a shared counter across threads (round 3), and every byte of many random gathers must land
where it belongs with no data race (tests/cpp/copy_pool_test.cc)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_copy_pool_under_sanitizer(tmp_path, san):
    exe = tmp_path / "copy_pool_test"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-pthread",
                           "-I", os.path.join(ROOT, "kv-separate_amd", "csrc"),
                           os.path.join(ROOT, "tests", "cpp", "copy_pool_test.cc"), "-o", str(exe)])
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1", ASAN_OPTIONS="detect_leaks=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "PASS" in r.stdout
