"""ASan + UBSan over the host framing walkers (untrusted file bytes), no GPU: SURVEY.md §5 asks for
sanitizers on the host layer."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no g++")
def test_framing_walkers_under_asan_ubsan(tmp_path):
    exe = tmp_path / "framing_fuzz"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-g", "-fsanitize=address,undefined",
                           "-fno-sanitize-recover=undefined", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "framing_fuzz.cc"),
                           os.path.join(ROOT, "kv-separate_amd", "csrc", "framing.cpp"), "-o", str(exe)])
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "PASS" in r.stdout
