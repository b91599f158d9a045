"""Host-side AddressSanitizer + UndefinedBehaviorSanitizer build of the C++ runtime pieces that
run without a GPU: the reducer's bucket state machine (bucket_schedule.h), the
FastDiv index arithmetic and ConvShape.  GPU sanitizers / xnack are not available on this pool,
so the sanitizers are applied to host code only (`-Xarch_host -fsanitize=...`)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "mxddp", "csrc")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


@pytest.mark.skipif(not os.path.exists(HIPCC) and shutil.which("hipcc") is None, reason="no hipcc")
def test_host_selftest_asan_ubsan(tmp_path):
    exe = tmp_path / "mx_selftest"
    cmd = [HIPCC, "-O1", "-g", "-std=c++17", f"-I{CSRC}",
           "-Xarch_host", "-fsanitize=address", "-Xarch_host", "-fsanitize=undefined",
           "-Xarch_host", "-fno-sanitize-recover=undefined", "-Xarch_host", "-fno-omit-frame-pointer",
           os.path.join(CSRC, "host_tests", "selftest.cpp"), "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, timeout=600)
    syms = subprocess.run(["nm", str(exe)], capture_output=True, text=True).stdout
    assert "__asan_report" in syms and "__ubsan_handle" in syms, "sanitizers not linked in"
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "ALL OK" in r.stdout
