"""Host-side planning of the native kernels (csrc/kernel_abi.h) under AddressSanitizer and
UndefinedBehaviorSanitizer (race detection / sanitizers): the C++
test tests/native/plan_test.cpp is compiled with ``-fsanitize=address,undefined`` for the
host (GPU sanitizers are not available for gfx950 kernels here) and run on the CPU."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLANG = next((c for c in ("/opt/rocm/lib/llvm/bin/clang++", shutil.which("clang++") or "") if c and os.path.exists(c)),
             None)


@pytest.mark.skipif(CLANG is None, reason="clang++ not found")
def test_kernel_planning_under_asan_ubsan(tmp_path):
    exe = tmp_path / "plan_test"
    cmd = [CLANG, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=address,undefined",
           "-fno-sanitize-recover=all", f"-I{ROOT}/raft_ros_amd/csrc", f"{ROOT}/tests/native/plan_test.cpp",
           "-o", str(exe)]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=0", UBSAN_OPTIONS="print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    p = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300, env=env)
    assert p.returncode == 0, p.stdout + p.stderr
    assert "ok" in p.stdout
