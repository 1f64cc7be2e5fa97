"""Host-side race / memory-error detection for the native loader: the torch-free core
(csrc/loader_core.h) is compiled with ThreadSanitizer and with AddressSanitizer + UBSan and driven by a
multi-worker stress harness (tests/native/loader_stress.cpp) that checks every batch against a
single-threaded decode.  GPU code is not sanitised (not available on this pool)."""
import os
import shutil
import subprocess

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(os.path.dirname(HERE), "pytorch_imageclassification_distributed_amd", "csrc")
SRC = os.path.join(HERE, "native", "loader_stress.cpp")

pytestmark = pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")


@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_loader_core_under_sanitizer(tmp_path, san):
    exe = str(tmp_path / "loader_stress")
    cmd = ["g++", "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer", f"-I{CSRC}", SRC,
           "-o", exe, "-lz", "-pthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0 and "sanitizer" in r.stderr.lower():
        pytest.skip(f"-fsanitize={san} unavailable: {r.stderr[-300:]}")
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="detect_leaks=1 halt_on_error=1", UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1")
    run = subprocess.run([exe, str(tmp_path)], capture_output=True, text=True, env=env, timeout=300)
    assert run.returncode == 0 and "loader_stress OK" in run.stdout, (run.stdout[-2000:], run.stderr[-4000:])
    assert "WARNING: ThreadSanitizer" not in run.stderr and "ERROR: AddressSanitizer" not in run.stderr
