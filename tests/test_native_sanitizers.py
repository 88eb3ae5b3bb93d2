"""Race detection / memory checking of the host runtime.

The threaded C++ core that ships in ``_C.so`` (csrc/runtime_core.h: BatchDispenser, StalenessGate)
is compiled twice on the host, without GPU code, into ``tests/native/runtime_stress.cpp``: once
with ThreadSanitizer and once with AddressSanitizer + UBSan.  The stress program races 8 workers and
a reader thread on one dispenser (claim / drop / complete, as the async parameter server does) and
checks exactly-once completion per (epoch, batch) under re-dispatch.  GPU sanitizers are not
available on the MI355X pool, so device code is covered by the numerics tests instead.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "runtime_stress.cpp")
CXX = shutil.which("g++") or shutil.which("clang++")


@pytest.mark.skipif(CXX is None, reason="no host C++ compiler")
@pytest.mark.timeout(300)
@pytest.mark.parametrize("san", ["thread", "address,undefined"])
def test_runtime_core_under_sanitizer(tmp_path, san):
    exe = tmp_path / f"stress_{san.split(',')[0]}"
    cmd = [CXX, "-std=c++17", "-O1", "-g", f"-fsanitize={san}", "-fno-omit-frame-pointer",
           f"-I{os.path.join(ROOT, 'csrc')}", SRC, "-o", str(exe), "-pthread"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-3000:]
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 second_deadlock_stack=1",
               ASAN_OPTIONS="halt_on_error=1 detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1 print_stacktrace=1")
    env.pop("LD_PRELOAD", None)
    r = subprocess.run([str(exe)], capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, (r.stdout + r.stderr)[-4000:]
    assert "runtime_stress ok" in r.stdout
