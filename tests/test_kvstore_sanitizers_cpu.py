"""Race detection for the native key/value store: the pybind-free core
(csrc/store/kvstore_core.h) is compiled with the host sanitizers into a standalone multi-threaded
stress driver (csrc/store/kvstore_stress.cpp) and run. ThreadSanitizer covers the server's
accept / worker / shutdown paths and the condition-variable WAIT; AddressSanitizer + UBSan cover the
frame parser and the connection bookkeeping. The reference has no native code of its own (its DHT is
hivemind's libp2p daemon), so there is no reference counterpart to compare against.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "csrc", "store", "kvstore_stress.cpp")

SANITIZERS = {
    "tsan": ["-fsanitize=thread"],
    "asan_ubsan": ["-fsanitize=address,undefined", "-fno-sanitize-recover=undefined", "-fno-omit-frame-pointer"],
}


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
@pytest.mark.parametrize("kind", sorted(SANITIZERS))
def test_kvstore_stress_under_sanitizer(kind, tmp_path):
    exe = str(tmp_path / f"kvstore_stress_{kind}")
    cmd = ["g++", "-std=c++17", "-O1", "-g", *SANITIZERS[kind], "-I", os.path.dirname(SRC), SRC, "-o", exe, "-pthread"]
    subprocess.run(cmd, check=True, capture_output=True, text=True, timeout=300)
    env = dict(os.environ)
    env["TSAN_OPTIONS"] = "halt_on_error=1 second_deadlock_stack=1"
    env["ASAN_OPTIONS"] = "halt_on_error=1 detect_leaks=1"
    env["UBSAN_OPTIONS"] = "halt_on_error=1 print_stacktrace=1"
    r = subprocess.run([exe, "8", "200"], capture_output=True, text=True, timeout=240, env=env)
    report = r.stdout + r.stderr
    assert r.returncode == 0, report[-4000:]
    assert "WARNING: ThreadSanitizer" not in report and "ERROR: AddressSanitizer" not in report, report[-4000:]
    assert "runtime error:" not in report, report[-4000:]
    assert "kvstore stress ok" in r.stdout
