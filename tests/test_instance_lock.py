"""The drop-in API's instance lock (siamese_amd/csrc/engine.h InstanceLock):
readers counted in per-thread slots, a writer that excludes every reader and
every other writer.  Built from the header with g++ and stressed on the CPU
(tests/instance_lock_test.cpp)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_instance_lock_excludes_readers_and_writers(tmp_path):
    exe = tmp_path / "instance_lock_test"
    subprocess.run(["g++", "-O2", "-std=c++17", "-pthread", "-DSGPU_DEBUG_LOCKS",
                    "-I", os.path.join(ROOT, "siamese_amd", "csrc"), "-I", os.path.join(ROOT, "include"),
                    os.path.join(ROOT, "tests", "instance_lock_test.cpp"), "-o", str(exe)],
                   check=True, timeout=120)
    out = subprocess.run([str(exe)], capture_output=True, text=True, timeout=60)
    assert out.returncode == 0, out.stdout + out.stderr
    assert "bad 0" in out.stdout
    # (the debug build catches a nested shared acquisition on one thread)
    nested = subprocess.run([str(exe), "nested"], capture_output=True, text=True, timeout=60)
    assert nested.returncode != 0 and "nested shared acquisition" in nested.stderr
