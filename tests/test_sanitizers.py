"""Host-code sanitizers over the native runtime.

tests/native/sanitize_driver.cpp builds the pybind-free cores of deepspeech_amd/runtime
(TFRecord codec incl. corrupted-input fuzzing, prefix beam search single/multi-threaded and
streaming, bucketed batch planning, the threaded mmap batch loader) twice:
  * -fsanitize=address,undefined  (memory errors, undefined behaviour)
  * -fsanitize=thread             (data races in the worker pools)
and runs each; any report fails the test (-fno-sanitize-recover). Device sanitizers
(GPU ASan / xnack+) are not available on the MI355X pool, so GPU kernels are covered by
host-side shape checks and bounded spins instead.
"""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "tests", "native", "sanitize_driver.cpp")


@pytest.mark.parametrize("san", ["address,undefined", "thread"])
def test_native_runtime_under_sanitizer(tmp_path, san):
    cxx = shutil.which("g++")
    if cxx is None:
        pytest.skip("g++ not available")
    exe = str(tmp_path / ("san_" + san.replace(",", "_")))
    cmd = [cxx, "-std=c++17", "-O1", "-g", "-fno-omit-frame-pointer", "-fsanitize=" + san,
           "-fno-sanitize-recover=all", "-pthread", SRC, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    if r.returncode != 0 and "cannot find" in (r.stderr or ""):
        pytest.skip("sanitizer runtime not installed: " + r.stderr[-200:])
    assert r.returncode == 0, r.stderr[-4000:]
    env = dict(os.environ, DS2_SAN_TMP=str(tmp_path), TSAN_OPTIONS="halt_on_error=1",
               ASAN_OPTIONS="detect_leaks=1:halt_on_error=1")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0 and "sanitize_driver ok" in r.stdout, (r.stdout[-2000:], r.stderr[-6000:])
