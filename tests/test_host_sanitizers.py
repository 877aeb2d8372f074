"""The C++ host runtime under sanitizers: tools/host_selftest.cpp (randomized documents through
the ICU oracle, the rule segmenter, the device-algorithm emulation, multi-threaded batch
resolution/assembly, JSON and HTML decoding) built with AddressSanitizer+UBSan and with
ThreadSanitizer. Host code only (GPU sanitizers are not available on the MI355X pool)."""
import glob
import os
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = [pytest.mark.slow,
              pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")]


def build_and_run(tmp_path, flags, ndocs):
    srcs = [s for s in sorted(glob.glob(os.path.join(REPO, "csrc", "host", "*.cpp"))) if not s.endswith("module.cpp")]
    exe = str(tmp_path / "selftest")
    subprocess.run(["g++", "-std=c++17", "-O1", "-g", *flags, os.path.join(REPO, "tools", "host_selftest.cpp"), *srcs,
                    "-licuuc", "-lpthread", "-o", exe], check=True, capture_output=True, timeout=600)
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=1:abort_on_error=1", UBSAN_OPTIONS="halt_on_error=1",
               TSAN_OPTIONS="halt_on_error=1")
    r = subprocess.run([exe, str(ndocs)], capture_output=True, text=True, timeout=600, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert "0 failures" in r.stdout


def test_asan_ubsan(tmp_path):
    build_and_run(tmp_path, ["-fsanitize=address,undefined", "-fno-omit-frame-pointer",
                             "-fno-sanitize-recover=undefined"], 600)


def test_tsan(tmp_path):
    build_and_run(tmp_path, ["-fsanitize=thread"], 200)
