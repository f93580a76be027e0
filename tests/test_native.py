"""Build the native C++ runtime with CMake under AddressSanitizer + UBSan (host code only)
and run its test driver (csrc/tests/native_tests.cpp).  Also checks that every HIP
source cross-compiles for gfx950 through the CMake HIP path is left to build();
this test covers the host side the sanitizers can see."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("cmake") is None, reason="cmake not available")
def test_native_tests_under_asan_ubsan(tmp_path):
    build = tmp_path / "build"
    env = dict(os.environ, TMPDIR=str(tmp_path), NO_COLOR="1", ASAN_OPTIONS="detect_leaks=1:abort_on_error=0",
               UBSAN_OPTIONS="print_stacktrace=1", OMP_NUM_THREADS="4")
    gen = ["-G", "Ninja"] if shutil.which("ninja") else []
    subprocess.run(["cmake", "-S", ROOT, "-B", str(build), *gen, "-DCME_SANITIZE=ON", "-DCMAKE_BUILD_TYPE=Debug"],
                   check=True, capture_output=True, env=env, timeout=300)
    subprocess.run(["cmake", "--build", str(build), "-j", "4", "--target", "native_tests"], check=True,
                   capture_output=True, env=env, timeout=600)
    r = subprocess.run([str(build / "native_tests")], capture_output=True, text=True, env=env, timeout=600)
    tail = "\n".join((r.stdout + r.stderr).splitlines()[-30:])
    assert r.returncode == 0, tail
    assert "0 failed" in r.stdout, tail
    assert "ERROR: AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, tail
