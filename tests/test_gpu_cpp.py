"""GPU: the C++ mirror of rlnc::full (include/rlnc/full.hpp) — the reference's unit tests and round trips
ported to C++ (tests/cpp/test_full_api.cpp), built with g++ against librlnc_hip.so and run as a child process."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_api_mirror():
    exe = os.path.join(ROOT, "build", "test_full_api")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    subprocess.check_call(["g++", "-std=c++17", "-O2", "-Wall", "-I" + os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "test_full_api.cpp"), "-L" + os.path.join(ROOT, "rlnc_amd"),
                           "-lrlnc_hip", "-Wl,-rpath," + os.path.join(ROOT, "rlnc_amd"), "-pthread", "-o", exe])
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "all passed" in r.stdout
