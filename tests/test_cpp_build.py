"""CPU: the C++ mirror header compiles and links against librlnc_hip.so (no device call is made)."""
import os
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cpp_mirror_compiles_and_links(tmp_path):
    exe = tmp_path / "t"
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I" + os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "cpp", "test_full_api.cpp"), "-L" + os.path.join(ROOT, "rlnc_amd"),
                           "-lrlnc_hip", "-pthread", "-o", str(exe)])
    assert exe.exists()
