"""The C++ drop-in headers (include/soundmath/*.h) compile as the reference's demos use
them and link against libhuygens_hip.so (run on the GPU in tests/test_cpp_gpu.py)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "huygens_amd", "lib")
EXE = os.path.join(ROOT, "tests", "cpp", "dropin")


def build_dropin():
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Wextra", "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "tests", "cpp", "dropin.cpp"), "-o", EXE, "-L", LIB, "-lhuygens_hip",
           f"-Wl,-rpath,{LIB}", "-Wl,-rpath-link,/opt/rocm/lib", "-Wl,-rpath,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    return r


def test_dropin_headers_build():
    if not os.path.exists(os.path.join(LIB, "libhuygens_hip.so")):
        pytest.skip("libhuygens_hip.so not built (make lib)")
    r = build_dropin()
    assert r.returncode == 0, r.stderr[-3000:]
    assert "warning" not in r.stderr, r.stderr[-3000:]


@pytest.mark.parametrize("hdr", ["filterbank.h", "oscbank.h", "additive.h", "sinusoids.h", "bowl.h", "delay.h",
                                 "delaybank.h", "fourier.h", "staticSTFT.h", "granulator.h", "harmbank.h", "audio.h"])
def test_each_header_standalone(hdr, tmp_path):
    src = tmp_path / "one.cpp"
    src.write_text(f'#include "soundmath/{hdr}"\nint main() {{ return 0; }}\n')
    r = subprocess.run(["g++", "-std=c++17", "-fsyntax-only", "-I", os.path.join(ROOT, "include"), str(src)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-2000:]
