"""CPU: the device x87 long-double emulation (csrc/mx_x87.hpp), compiled for
the host, agrees bit-for-bit with the host's real x87 add/mul/compare over a
randomized sweep (normals, denormals, pseudo-denormals, NaN/inf, exact
cancellation, near-equal exponents)."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.skipif(shutil.which("g++") is None, reason="no host C++ compiler")
def test_x87_emulation_matches_host_x87(tmp_path):
    exe = tmp_path / "x87_check"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(ROOT, "zhpe-ompi_amd", "csrc"),
                    os.path.join(ROOT, "tests", "native", "x87_check.cpp"), "-o", str(exe)], check=True)
    r = subprocess.run([str(exe), "400000"], capture_output=True, text=True)
    assert r.returncode == 0, r.stdout[-2000:]
