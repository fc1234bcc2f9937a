"""cubic_map's clamp thresholds (csrc/pf_internal.hpp) -- CPU only.

Depth2DepthTransform (Depth.cpp:245-274) clamps X by comparing the float against the double
constants 1e-4 and 1 - 1e-4.  The library compares against the two float thresholds that decide
the same way (no f64 conversion per value in the targets gather, the smoothing source and the
transform kernels).  tests/cpp/cubic_thresholds.cpp runs the library's host copy of cubic_map
against the reference form on every one of the 2^32 float bit patterns (~20 s)."""
import os
import shutil
import subprocess

import pytest

import panofuse

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_cubic_thresholds_exhaustive(tmp_path):
    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    if not os.path.exists(hipcc):
        pytest.skip("no hipcc")
    csrc = os.path.join(os.path.dirname(os.path.dirname(panofuse.LIB_PATH)), "csrc")
    exe = tmp_path / "cubic_chk"
    r = subprocess.run([hipcc, "-O2", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-I",
                        csrc, "-x", "hip", "--offload-arch=gfx950",
                        os.path.join(ROOT, "tests", "cpp", "cubic_thresholds.cpp"), "-o",
                        str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    r = subprocess.run([str(exe)], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "0 mismatches" in r.stdout
