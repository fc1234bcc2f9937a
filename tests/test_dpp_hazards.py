"""The built device code has no DPP read-after-write hazard (CPU, no GPU needed).

Some DPP instructions come from inline asm (v_fmac_f32_dpp in pf_jacobi.hip / pf_jres.hip), which
the compiler's hazard recognizer does not inspect: a VGPR written by a VALU instruction and read
through DPP by one of the next two instructions, with no s_nop between, reads a stale value on
gfx9.  tools/dpp_hazards.py disassembles every device object of the build and checks it."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BUILD = os.path.join(ROOT, "wacv2023-high-resolution-depth-estimation-for-panoramas-through-"
                           "perspective-map-registrations_amd", "build")


@pytest.mark.skipif(not os.path.exists("/opt/rocm/lib/llvm/bin/llvm-objdump")
                    or not os.path.isdir(BUILD), reason="needs the ROCm LLVM tools and the build")
def test_no_dpp_read_after_write_hazard():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "dpp_hazards.py"), BUILD],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "pf_jacobi_t10.o" in r.stdout and "pf_jres.o" in r.stdout
