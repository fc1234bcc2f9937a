"""Scan the gfx950 code of libpanofuse's objects for DPP read-after-write hazards.

The Jacobi and resident kernels issue some DPP instructions from inline asm (v_fmac_f32_dpp: the
neighbour lane's value read inside the FMA, which hipcc's DPP combiner does not form), and the
compiler's hazard recognizer does not look inside inline asm.  On gfx9 a VALU write of a VGPR
followed by a DPP read of it needs two wait states in between.  This disassembles every device
object under the build directory (the .hip_fatbin bundle, llvm-objdump) and reports each DPP
instruction whose DPP source was written by one of the two preceding instructions with no
s_nop between.  Exit status 1 if any is found.

    python3 tools/dpp_hazards.py [build_dir]
"""
import glob
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"


def disasm(obj, tmp):
    fb = os.path.join(tmp, "fb.bin")
    co = os.path.join(tmp, "dev.co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fb}", obj,
                    os.path.join(tmp, "junk.o")], check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", "--unbundle", f"--input={fb}",
                    f"--output={co}", "--targets=hipv4-amdgcn-amd-amdhsa--gfx950"],
                   check=True, capture_output=True)
    out = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--mcpu=gfx950", "--no-show-raw-insn",
                          co], check=True, capture_output=True, text=True).stdout
    return out


def vregs(op):
    """VGPR numbers named by one operand (v7, v[4:5])."""
    m = re.match(r"v\[(\d+):(\d+)\]", op)
    if m:
        return set(range(int(m.group(1)), int(m.group(2)) + 1))
    m = re.match(r"v(\d+)$", op)
    return {int(m.group(1))} if m else set()


def scan(text):
    bad, ndpp = [], 0
    lines = [ln.strip() for ln in text.splitlines()]
    insts = [ln for ln in lines if ln and not ln.endswith(":") and not ln.startswith(("<", "Disass", ";"))]
    insts = [re.sub(r"\s*//.*$", "", i) for i in insts]
    for i, ins in enumerate(insts):
        parts = ins.split(None, 1)
        if len(parts) < 2 or "_dpp" not in parts[0] and "quad_perm" not in ins and "row_" not in ins \
                and "wave_" not in ins:
            continue
        ndpp += 1
        ops = [o.strip() for o in parts[1].split(",")]
        src = vregs(ops[1]) if len(ops) > 1 else set()
        for j in (i - 1, i - 2):
            if j < 0:
                break
            p = insts[j].split(None, 1)
            if p[0].startswith("s_nop"):
                break
            if p[0].startswith("v_") and len(p) > 1:
                dst = vregs(p[1].split(",")[0].strip())
                if dst & src:
                    bad.append((insts[j], ins))
                    break
            if p[0].startswith("s_nop") or not p[0].startswith(("v_", "s_")):
                continue
    return ndpp, bad


def main():
    bdir = sys.argv[1] if len(sys.argv) > 1 else os.path.join(
        os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
        "wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-"
        "registrations_amd", "build")
    total_bad = 0
    with tempfile.TemporaryDirectory() as tmp:
        for obj in sorted(glob.glob(os.path.join(bdir, "*.o"))):
            try:
                text = disasm(obj, tmp)
            except subprocess.CalledProcessError:
                continue  # no device code in this object
            n, bad = scan(text)
            total_bad += len(bad)
            print(f"{os.path.basename(obj):28s} DPP instructions {n:6d}  hazards {len(bad)}")
            for w, r in bad[:5]:
                print(f"    {w}  ->  {r}")
    return 1 if total_bad else 0


if __name__ == "__main__":
    sys.exit(main())
