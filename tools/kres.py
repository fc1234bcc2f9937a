"""Tabulate hipcc -Rpass-analysis=kernel-resource-usage remarks: name, VGPRs, spills, occupancy.
Usage: python tools/kres.py <source.hip> [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
flt = sys.argv[2] if len(sys.argv) > 2 else ""
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
       "-fno-fast-math", "-fhip-fp32-correctly-rounded-divide-sqrt", "--cuda-device-only", "-c",
       src, "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
err = subprocess.run(cmd, capture_output=True, text=True).stderr
cur = None
rows = []
for line in err.splitlines():
    m = re.search(r"remark: +(Function Name|VGPRs|AGPRs|ScratchSize \[bytes/lane\]|Occupancy \[waves/SIMD\]|VGPRs Spill|SGPRs): (\S+)", line)
    if not m:
        continue
    k, v = m.group(1), m.group(2)
    if k == "Function Name":
        cur = {"name": v}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    if flt in r["name"]:
        print(f"{r.get('VGPRs','?'):>4} vgpr {r.get('VGPRs Spill','?'):>3} spill "
              f"{r.get('ScratchSize [bytes/lane]','?'):>4} scratch occ {r.get('Occupancy [waves/SIMD]','?')}  {r['name']}")
