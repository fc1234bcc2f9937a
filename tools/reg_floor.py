"""The registration gather's line floor: per panorama of the C3 layout,
the distinct 128-B lines the registration samples touch -- in the tiles, and in the 512x256
baseline per tile and over the whole panorama -- against the k_register bytes PMC measures per
launch (profiles/r04/pmc_traffic.txt).  Host only: builds tools/regfloor/reg_lines.c against the
oracle (test/analysis tooling).
    python3 tools/reg_floor.py"""
import os
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle")] + [os.path.join(ROOT, d) for d in os.listdir(ROOT)
                                                  if d.endswith("_amd")]
import pf_layouts as PL  # noqa: E402
import pyoracle as O  # noqa: E402

lay = PL.config_layout("C2")
zr = PL.ZENITH_RANGE
tiles, total = O.make_tiles(lay)
d = tempfile.mkdtemp()
exe = os.path.join(d, "reg_lines")
subprocess.check_call(["gcc", "-O2", "-std=gnu11", "-ffp-contract=off", "-fopenmp", "-I",
                       os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tools", "regfloor",
                                                                  "reg_lines.c"),
                       os.path.join(ROOT, "oracle", "pf_oracle.c"),
                       os.path.join(ROOT, "oracle", "pf_oracle_lm.c"), "-lm", "-o", exe])
open(os.path.join(d, "tiles.bin"), "wb").write(bytes(tiles))
out = subprocess.check_output([exe, os.path.join(d, "tiles.bin"), str(lay.ntiles), "512", "256",
                               repr(zr[0]), repr(zr[1])], text=True)
v = dict(zip(out.split()[0::2], map(int, out.split()[1::2])))
B = 64
mb = lambda lines: lines * 128 * B / 1e6  # noqa: E731
print(out.strip())
print(f"per C3 launch (64 panoramas): samples {v['samples'] * B / 1e6:.2f} M "
      f"({v['samples'] * B * 8 / 1e6:.1f} MB of 4-B tile + 4-B baseline values)")
print(f"  tile lines {mb(v['tile_lines']):.1f} MB; baseline lines per tile {mb(v['emap_lines_per_tile_sum']):.1f} MB, "
      f"per panorama (union) {mb(v['emap_lines_union']):.1f} MB")
print(f"  floor with the baseline read once per panorama: "
      f"{mb(v['tile_lines'] + v['emap_lines_union']):.1f} MB; with it read per tile: "
      f"{mb(v['tile_lines'] + v['emap_lines_per_tile_sum']):.1f} MB")
