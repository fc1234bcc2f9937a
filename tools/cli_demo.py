"""End-to-end run of the mode-0 command line on a synthetic dataset (PNG files), for the
host-buffer / file-I/O inclusive rate of the drop-in.

Writes N panoramas' inputs with the reference's naming (2048x1024 u16 gt, 512x256 u16 baseline
in hohonet naming, 15 LeReS tiles of 1024x988 u16), then runs bin/panofuse_main 0 and prints its
log plus the wall time per panorama.  Usage: python tools/cli_demo.py OUTDIR [N]"""
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "wacv2023-high-resolution-depth-estimation-for-panoramas-through-"
                         "perspective-map-registrations_amd")
sys.path[:0] = [PKG, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "tests")]

import pf_layouts as PL  # noqa: E402
import pf_synth  # noqa: E402
import pyoracle as O  # noqa: E402
from test_gpu_cli import _cround, _png16_write, _q16, MYPI  # noqa: E402


def main():
    out = sys.argv[1]
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 4
    d = {k: os.path.join(out, k) for k in ("rgb", "gt", "base", "result_hohonet", "tiles")}
    for p in d.values():
        os.makedirs(p, exist_ok=True)
    lay = PL.leres_layout(1024, 988)
    tiles_o, total = O.make_tiles(lay)
    for i in range(n):
        raw = f"pano{i:03d}_rgb"
        open(os.path.join(d["rgb"], raw + ".jpg"), "wb").write(b"\xff\xd8")
        seeds = pf_synth.seeds_for(1, 20261015 + 7 * i)
        gt = _q16(pf_synth.scene_depth(seeds, 2048, 1024)[0].numpy())
        _png16_write(os.path.join(d["gt"], raw.replace("_rgb", "_depth") + ".png"), gt)
        _png16_write(os.path.join(d["base"], raw + ".depth.png"),
                     _q16(pf_synth.baseline_emap(seeds, 512, 256)[0].numpy()))
        tq = _q16(O.warp_depth(gt.astype(np.float32) / np.float32(65535.0), tiles_o, total,
                               O.responses(pf_synth.responses(seeds, lay.ntiles))))
        off = 0
        for t in range(lay.ntiles):
            f = [_cround(float(v) / MYPI * 180.0) for v in lay.fovs[t]]
            _png16_write(os.path.join(d["tiles"], f"{raw}.{f[0]}_{f[1]}_{f[2]}_{f[3]}.png"),
                         tq[off:off + 1024 * 988].reshape(988, 1024))
            off += 1024 * 988
    cmd = [os.path.join(PKG, "bin", "panofuse_main"), "0", d["rgb"], d["gt"], d["base"],
           d["result_hohonet"], "--tiles", d["tiles"]]
    t0 = time.perf_counter()
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    dt = time.perf_counter() - t0
    print(r.stdout)
    print(f"rc={r.returncode} panoramas={n} wall={dt:.2f}s per_panorama={dt / n * 1e3:.1f} ms "
          f"(process start, HIP init, PNG decode of 15x1024x988 u16 tiles + gt + baseline, "
          f"H2D, register+fuse, D2H, PNG encode of 3 outputs, metrics)")
    return r.returncode


if __name__ == "__main__":
    sys.exit(main())
