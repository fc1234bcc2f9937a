"""Generate tests/golden/large_merge.npz: checksums of the oracle's MergeDepthMaps output for the
large configurations ("as SHA-256 + strided subsample").

* W4096: 4096x2048 output, 20 tiles of 1024^2 (the C2 5x4 layout at twice the resolution),
  1024x512 baseline -- the 4-level path (Depth.cpp:1423-1424, 1665-1675).
* C5: 8192x4096 output, 80 tiles of 1024^2 (10x8 layout), 2048x1024
  baseline.

Inputs are the deterministic synthetic scene (pf_synth, torch CPU fp64) warped into tiles by the
oracle (pfo_warp_depth); their SHA-256 is stored too, so a drift of the generator is told apart
from a drift of the fusion.  These are regression vectors of the oracle restatement, not outputs
of the reference (which cannot be built here; see oracle/pf_oracle.h).
Usage: python tools/make_golden_large.py
"""
import hashlib
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "wacv2023-high-resolution-depth-estimation-for-panoramas-"
                                      "through-perspective-map-registrations_amd"))
import pf_layouts as PL  # noqa: E402
import pf_synth  # noqa: E402
import pyoracle as O  # noqa: E402

# name -> (layout, out_w, emap_w, seed)
CASES = {
    "W4096": (lambda: PL.band_layout(5, 4, 1024, 1024, 3, 12, "C2@4096"), 4096, 1024, 20261015 + 41),
    "C5": (lambda: PL.config_layout("C5"), 8192, 2048, 20261015 + 55),
}
STRIDE = 97  # strided subsample of the u16 output (prime, so it walks every column phase)


def sha(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)


def case_inputs(name):
    """(layout, tiles, emap, tile_data, out_w) of a case, deterministic on any host."""
    mk, out_w, ew, seed = CASES[name]
    lay = mk()
    seeds = [seed]
    gt = pf_synth.scene_depth(seeds, out_w, out_w // 2)[0].numpy()
    emap = pf_synth.baseline_emap(seeds, ew, ew // 2)[0].numpy()
    tiles, total = O.make_tiles(lay)
    data = O.warp_depth(gt, tiles, total, O.responses(pf_synth.responses(seeds, lay.ntiles)))
    return lay, tiles, emap, data, out_w


def main():
    zr = PL.ZENITH_RANGE
    rec = {}
    for name in CASES:
        lay, tiles, emap, data, out_w = case_inputs(name)
        rec[f"{name}_in_sha256"] = sha(np.concatenate([emap.ravel(), data.ravel()]))
        out, abcd = O.merge(emap, tiles, data.copy(), out_w, zr)
        rec[f"{name}_abcd"] = abcd
        rec[f"{name}_out_sha256"] = sha(out)
        rec[f"{name}_out_sub"] = out.ravel()[::STRIDE].copy()
        print(name, out.shape, "nonzero", int((out != 0).sum()), flush=True)
    path = os.path.join(ROOT, "tests", "golden", "large_merge.npz")
    np.savez_compressed(path, stride=np.int64(STRIDE), **rec)
    print("wrote", path, os.path.getsize(path), "bytes")


if __name__ == "__main__":
    main()
