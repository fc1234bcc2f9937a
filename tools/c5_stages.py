"""Stage times of ONE panorama through pf_warp_depth + pf_merge on one context (the library's
hipEvent stage timers), plus the per-level Jacobi plans (PF_JPLAN=1 prints them on stderr).
    python3 tools/c5_stages.py [C5|C2]   (C5: 8192x4096, 80 tiles, 4 levels; C2: 2048x1024, 20 tiles)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, [os.path.join(ROOT, d) for d in os.listdir(ROOT) if d.endswith("_amd")][0])
import torch  # noqa: E402

import panofuse  # noqa: E402
import pf_layouts as PL  # noqa: E402
import pf_synth  # noqa: E402

dev = torch.device("cuda:0")
cfg = sys.argv[1] if len(sys.argv) > 1 else "C5"
out_w, ew = PL.CONFIGS[cfg] if cfg in PL.CONFIGS else (2048, 512)
lay = PL.config_layout(cfg)
zr = PL.ZENITH_RANGE
seeds = pf_synth.seeds_for(1, 20261015)
gt = pf_synth.scene_depth(seeds, out_w, out_w // 2, dev).contiguous()
emap = pf_synth.baseline_emap(seeds, ew, ew // 2, dev).contiguous()
resp = panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), dev)
fz = panofuse.Fuser(0)
fz.set_tiles(lay)
tiles = torch.zeros((1, fz.tile_elems), dtype=torch.float32, device=dev)
out = torch.empty((1, out_w // 2, out_w), dtype=torch.int16, device=dev)
co = torch.zeros((1, lay.ntiles, 4), dtype=torch.float32, device=dev)
for _ in range(2):
    fz.warp_depth(gt, tiles, resp)
    fz.merge(emap, tiles, out, zr, coeffs=co)
torch.cuda.synchronize()
fz.profile(True)
res = []
for _ in range(5):
    fz.warp_depth(gt, tiles, resp)
    fz.merge(emap, tiles, out, zr, coeffs=co)
    res.append(fz.profile_read())
fz.profile(False)
med = {k: sorted(r[k][0] for r in res)[2] for k in res[0]}
nl = panofuse.level_info(out_w, out_w // 2, zr, 0)[5]
print(json.dumps({"config": cfg, "stage_ms": med,
                  "levels": [panofuse.level_info(out_w, out_w // 2, zr, l) for l in range(nl)]}))
