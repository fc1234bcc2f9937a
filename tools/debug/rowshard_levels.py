"""Debug: where does the row-sharded fusion (threads on one GPU) differ from the one-GPU
per-level path?  Prints, per level, the rows whose buffer differs."""
import os
import sys
import threading

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "wacv2023-high-resolution-depth-estimation-for-panoramas-through-perspective-map-registrations_amd"))
import numpy as np
import torch

import panofuse
import pf_dist
import pf_layouts as PL
import pf_synth
from test_gpu_rowshard import ThreadComm

DEV = "cuda:0"
ZR = PL.ZENITH_RANGE
world = int(sys.argv[1]) if len(sys.argv) > 1 else 2
lay = PL.config_layout("C2")
out_w, ew = 2048, 512
seeds = pf_synth.seeds_for(1, 20261015 + 11)
gt = pf_synth.scene_depth(seeds, out_w, out_w // 2, DEV).contiguous()
emap = pf_synth.baseline_emap(seeds, ew, ew // 2, DEV).contiguous()
fz = panofuse.Fuser(0)
fz.set_tiles(lay)
tiles = torch.zeros((1, fz.tile_elems), dtype=torch.float32, device=DEV)
fz.warp_depth(gt, tiles, panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), DEV))
coeffs = torch.zeros((1, lay.ntiles, 4), dtype=torch.float32, device=DEV)
fz.register(emap, tiles, ZR, apply=False, coeffs=coeffs)
# one-GPU per-level reference buffers
ref_levels = []
prev = None
for level in range(3):
    w, h = panofuse.level_info(out_w, out_w // 2, ZR, level)[:2]
    buf = torch.zeros(w * h, dtype=torch.float32, device=DEV)
    fz.fuse_seed(emap if level == 0 else None, prev, out_w, ZR, level, buf)
    ls, cn = torch.zeros_like(buf), torch.zeros_like(buf)
    fz.fuse_partial(tiles, coeffs[0], 0, lay.ntiles, out_w, ZR, level, ls, cn)
    fz.fuse_finish_level(ls, cn, out_w, ZR, level, buf)
    ref_levels.append(buf.clone())
    prev = buf
torch.cuda.synchronize()

got_levels = {}


class Rec(pf_dist.HipRowShardBackend):
    def border(self, level, prev, a, b):
        if level > 0 and self.rank == 0:
            got_levels[level - 1] = prev.clone()
        super().border(level, prev, a, b)


comm = ThreadComm(world)
outs = [None] * world


def main(r):
    f = panofuse.Fuser(0)
    f.set_tiles(lay)
    out = torch.zeros(out_w * (out_w // 2), dtype=torch.int16, device=DEV)
    be = Rec(f, emap, tiles, coeffs[0], out_w, ZR, out)
    be.rank = r
    if r == 0:
        for lv in range(3):
            print("plan", lv, be.plan(lv, world), be.dims(lv), flush=True)
    pf_dist.fuse_row_sharded(be, 3, lay.ntiles, r, world, comm.rank(r))
    torch.cuda.synchronize()
    outs[r] = out


th = [threading.Thread(target=main, args=(r,)) for r in range(world)]
[t.start() for t in th]
[t.join() for t in th]
for lv in (0, 1):
    w, h, h0, h1 = panofuse.level_info(out_w, out_w // 2, ZR, lv)[:4]
    d = (got_levels[lv].view(h, w) != ref_levels[lv].view(h, w)).sum(1).cpu().numpy()
    rows = np.nonzero(d)[0]
    print("level", lv, "band", h0, h1, "bands", [pf_dist.band_rows(h0, h1, r, world) for r in range(world)],
          "differing rows", rows[:40], "count", int(d.sum()))
ref16 = (ref_levels[2].clamp(0, 1) * 65535.0).to(torch.int32)
w, h, h0, h1 = panofuse.level_info(out_w, out_w // 2, ZR, 2)[:4]
o = outs[0].view(h, w).to(torch.int32) & 0xFFFF
d = (o != ref16.view(h, w)).sum(1).cpu().numpy()
print("level 2 band", h0, h1, [pf_dist.band_rows(h0, h1, r, world) for r in range(world)], "rows", np.nonzero(d)[0][:40], int(d.sum()))
# the fused one-GPU pipeline (side stream) as the test's reference
ref2 = torch.zeros((1, out_w // 2, out_w), dtype=torch.int16, device=DEV)
fz.fuse(emap, tiles, ref2, ZR, coeffs=coeffs)
torch.cuda.synchronize()
r2 = ref2[0].to(torch.int32) & 0xFFFF
d = (r2 != ref16.view(h, w)).sum(1).cpu().numpy()
print("fuse() vs per-level path: rows", np.nonzero(d)[0][:40], int(d.sum()))
d = (o != r2).sum(1).cpu().numpy()
print("sharded vs fuse(): rows", np.nonzero(d)[0][:40], int(d.sum()))
