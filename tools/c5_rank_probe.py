"""One rank's compute of the row-sharded C5 fusion (rank R of N, pf_dist.NullComm: nothing is
exchanged, so the values are not the sharded result -- only its kernels and host work), timed
with hipEvents and wall clock, for kernel traces under rocprofv3.

    python tools/c5_rank_probe.py [--rank 3] [--world 8] [--rep 2] [--reps 5]"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "wacv2023-high-resolution-depth-estimation-for-panoramas-"
                                      "through-perspective-map-registrations_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rank", type=int, default=3)
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rep", type=int, default=2)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--one-call", action="store_true",
                    help="the same panorama through pf_warp_depth + pf_merge on one context")
    a = ap.parse_args()
    import torch

    import panofuse
    import pf_dist
    import pf_layouts as PL
    import pf_synth
    dev = torch.device("cuda:0")
    out_w, ew = PL.CONFIGS["C5"]
    lay = PL.config_layout("C5")
    zr = PL.ZENITH_RANGE
    seeds = pf_synth.seeds_for(1, 20261015)
    gt = pf_synth.scene_depth(seeds, out_w, out_w // 2, dev).contiguous()
    emap = pf_synth.baseline_emap(seeds, ew, ew // 2, dev).contiguous()
    fz = panofuse.Fuser(0)
    fz.set_tiles(lay)
    t0, t1 = pf_dist.shard_range(lay.ntiles, a.rank, a.world)
    fs = panofuse.Fuser(0)
    fs.set_tiles(PL.Layout("sub", lay.fovs[t0:t1], lay.ranges[t0:t1], lay.tile_w[t0:t1],
                           lay.tile_h[t0:t1]))
    resp = panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles)[t0:t1], dev)
    tiles = torch.zeros((1, fz.tile_elems), dtype=torch.float32, device=dev)
    off = int(sum(int(lay.tile_w[i]) * int(lay.tile_h[i]) for i in range(t0)))
    mine = tiles[:, off:off + fs.tile_elems]
    coeffs = torch.zeros((lay.ntiles, 4), dtype=torch.float32, device=dev)
    out = torch.empty(out_w * (out_w // 2), dtype=torch.int16, device=dev)
    be = pf_dist.HipRowShardBackend(fz, emap, tiles, coeffs, out_w, zr, out)
    nlev = be.nlevels

    if a.one_call:
        rall = panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), dev)
        o2 = out.view(1, out_w // 2, out_w)

        def step():
            fz.warp_depth(gt, tiles, rall)
            fz.merge(emap, tiles, o2, zr, coeffs=coeffs[None])
    else:
        def step():
            fs.warp_depth(gt, mine, resp)
            fs.register(emap, mine, zr, degree=3, apply=False, coeffs=coeffs[t0:t1][None])
            pf_dist.fuse_row_sharded(be, nlev, lay.ntiles, a.rank, a.world, pf_dist.NullComm(),
                                     rep_levels=a.rep)
    step()
    torch.cuda.synchronize()
    for _ in range(a.reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        w0 = time.perf_counter()
        e0.record()
        step()
        e1.record()
        w1 = time.perf_counter()
        torch.cuda.synchronize()
        tag = "one call" if a.one_call else f"rank {a.rank}/{a.world} rep {a.rep}"
        print(f"{tag}: {e0.elapsed_time(e1):.3f} ms (events), "
              f"host enqueue {1e3 * (w1 - w0):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
