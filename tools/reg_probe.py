"""Registration probe on the GPU box: pf_register time at C3 (64 panoramas x 20 tiles) with the
Ceres-LM solve (default) and with the normal equations, to split k_register's time between the
moment sums and the per-tile solve.  Usage: python tools/reg_probe.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "wacv2023-high-resolution-depth-estimation-for-panoramas-"
                                      "through-perspective-map-registrations_amd"))


def main():
    import torch

    import panofuse
    import pf_layouts as PL
    import pf_synth

    dev = "cuda:0"
    B = 64
    lay = PL.config_layout("C2")
    seeds = pf_synth.seeds_for(B, 20261015)
    gt = pf_synth.scene_depth(seeds, 2048, 1024, dev).contiguous()
    emap = pf_synth.baseline_emap(seeds, 512, 256, dev).contiguous()
    resp = panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), dev)
    fz = panofuse.Fuser(0)
    fz.set_tiles(lay)
    tiles = torch.empty((B, fz.tile_elems), dtype=torch.float32, device=dev)
    fz.warp_depth(gt, tiles, resp)
    coeffs = torch.empty((B, lay.ntiles, 4), dtype=torch.float32, device=dev)
    for solver in ("lm", "normal", "lm"):
        fz.set_solver(solver)
        for _ in range(2):
            fz.register(emap, tiles, PL.ZENITH_RANGE, degree=3, apply=False, coeffs=coeffs)
        torch.cuda.synchronize()
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(10):
            fz.register(emap, tiles, PL.ZENITH_RANGE, degree=3, apply=False, coeffs=coeffs)
        b.record()
        torch.cuda.synchronize()
        print(f"{solver}: {a.elapsed_time(b) / 10 * 1e3:.1f} us per register call (B={B})")


if __name__ == "__main__":
    main()
