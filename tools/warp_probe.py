"""Warp-kernel probe on the GPU box: times pf_warp_depth (C3: 64 panoramas, 20 tiles of 512^2)
beside torch's own write/copy kernels on buffers of the same size, to separate the kernel's
gather cost from the raw HBM write rate.  Usage: python tools/warp_probe.py [--batch 64]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "wacv2023-high-resolution-depth-estimation-for-panoramas-"
                                      "through-perspective-map-registrations_amd"))


def timed(fn, reps=10):
    import torch
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--batch", type=int, default=64)
    args = ap.parse_args()
    import torch
    import panofuse
    import pf_layouts as PL
    import pf_synth
    dev = torch.device("cuda:0")
    B = args.batch
    lay = PL.config_layout("C2")
    seeds = pf_synth.seeds_for(B)
    gt = pf_synth.scene_depth(seeds, 2048, 1024, dev).contiguous()
    resp = panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), dev)
    fz = panofuse.Fuser(0)
    fz.set_tiles(lay)
    tiles = torch.empty((B, fz.tile_elems), dtype=torch.float32, device=dev)
    res = {}
    res["warp_ms"] = timed(lambda: fz.warp_depth(gt, tiles, resp))
    import hashlib
    fz.warp_depth(gt, tiles, resp)
    torch.cuda.synchronize()
    res["sha"] = hashlib.sha256(tiles.cpu().numpy().tobytes()).hexdigest()[:16]
    res["warp_noresp_ms"] = timed(lambda: fz.warp_depth(gt, tiles))
    res["fill_tiles_ms"] = timed(lambda: tiles.fill_(0.5))
    src = torch.empty_like(tiles)
    res["copy_tiles_ms"] = timed(lambda: tiles.copy_(src))
    res["read_pano_sum_ms"] = timed(lambda: gt.sum())
    wbytes = tiles.numel() * 4
    rbytes = gt.numel() * 4
    res["warp_GBps"] = (wbytes + rbytes) / (res["warp_ms"] * 1e-3) / 1e9
    res["fill_GBps"] = wbytes / (res["fill_tiles_ms"] * 1e-3) / 1e9
    res["copy_GBps"] = 2 * wbytes / (res["copy_tiles_ms"] * 1e-3) / 1e9
    res["sum_GBps"] = rbytes / (res["read_pano_sum_ms"] * 1e-3) / 1e9
    print(json.dumps(res))


if __name__ == "__main__":
    main()
