"""C2 latency probe for rocprofv3 kernel traces: one 2048x1024 panorama, 20 tiles of 512^2,
warp + registration + 3-level fusion per run (bench.py's c2_latency loop), `reps` runs.

    python tools/c2_probe.py [--reps 20]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "wacv2023-high-resolution-depth-estimation-for-panoramas-"
                                      "through-perspective-map-registrations_amd"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    a = ap.parse_args()
    import torch

    import panofuse
    import pf_layouts as PL
    import pf_synth
    dev = torch.device("cuda:0")
    lay = PL.config_layout("C2")
    seeds = pf_synth.seeds_for(1, 424242)
    gt = pf_synth.scene_depth(seeds, 2048, 1024, dev).contiguous()
    emap = pf_synth.baseline_emap(seeds, 512, 256, dev).contiguous()
    resp = panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), dev)
    f = panofuse.Fuser(0)
    f.set_tiles(lay)
    tiles = torch.empty((1, f.tile_elems), dtype=torch.float32, device=dev)
    out = torch.empty((1, 1024, 2048), dtype=torch.int16, device=dev)
    coeffs = torch.empty((1, lay.ntiles, 4), dtype=torch.float32, device=dev)
    times = []
    for i in range(a.reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f.warp_depth(gt, tiles, resp)
        f.merge(emap, tiles, out, PL.ZENITH_RANGE, coeffs=coeffs)
        e1.record()
        torch.cuda.synchronize()
        if i >= 2:
            times.append(e0.elapsed_time(e1))
    times.sort()
    print(f"C2 one panorama: median {times[len(times) // 2]:.3f} ms, min {times[0]:.3f} ms "
          f"over {a.reps} runs", flush=True)


if __name__ == "__main__":
    main()
