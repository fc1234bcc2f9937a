"""Synthetic workload for tests and benchmarks.  There are no datasets or
depth-net checkpoints offline, so every panorama is generated:

* ground truth: ray distance to an axis-aligned room box around the camera (lo in U[-3,-1]^3,
  hi in U[1,3]^3) with a mild wall relief, depth = dist/10, in [0, 1];
* baseline emap (the low-resolution UniFuse/BiFuse stand-in): the same scene at (W/4)x(H/4),
  times (1 + 0.05 sin(az) cos(zen)), plus N(0, 0.003), quantised to u16;
* tiles: produced by the E->P warp of the ground truth followed by a per-tile response
  d' = alpha d + kappa d^2 + beta + sigma u (the affine-invariant depth net stand-in), see
  pf_response in include/panofuse.h.

Generation is device-agnostic torch (CPU for tests, GPU for the benchmark); it is input plumbing,
not part of the measured path.
"""
import numpy as np

MYPI = 3.14159265359


def _scene_params(seed):
    rs = np.random.RandomState(seed & 0x7FFFFFFF)
    lo = rs.uniform(-3.0, -1.0, size=3)
    hi = rs.uniform(1.0, 3.0, size=3)
    relief = rs.uniform(0.01, 0.04)
    fa, fz = rs.randint(3, 9), rs.randint(2, 7)
    return lo, hi, relief, fa, fz


def scene_depth(seeds, w, h, device="cpu"):
    """[B, h, w] float32 depth for pixel (x, y) at az = x/(w-1)*2pi, zen = y/(h-1)*pi."""
    import torch
    x = torch.arange(w, dtype=torch.float64, device=device)
    y = torch.arange(h, dtype=torch.float64, device=device)
    az = (x / (w - 1) * 2 * MYPI)[None, :]
    zen = (y / (h - 1) * MYPI)[:, None]
    d = torch.stack([torch.sin(zen) * torch.cos(az), torch.sin(zen) * torch.sin(az),
                     torch.cos(zen).expand(h, w)], 0)
    out = []
    for s in seeds:
        lo, hi, relief, fa, fz = _scene_params(int(s))
        t = torch.full((h, w), float("inf"), dtype=torch.float64, device=device)
        for k in range(3):
            dk = d[k]
            with torch.no_grad():
                pos = torch.where(dk > 1e-12, hi[k] / dk.clamp(min=1e-12),
                                  torch.full_like(dk, float("inf")))
                neg = torch.where(dk < -1e-12, lo[k] / dk.clamp(max=-1e-12),
                                  torch.full_like(dk, float("inf")))
            t = torch.minimum(t, torch.minimum(pos, neg))
        dep = t / 10.0 * (1.0 + relief * torch.sin(fa * az) * torch.sin(fz * zen))
        out.append(dep.clamp(0.0, 1.0).to(torch.float32))
    return torch.stack(out, 0)


def baseline_emap(seeds, w, h, device="cpu"):
    """[B, h, w] float32 baseline: biased, noisy, u16-quantised low-resolution depth."""
    import torch
    gt = scene_depth(seeds, w, h, device).double()
    x = torch.arange(w, dtype=torch.float64, device=device)
    y = torch.arange(h, dtype=torch.float64, device=device)
    az = (x / (w - 1) * 2 * MYPI)[None, :]
    zen = (y / (h - 1) * MYPI)[:, None]
    bias = 1.0 + 0.05 * torch.sin(az) * torch.cos(zen)
    out = []
    for i, s in enumerate(seeds):
        g = torch.Generator(device="cpu").manual_seed(int(s) * 7 + 1)
        noise = torch.randn((h, w), generator=g, dtype=torch.float64).to(device) * 0.003
        v = (gt[i] * bias + noise).clamp(0.0, 1.0)
        q = torch.round(v * 65535.0) / 65535.0
        out.append(q.to(torch.float32))
    return torch.stack(out, 0)


def responses(seeds, ntiles):
    """(B*ntiles, 5) float64 rows (alpha, kappa, beta, sigma, seed) of the depth-net stand-in."""
    rows = []
    for s in seeds:
        rs = np.random.RandomState((int(s) * 31 + 5) & 0x7FFFFFFF)
        for t in range(ntiles):
            rows.append((rs.uniform(0.8, 1.2), rs.uniform(-0.3, 0.3), rs.uniform(-0.03, 0.03),
                         0.002, (int(s) * 1000003 + t) & 0xFFFFFFFF))
    return np.array(rows, dtype=np.float64)


def seeds_for(n, base=20261015):
    return [base + i for i in range(n)]
