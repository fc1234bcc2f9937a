"""LDS bank-conflict model of k_warp_depth's box reads (host only, no GPU).

For every 32x32 patch of a layout this rebuilds the staged footprint box the way k_patch_box does
(azimuth-unwrapped, origin and width in whole quads), places each pixel's bilinear corner in it at a
given row pitch, and prices the four ds_read_b32 halves of the two ds_read2_b32 per pixel (offsets 0,
1, pitch, pitch + 1) with the MI355X rule: a 32-lane group costs one LDS cycle per distinct address
on its busiest bank (MI355X_MICROARCH.md, LDS table).  Printed: mean cycles per group (1.0 = no
conflict) for lane-group shapes (32x1 = the kept kernel's one tile row per group) and pitch rules.

    python3 tools/warp_lds_sim.py [C3]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, d) for d in os.listdir(ROOT) if d.endswith("_amd")]
import panofuse  # noqa: E402
import pf_layouts as PL  # noqa: E402

PW, PH, P, CAP = 2048, 1024, 32, 4096


def group_cycles(G):
    """G: (n, 32) dword addresses -> per group the max over banks of distinct addresses."""
    k = np.sort((G % 32) * (1 << 24) + G, axis=1)
    new = np.ones_like(k, dtype=bool)
    new[:, 1:] = k[:, 1:] != k[:, :-1]
    cnt = np.zeros((G.shape[0], 32), np.int64)
    rows = np.repeat(np.arange(G.shape[0]), 32).reshape(G.shape)
    np.add.at(cnt, (rows[new], k[new] >> 24), 1)
    return cnt.max(axis=1)


def patches(cfg, step=2):
    lay = PL.config_layout(cfg)
    out = []
    for i in range(0, lay.ntiles, step):
        w, h = int(lay.tile_w[i]), int(lay.tile_h[i])
        wxy, _ = panofuse.warp_coords(lay.fovs[i], w, h, PW, PH)
        x0 = (wxy & 0xFFFF).astype(np.int64).reshape(h, w)
        y0 = (wxy >> 16).astype(np.int64).reshape(h, w)
        for Y0 in range(0, h - P + 1, P):
            for X0 in range(0, w - P + 1, P):
                xs, ys = x0[Y0:Y0 + P, X0:X0 + P], y0[Y0:Y0 + P, X0:X0 + P]
                du = xs - xs[0, 0]
                du = np.where(du > PW // 2, du - PW, du)
                du = np.where(du < -(PW // 2), du + PW, du)
                a = (xs[0, 0] + du.min()) & 3
                bw = (du.max() - du.min() + 2 + a + 3) & ~3
                if bw * (ys.max() - ys.min() + 2) <= CAP:
                    out.append((bw, ys - ys.min(), du - du.min() + a))
    return out


def lane_groups(gw):
    """(rows, cols) index arrays of the 32-lane groups: gw columns x 32/gw rows."""
    gh = 32 // gw
    idx = [[(R + i // gw, C + i % gw) for i in range(32)]
           for R in range(0, P, gh) for C in range(0, P, gw)]
    a = np.array(idx)
    return a[..., 0], a[..., 1]


def mean_cycles(pl, gw, pitch_rule):
    R, C = lane_groups(gw)
    tot = n = 0
    for bw, yy, xx in pl:
        pitch = pitch_rule(bw)
        if pitch * (yy.max() + 2) > CAP:
            pitch = bw
        G = (yy * pitch + xx)[R, C]
        for off in (0, 1, pitch, pitch + 1):
            c = group_cycles(G + off)
            tot += c.sum()
            n += len(c)
    return tot / n


if __name__ == "__main__":
    pl = patches(sys.argv[1] if len(sys.argv) > 1 else "C3")
    rules = {"bw": lambda bw: bw, "odd": lambda bw: bw | 1,
             "0 mod 32": lambda bw: bw + (-bw % 32), "8 mod 32": lambda bw: bw + ((8 - bw) % 32),
             "16 mod 32": lambda bw: bw + ((16 - bw) % 32)}
    print(f"{len(pl)} patches")
    for gw in (32, 16, 8):
        print(f"{gw:2d}x{32 // gw:<2d} " + "  ".join(f"{k}: {mean_cycles(pl, gw, f):.3f}"
                                                  for k, f in rules.items()), flush=True)
