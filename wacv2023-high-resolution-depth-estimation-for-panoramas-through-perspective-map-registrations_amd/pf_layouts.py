"""Tile layouts: viewing windows (FOVs) and valid ranges, built with the reference's float32
rounding so the drop-in receives bit-identical window parameters.

* ``leres_layout`` is the active "5-fold for LeReS" table of ``Main.cpp:788-843``.
* ``band_layout`` generalises the same generator pattern: azimuth sectors x
  zenith bands over [25, 155] degrees, FOV = (a_i - m, a_{i+1} + m, z_lo - zm, z_hi + zm) and range
  = (a_{i+1}, a_i, z_lo, z_hi) built exactly as ``Main.cpp:790-843`` builds them.
* ``ZENITH_RANGE`` is ``g_zenith_range`` (``Depth.cpp:22``).

Angles are radians, stored as numpy float32 arrays of shape (ntiles, 4).
"""
from dataclasses import dataclass

import numpy as np

MYPI = 3.14159265359  # Basic.h:11 (not exact pi)


def D2R(a):
    """Basic.h:14 -- ((a)/180.0*MYPI) in double."""
    return (a / 180.0) * MYPI


def f32(x):
    return np.float32(x)


ZENITH_RANGE = (f32(D2R(26)), f32(D2R(154)))  # Depth.cpp:22 Vec2f(D2R(26), D2R(154))
RANGE_CAP = D2R(359.9)  # Depth.cpp:783-784 MIN2(range, D2R(359.9)) (double compare)


@dataclass
class Layout:
    name: str
    fovs: np.ndarray     # (n,4) float32 {azi_left, azi_right, zen_top, zen_down}
    ranges: np.ndarray   # (n,4) float32 {azi_left, azi_right, zen_up, zen_down}, as passed in
    tile_w: np.ndarray   # (n,) int32
    tile_h: np.ndarray   # (n,) int32

    @property
    def ntiles(self):
        return int(self.fovs.shape[0])

    def capped_ranges(self):
        """The ranges MergeDepthMaps stores in each pmap (Depth.cpp:783-786)."""
        r = self.ranges.copy()
        for i in range(r.shape[0]):
            for k in (0, 1):
                v = float(r[i, k])
                r[i, k] = f32(v if v < RANGE_CAP else RANGE_CAP)
        return r


def _sector_edges(margin, a_lo_deg, a_hi_deg):
    lo = f32(D2R(a_lo_deg) - float(margin))   # float azi00 = D2R(0) - margin;
    hi = f32(D2R(a_hi_deg) + float(margin))   # float azi01 = D2R(72) + margin;
    return lo, hi


def leres_layout(tile_w=1024, tile_h=988):
    """Main.cpp:788-843 (active block): 5 sectors x 3 bands, FOV zen 18-94/52-128/86-162."""
    margin = f32(D2R(3))
    sectors = [_sector_edges(margin, 72 * i, 72 * (i + 1)) for i in range(5)]
    fov_z = [(D2R(18), D2R(94)), (D2R(52), D2R(128)), (D2R(86), D2R(162))]
    rng_z = [(D2R(25), D2R(60)), (D2R(60), D2R(120)), (D2R(120), D2R(155))]
    fovs, ranges = [], []
    for (z0, z1) in fov_z:
        for (a0, a1) in sectors:
            fovs.append((a0, a1, f32(z0), f32(z1)))
    for (z0, z1) in rng_z:
        for (a0, a1) in sectors:
            ranges.append((a1 - margin, a0 + margin, f32(z0), f32(z1)))  # float - float
    n = len(fovs)
    return Layout("leres5x3", np.array(fovs, np.float32), np.array(ranges, np.float32),
                  np.full(n, tile_w, np.int32), np.full(n, tile_h, np.int32))


def band_layout(n_az, n_bands, tile_w, tile_h, margin_deg, zmargin_deg, name=None,
                z_lo=25.0, z_hi=155.0):
    """SURVEY.md Appendix C generator (same pattern as Main.cpp:790-843)."""
    margin = f32(D2R(margin_deg))
    step = 360.0 / n_az
    sectors = [_sector_edges(margin, step * i, step * (i + 1)) for i in range(n_az)]
    zstep = (z_hi - z_lo) / n_bands
    fovs, ranges = [], []
    for j in range(n_bands):
        zl, zh = z_lo + zstep * j, z_lo + zstep * (j + 1)
        for (a0, a1) in sectors:
            fovs.append((a0, a1, f32(D2R(zl - zmargin_deg)), f32(D2R(zh + zmargin_deg))))
            ranges.append((a1 - margin, a0 + margin, f32(D2R(zl)), f32(D2R(zh))))
    n = len(fovs)
    return Layout(name or f"band{n_az}x{n_bands}", np.array(fovs, np.float32),
                  np.array(ranges, np.float32), np.full(n, tile_w, np.int32),
                  np.full(n, tile_h, np.int32))


def config_layout(cfg):
    """Layouts of BASELINE.json's configs."""
    if cfg == "C1":
        return band_layout(3, 2, 256, 256, 10, 24, "C1:3x2@256")
    if cfg in ("C2", "C3", "C4"):
        return band_layout(5, 4, 512, 512, 3, 12, "C2:5x4@512")
    if cfg == "C5":
        return band_layout(10, 8, 1024, 1024, 3, 8, "C5:10x8@1024")
    if cfg == "LERES":
        return leres_layout()
    raise ValueError(cfg)


CONFIGS = {
    # name: (out_w, emap_w, layout)
    "C1": (512, 128),
    "C2": (2048, 512),
    "C5": (8192, 2048),
}
