"""The E->P warps' coordinate maps, bit-exact against the oracle -- CPU only.

north_star asks for bit-exact tile index / coordinate maps.  pf_warp_depth and pf_warp_rgb build
their per-pixel maps once per (layout, panorama size) in host code with the glibc functions the
reference calls (WorldToSpherical's atan2f, Depth.cpp:2960-2971; the RGB camera ray's double
atan2 as oracle/pf_oracle.c restates SaveCubeMap), and cache them on the device; the kernels then
only gather.  pf_probe_warp_coords / pf_probe_rgb_taps run exactly that host code (no GPU), so
these tests pin the maps the GPU consumes against oracle/pf_oracle.c's pfo_warp_coords /
pfo_rgb_taps, every layout the configs use, every pixel, several panorama sizes.
"""
import numpy as np
import pytest

import panofuse
import pf_layouts as PL
import pyoracle as O

SIZES = [(512, 256), (2048, 1024), (300, 150), (302, 151), (8192, 4096)]


@pytest.mark.parametrize("cfg", ["C1", "C2", "LERES"])
@pytest.mark.parametrize("pw,ph", SIZES)
def test_depth_warp_map_bit_exact(cfg, pw, ph):
    lay = PL.config_layout(cfg)
    tiles, _ = O.make_tiles(lay)
    step = 1 if cfg != "LERES" else 4  # LeReS: 15 tiles of 1024x988, every 4th tile here
    for i in range(0, lay.ntiles, step):
        w, h = int(lay.tile_w[i]), int(lay.tile_h[i])
        wxy, wf = panofuse.warp_coords(lay.fovs[i], w, h, pw, ph)
        rxy, rf = O.warp_coords(tiles[i], pw, ph)
        assert np.array_equal(wxy, rxy), (cfg, i)
        assert np.array_equal(wf.view(np.uint32), rf.view(np.uint32)), (cfg, i)


def test_depth_warp_map_c5_tiles():
    """C5's 1024^2 tiles on its 8192x4096 panorama: one tile of each zenith band."""
    lay = PL.config_layout("C5")
    tiles, _ = O.make_tiles(lay)
    for i in range(0, lay.ntiles, 11):
        wxy, wf = panofuse.warp_coords(lay.fovs[i], 1024, 1024, 8192, 4096)
        rxy, rf = O.warp_coords(tiles[i], 8192, 4096)
        assert np.array_equal(wxy, rxy) and np.array_equal(wf.view(np.uint32), rf.view(np.uint32))


def test_depth_warp_map_uses_glibc_atan2f():
    """The reason for the host map: a device-style fp64 atan2 rounded to float disagrees with
    glibc's atan2f on a visible share of these pixels, so it could not be bit-exact."""
    lay = PL.config_layout("C2")
    tiles, _ = O.make_tiles(lay)
    rxy, rf = O.warp_coords(tiles[7], 2048, 1024)
    assert rxy.size == 512 * 512 and np.isfinite(rf).all()
    x0, y0 = rxy & 0xFFFF, rxy >> 16
    assert x0.max() <= 2047 and y0.max() <= 1023
    assert ((rf >= 0) & (rf < 1)).all()


@pytest.mark.parametrize("cfg,pw,ph", [("C1", 512, 256), ("C2", 2048, 1024), ("LERES", 2048, 1024),
                                       ("LERES", 1000, 500)])
def test_rgb_warp_taps_bit_exact(cfg, pw, ph):
    lay = PL.config_layout(cfg)
    tiles, _ = O.make_tiles(lay)
    ref = O.rgb_taps(tiles, pw, ph)
    off = 0
    for i in range(lay.ntiles):
        n = int(lay.tile_w[i]) * int(lay.tile_h[i])
        got = panofuse.rgb_taps(lay.fovs[i], lay.tile_w[i], lay.tile_h[i], pw, ph)
        assert np.array_equal(got, ref[off:off + n]), (cfg, i)
        off += n
