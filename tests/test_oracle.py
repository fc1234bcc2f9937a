"""CPU tests of the oracle (the checker the HIP path is held to).

The reference ships no tests or golden vectors for this path and cannot be built here
(pf_oracle.h), so the oracle is pinned by the structural facts SURVEY.md measured on the compiled
reference (section 6, Appendix A/C) and by independent re-derivations (numpy lstsq for the
registration, a numpy Jacobi for the sweep, the committed regression fixture).
"""
import os
import sys

import numpy as np
import pytest

import pf_layouts as PL
import pf_synth
import pyoracle as O

ZR = PL.ZENITH_RANGE
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden", "c1_merge.npz")


def test_zenith_range_constant():
    # Depth.cpp:22 g_zenith_range(D2R(26), D2R(154)) stored as Vec2f
    assert ZR[0] == np.float32(26 / 180.0 * 3.14159265359)
    assert ZR[1] == np.float32(154 / 180.0 * 3.14159265359)


@pytest.mark.parametrize("out_w,expect", [
    (512, [(128, 9, 55), (256, 18, 110), (512, 36, 220)]),
    (2048, [(512, 36, 220), (1024, 73, 439), (2048, 147, 877)]),
    (8192, [(1024, 73, 439), (2048, 147, 877), (4096, 295, 1753), (8192, 591, 3505)]),
])
def test_level_bands_match_survey(out_w, expect):
    """SURVEY.md Appendix A item 2 (probe of the compiled reference)."""
    got = []
    for level in range(O.num_levels(out_w)):
        lv = O.level_dims(out_w, out_w // 2, ZR, level)
        got.append((lv.w, lv.h0, lv.h1))
    assert got == expect
    iters = [O.level_dims(out_w, out_w // 2, ZR, l).iters for l in range(O.num_levels(out_w))]
    assert iters == ([200, 100, 50] if out_w < 4096 else [200, 150, 100, 50])


def _oops_and_seams(cfg, out_w):
    lay = PL.config_layout(cfg)
    tiles, total = O.make_tiles(lay)
    data = np.zeros(total, np.float32)
    oops, seams, covered = 0, [], []
    for level in range(O.num_levels(out_w)):
        lv = O.level_dims(out_w, out_w // 2, ZR, level)
        Ls, n, o, _ = O.targets(tiles, data, lv)
        oops += o
        covered.append(int((n > 0).sum()))
        if n[:, lv.w - 1].any():
            seams.append(lv.w)
        assert n.max() <= 2
    return oops, seams, covered


def test_leres_oops_counts_match_survey():
    """58 out-of-tile taps at 512-wide output, 0 at 2048."""
    assert _oops_and_seams("LERES", 512)[0] == 58
    assert _oops_and_seams("LERES", 2048)[0] == 0


def test_seam_quirk_widths_match_survey():
    """seam at widths 128..1024 (every C1 level, C2 levels 0-1)."""
    assert _oops_and_seams("C1", 512)[1] == [128, 256, 512]
    assert _oops_and_seams("C2", 2048)[1] == [512, 1024]


def test_appendix_c_layouts_have_no_oops_and_survey_coverage():
    oops, _, covered = _oops_and_seams("C2", 2048)
    assert oops == 0
    # ~93.5k / 373.4k / 1.493M covered pixels per level at C2
    assert abs(covered[0] - 93.5e3) < 500 and abs(covered[1] - 373.4e3) < 2000
    assert abs(covered[2] - 1.493e6) < 5000
    assert _oops_and_seams("C1", 512)[0] == 0


def test_leres_layout_values():
    """Main.cpp:790-843: range 0 = (72 deg, 0 deg, 25, 60); FOV 0 = (-3, 75, 18, 94)."""
    lay = PL.leres_layout()
    deg = np.degrees(lay.ranges.astype(np.float64) * np.pi / 3.14159265359)
    assert np.allclose(deg[0], [72, 0, 25, 60], atol=1e-4)
    assert np.allclose(deg[14], [360, 288, 120, 155], atol=1e-4)
    fdeg = np.degrees(lay.fovs.astype(np.float64) * np.pi / 3.14159265359)
    assert np.allclose(fdeg[0], [-3, 75, 18, 94], atol=1e-4)
    capped = lay.capped_ranges()
    assert capped[4, 0] == np.float32(359.9 / 180.0 * 3.14159265359)


def test_sph_to_2d_inverts_to_spherical_coord():
    lay = PL.config_layout("C2")
    tiles, _ = O.make_tiles(lay)
    import ctypes as C
    L = O.lib()
    out = (C.c_float * 2)()
    back = (C.c_float * 2)()
    for p in (0, 7, 19):
        for (x, y) in ((0.1, 0.2), (0.5, 0.5), (0.9, 0.75)):
            L.pfo_to_spherical_coord(C.byref(tiles[p]), x, y, out)
            L.pfo_sph_to_2d(C.byref(tiles[p]), out[0], out[1], back)
            assert abs(back[0] - x) < 2e-5 and abs(back[1] - y) < 2e-5


def test_registration_matches_lstsq():
    lay = PL.config_layout("C1")
    tiles, total = O.make_tiles(lay)
    seeds = pf_synth.seeds_for(1)
    emap = pf_synth.baseline_emap(seeds, 128, 64)[0].numpy()
    gt = pf_synth.scene_depth(seeds, 512, 256)[0].numpy()
    data = O.warp_depth(gt, tiles, total, O.responses(pf_synth.responses(seeds, lay.ntiles)))
    for p in range(lay.ntiles):
        xs, ys, cols, rows = O.reg_samples(tiles[p], data, emap, ZR)
        assert xs.size == (cols + 1) * (rows + 1)
        assert xs.min() >= 1e-4 and xs.max() <= 1 - 1e-4
        c64, abcd, deg = O.register_tile(tiles[p], data, emap, ZR, solver="normal")
        assert deg == 3
        A = np.stack([xs ** 3, xs ** 2, xs, np.ones_like(xs)], 1)
        sol, *_ = np.linalg.lstsq(A, ys, rcond=None)
        assert np.max(np.abs(A @ c64 - A @ sol)) < 1e-6
        assert np.array_equal(abcd, c64.astype(np.float32))


def test_registration_rank_deficient_falls_back():
    lay = PL.config_layout("C1")
    tiles, total = O.make_tiles(lay)
    data = np.full(total, 0.5, np.float32)  # constant tile: only the constant term is defined
    emap = np.full((64, 128), 0.25, np.float32)
    c64, abcd, deg = O.register_tile(tiles[0], data, emap, ZR, solver="normal")
    assert deg == 0 and abs(c64[3] - 0.25) < 1e-12 and not c64[:3].any()
    # the reference's solver (Ceres LM, damped) needs no fallback: it stops at a point that fits
    c64, abcd, deg = O.register_tile(tiles[0], data, emap, ZR, solver="lm")
    assert deg == 3
    x = 0.5
    assert abs(((c64[0] * x + c64[1]) * x + c64[2]) * x + c64[3] - 0.25) < 1e-5


def _numpy_jacobi(buf, Lnorm, lv, iters):
    marker = np.uint32(O.lib().pfo_nan_marker())
    b = buf.astype(np.float32).ravel().copy()
    L = Lnorm.ravel()
    w = lv.w
    idx = np.arange(lv.h0 * w, (lv.h1 + 1) * w)
    win = L[idx].view(np.uint32) != marker
    reg = np.float32(1e-4)
    reg_ = np.float32(1) - reg
    q = np.float32(-0.25)
    for _ in range(iters):
        cur = np.zeros(idx.size, np.float32)
        cur = cur + b[idx - 1] * q
        cur = cur + b[idx - w] * q
        cur = cur + b[idx]
        cur = cur + b[idx + w] * q
        cur = cur + b[idx + 1] * q
        cur = np.where(win, cur, np.float32(0))
        tgt = np.where(win, L[idx], np.float32(0))
        t = b[idx] + (tgt - cur) * np.float32(0.5)
        v = t * reg_ + b[idx] * reg
        b[idx] = np.clip(v, 0, 1)
    return b.reshape(lv.h, lv.w)


def test_jacobi_matches_numpy_restatement():
    lay = PL.config_layout("C1")
    tiles, total = O.make_tiles(lay)
    rs = np.random.RandomState(1)
    data = rs.rand(total).astype(np.float32)
    lv = O.level_dims(512, 256, ZR, 0)
    Ls, n, _, _ = O.targets(tiles, data, lv)
    Ln = O.normalize(Ls, n, lv)
    seed = rs.rand(lv.h, lv.w).astype(np.float32)
    a = O.jacobi(seed, Ln, lv, 7)
    b = _numpy_jacobi(seed, Ln, lv, 7)
    assert np.array_equal(a.view(np.uint32), b.view(np.uint32))
    # rows outside the band never change
    assert np.array_equal(a[: lv.h0], seed[: lv.h0]) and np.array_equal(a[lv.h1 + 1:], seed[lv.h1 + 1:])


def test_quantize_truncates():
    v = np.array([[0.0, 1.0, 0.5, -0.2, 1.3, 1.0 / 65535.0 * 0.999]], np.float32)
    q = O.quantize(v)
    assert q.tolist() == [[0, 65535, 32767, 0, 65535, 0]]


def test_threads_do_not_change_output():
    lay = PL.config_layout("C1")
    tiles, total = O.make_tiles(lay)
    seeds = pf_synth.seeds_for(1, 99)
    emap = pf_synth.baseline_emap(seeds, 128, 64)[0].numpy()
    rs = np.random.RandomState(3)
    data = rs.rand(total).astype(np.float32)
    O.set_threads(1)
    a, _ = O.solve_depth_all(emap, tiles, data, 512, ZR)
    O.set_threads(4)
    b, _ = O.solve_depth_all(emap, tiles, data, 512, ZR)
    assert np.array_equal(a, b)


def test_golden_fixture_regression():
    """The committed C1 fixture (tools/make_golden.py) still reproduces bit for bit."""
    g = np.load(GOLDEN)
    lay = PL.config_layout("C1")
    tiles, total = O.make_tiles(lay)
    emap = g["emap_u16"].astype(np.float32) / np.float32(65535.0)
    data = g["tiles_u8"].astype(np.float32).ravel() / np.float32(255.0)
    out, abcd = O.merge(emap, tiles, data.copy(), 512, ZR)
    assert np.array_equal(abcd, g["abcd"])
    assert np.array_equal(out, g["out_u16"])
    import hashlib
    for level in range(3):
        lv = O.level_dims(512, 256, ZR, level)
        got = hashlib.sha256(O.probe_taps(tiles, lv).tobytes()).digest()
        assert got == g[f"taps_sha256_l{level}"].tobytes()


def test_golden_large_regression():
    """The committed 4-level checksums (tools/make_golden_large.py): the W4096 case is re-run
    here in full (SHA-256 of the u16 output and its strided subsample); the C5 case is checked
    on the GPU box (tests/test_gpu_configs.py), which runs the oracle beside the kernel."""
    import hashlib
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_golden_large as G
    g = np.load(os.path.join(ROOT, "tests", "golden", "large_merge.npz"))
    O.set_threads(min(8, os.cpu_count() or 1))
    lay, tiles, emap, data, out_w = G.case_inputs("W4096")
    assert hashlib.sha256(np.concatenate([emap.ravel(), data.ravel()]).tobytes()).digest() == \
        g["W4096_in_sha256"].tobytes()
    out, abcd = O.merge(emap, tiles, data.copy(), out_w, ZR)
    assert np.array_equal(abcd, g["W4096_abcd"])
    assert np.array_equal(out.ravel()[::int(g["stride"])], g["W4096_out_sub"])
    assert hashlib.sha256(out.tobytes()).digest() == g["W4096_out_sha256"].tobytes()


def test_layout_coverage_counts():
    """Per-pixel tile coverage of the BASELINE layouts (the sharded fusion's exactness argument,
    pf_dist.py): at most 2 for C1, C2 and LeReS at every level; the C5 layout has exactly 7
    pixels per level covered by 4 tiles (column w/2, where the float-rounded 180-degree sector
    edges round to the same column, on the shared rows of two zenith bands)."""
    for cfg, out_w in (("C1", 512), ("C2", 2048), ("LERES", 2048), ("C5", 8192)):
        lay = PL.config_layout(cfg)
        tiles, total = O.make_tiles(lay)
        data = np.zeros(total, np.float32)
        for level in range(O.num_levels(out_w)):
            lv = O.level_dims(out_w, out_w // 2, ZR, level)
            _, n, _, _ = O.targets(tiles, data, lv)
            many = np.argwhere(n > 2)
            if cfg != "C5":
                assert n.max() <= 2, (cfg, level)
            else:
                assert n.max() == 4 and len(many) == 7, (level, len(many))
                assert set(many[:, 1].tolist()) == {lv.w // 2}


def test_oracle_smoothing_restatement():
    """SolveDepthBySmoothing (Depth.cpp:1773-1878): pixels no tile covers stay 0 (the poles, and
    column 0: every box stops before x1 = 0), smoothing never leaves the range of its inputs, and
    a zenith range whose stencil leaves the buffer is refused (the reference reads out of
    bounds there)."""
    lay = PL.config_layout("C1")
    tiles, total = O.make_tiles(lay)
    data = np.random.default_rng(3).uniform(0.2, 0.8, total).astype(np.float32)
    out = O.solve_smoothing(tiles, data, 512, 256, PL.ZENITH_RANGE)
    again = O.solve_smoothing(tiles, data, 512, 256, PL.ZENITH_RANGE)
    assert np.array_equal(out, again)
    assert out[0].max() == 0 and out[-1].max() == 0  # the poles: outside every tile box
    assert out[:, 0].max() == 0
    covered = out[40:216, 1:]
    assert covered.max() <= int(0.8 * 65535) and (covered >= int(0.2 * 65535) - 1).mean() > 0.95
    with pytest.raises(ValueError):
        O.solve_smoothing(tiles, data, 512, 256, (0.0, PL.ZENITH_RANGE[1]))
