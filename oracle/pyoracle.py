"""ctypes binding of the CPU oracle (oracle/liboracle.so).

TEST INFRASTRUCTURE ONLY -- imported by tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg, never by the product path.  Parity unpinned (see pf_oracle.h).
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "liboracle.so")


class Tile(C.Structure):
    _fields_ = [
        ("width", C.c_int), ("height", C.c_int), ("channels", C.c_int),
        ("offset", C.c_longlong),
        ("az_left", C.c_float), ("az_right", C.c_float),
        ("zen_top", C.c_float), ("zen_down", C.c_float),
        ("ranges", C.c_float * 4),
        ("middle", C.c_float * 3), ("hedge", C.c_float * 3), ("vedge", C.c_float * 3),
        ("corner0", C.c_float * 3), ("corner1", C.c_float * 3),
        ("corner2", C.c_float * 3), ("corner3", C.c_float * 3),
    ]


class Response(C.Structure):
    _fields_ = [("alpha", C.c_float), ("kappa", C.c_float), ("beta", C.c_float),
                ("sigma", C.c_float), ("seed", C.c_uint32), ("pad", C.c_uint32)]


class Level(C.Structure):
    _fields_ = [("w", C.c_int), ("h", C.c_int), ("h0", C.c_int), ("h1", C.c_int),
                ("iters", C.c_int), ("max_level", C.c_int)]


class LmSummary(C.Structure):
    _fields_ = [("iterations", C.c_int), ("successful", C.c_int), ("unsuccessful", C.c_int),
                ("termination", C.c_int), ("initial_cost", C.c_double),
                ("final_cost", C.c_double)]


LM_TERMINATION = ("no_convergence", "function_tolerance", "parameter_tolerance",
                  "gradient_tolerance", "min_trust_region_radius", "failure")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError(f"oracle not built: {LIB_PATH} (run make -C oracle)")
        L = C.CDLL(LIB_PATH)
        fp, ip, dp = C.POINTER(C.c_float), C.POINTER(C.c_int), C.POINTER(C.c_double)
        TP = C.POINTER(Tile)
        L.pfo_set_window.argtypes = [TP, C.c_float, C.c_float, C.c_float, C.c_float]
        L.pfo_sph_to_2d.argtypes = [TP, C.c_float, C.c_float, fp]
        L.pfo_to_spherical_coord.argtypes = [TP, C.c_float, C.c_float, fp]
        L.pfo_world_to_sph.argtypes = [fp, fp]
        L.pfo_sph_to_world.argtypes = [C.c_float, C.c_float, fp]
        L.pfo_tile_index.argtypes = [TP, C.c_float, C.c_float]
        L.pfo_tile_index.restype = C.c_longlong
        L.pfo_grid_azimuth.argtypes = [C.c_int, C.c_int]
        L.pfo_grid_azimuth.restype = C.c_float
        L.pfo_grid_zenith.argtypes = [C.c_int, C.c_int]
        L.pfo_grid_zenith.restype = C.c_float
        L.pfo_emap_value_at_coord.argtypes = [fp, C.c_int, C.c_int, C.c_int, C.c_float, C.c_float]
        L.pfo_emap_value_at_coord.restype = C.c_float
        L.pfo_reg_grid.argtypes = [TP, C.c_float, C.c_float, ip, ip, fp, fp]
        L.pfo_reg_samples.argtypes = [TP, fp, fp, C.c_int, C.c_int, C.c_int, C.c_float,
                                      C.c_float, dp, dp]
        L.pfo_register_tile.argtypes = [TP, fp, fp, C.c_int, C.c_int, C.c_int, C.c_float,
                                        C.c_float, C.c_int, dp, fp]
        L.pfo_register_tile_solver.argtypes = [TP, fp, fp, C.c_int, C.c_int, C.c_int, C.c_float,
                                               C.c_float, C.c_int, C.c_int, dp, fp]
        L.pfo_lm_moments.argtypes = [dp, dp, C.POINTER(LmSummary)]
        L.pfo_depth_to_depth.argtypes = [TP, fp, fp]
        L.pfo_level_dims.argtypes = [C.c_int, C.c_int, C.c_float, C.c_float, C.c_int,
                                     C.POINTER(Level)]
        L.pfo_seed_level0.argtypes = [fp, C.c_int, C.c_int, C.c_int, C.POINTER(Level), fp]
        L.pfo_upsample.argtypes = [fp, C.POINTER(Level), fp]
        L.pfo_tile_box.argtypes = [TP, C.POINTER(Level), ip, ip, ip, ip, ip]
        L.pfo_targets.argtypes = [TP, C.c_int, fp, C.POINTER(Level), fp,
                                  C.POINTER(C.c_int32), C.POINTER(C.c_longlong),
                                  C.POINTER(C.c_longlong)]
        L.pfo_normalize.argtypes = [fp, C.POINTER(C.c_int32), C.POINTER(Level), fp]
        L.pfo_jacobi.argtypes = [fp, fp, fp, C.POINTER(Level), C.c_int]
        L.pfo_quantize.argtypes = [fp, C.c_int, C.POINTER(C.c_uint16)]
        L.pfo_solve_depth_all.argtypes = [fp, C.c_int, C.c_int, C.c_int, TP, C.c_int, fp,
                                          C.c_int, C.c_int, C.c_float, C.c_float,
                                          C.POINTER(C.c_uint16), C.POINTER(C.c_longlong)]
        L.pfo_merge.argtypes = [fp, C.c_int, C.c_int, C.c_int, TP, C.c_int, fp, C.c_int,
                                C.c_float, C.c_float, C.c_int, C.c_int, C.POINTER(C.c_uint16),
                                fp]
        L.pfo_warp_depth.argtypes = [fp, C.c_int, C.c_int, TP, C.c_int, C.POINTER(Response), fp]
        L.pfo_solve_smoothing.argtypes = [TP, C.c_int, fp, C.c_int, C.c_int, C.c_float,
                                          C.c_float, C.POINTER(C.c_uint16)]
        L.pfo_warp_rgb.argtypes = [C.POINTER(C.c_uint8), C.c_int, C.c_int, TP, C.c_int,
                                   C.POINTER(C.c_uint8)]
        L.pfo_warp_coords.argtypes = [TP, C.c_int, C.c_int, C.POINTER(C.c_uint32), fp]
        L.pfo_rgb_taps.argtypes = [C.c_int, C.c_int, TP, C.c_int, C.POINTER(C.c_uint32)]
        L.pfo_hash32.argtypes = [C.c_uint32, C.c_uint32]
        L.pfo_hash32.restype = C.c_uint32
        L.pfo_set_threads.argtypes = [C.c_int]
        L.pfo_nan_marker.restype = C.c_uint32
        L.pfo_lm_fit.argtypes = [dp, dp, C.c_int, dp, C.POINTER(LmSummary)]
        L.pfo_register_tile_lm.argtypes = [TP, fp, fp, C.c_int, C.c_int, C.c_int, C.c_float,
                                           C.c_float, dp, fp, C.POINTER(LmSummary)]
        L.pfo_merge_lm.argtypes = [fp, C.c_int, C.c_int, C.c_int, TP, C.c_int, fp, C.c_int,
                                   C.c_float, C.c_float, C.POINTER(C.c_uint16), fp]
        L.pfo_error_metrics.argtypes = [fp, C.c_int, C.c_int, C.c_int, fp, C.POINTER(C.c_uint16),
                                        C.c_int, C.c_int, C.c_int, C.c_float, C.c_float,
                                        C.c_int, C.c_int, fp, C.POINTER(C.c_int)]
        _lib = L
    return _lib


def _p(a, t=C.c_float):
    return a.ctypes.data_as(C.POINTER(t))


def make_tiles(layout, channels=1, capped=True):
    """pfo_tile array for a layout (SetWindow + ranges as MergeDepthMaps sets them)."""
    L = lib()
    n = layout.ntiles
    arr = (Tile * n)()
    rng = layout.capped_ranges() if capped else layout.ranges
    off = 0
    for i in range(n):
        t = arr[i]
        t.width, t.height, t.channels = int(layout.tile_w[i]), int(layout.tile_h[i]), channels
        t.offset = off
        off += t.width * t.height * channels
        f = layout.fovs[i]
        L.pfo_set_window(C.byref(t), float(f[0]), float(f[1]), float(f[2]), float(f[3]))
        for k in range(4):
            t.ranges[k] = float(rng[i, k])
    return arr, off


def level_dims(out_w, out_h, zr, level):
    lv = Level()
    if lib().pfo_level_dims(out_w, out_h, zr[0], zr[1], level, C.byref(lv)) != 0:
        raise ValueError("bad level")
    return lv


def num_levels(out_w):
    return 4 if out_w >= 4096 else 3


def targets(tiles, tile_data, lv):
    n = len(tiles)
    Lsum = np.zeros(lv.w * lv.h, np.float32)
    cnt = np.zeros(lv.w * lv.h, np.int32)
    oops, oob = C.c_longlong(0), C.c_longlong(0)
    rc = lib().pfo_targets(tiles, n, _p(tile_data), C.byref(lv), _p(Lsum),
                           _p(cnt, C.c_int32), C.byref(oops), C.byref(oob))
    if rc != 0:
        raise ValueError(f"pfo_targets rc={rc}")
    return Lsum.reshape(lv.h, lv.w), cnt.reshape(lv.h, lv.w), oops.value, oob.value


def normalize(Lsum, cnt, lv):
    out = np.zeros(lv.w * lv.h, np.float32)
    lib().pfo_normalize(_p(np.ascontiguousarray(Lsum).ravel()),
                        _p(np.ascontiguousarray(cnt).ravel(), C.c_int32), C.byref(lv), _p(out))
    return out.reshape(lv.h, lv.w)


def seed_level0(emap, lv):
    eh, ew = emap.shape[:2]
    ec = emap.shape[2] if emap.ndim == 3 else 1
    buf = np.zeros(lv.w * lv.h, np.float32)
    lib().pfo_seed_level0(_p(np.ascontiguousarray(emap, np.float32)), ew, eh, ec, C.byref(lv),
                          _p(buf))
    return buf.reshape(lv.h, lv.w)


def upsample(prev, lv):
    buf = np.zeros(lv.w * lv.h, np.float32)
    lib().pfo_upsample(_p(np.ascontiguousarray(prev, np.float32)), C.byref(lv), _p(buf))
    return buf.reshape(lv.h, lv.w)


def jacobi(buf, Lnorm, lv, iters):
    b = np.ascontiguousarray(buf, np.float32).copy().ravel()
    tmp = np.empty_like(b)
    lib().pfo_jacobi(_p(b), _p(tmp), _p(np.ascontiguousarray(Lnorm, np.float32).ravel()),
                     C.byref(lv), iters)
    return b.reshape(lv.h, lv.w)


def quantize(buf):
    b = np.ascontiguousarray(buf, np.float32).ravel()
    out = np.zeros(b.size, np.uint16)
    lib().pfo_quantize(_p(b), b.size, _p(out, C.c_uint16))
    return out.reshape(buf.shape)


def solve_depth_all(emap, tiles, tile_data, out_w, zr):
    eh, ew = emap.shape[:2]
    ec = emap.shape[2] if emap.ndim == 3 else 1
    out = np.zeros(out_w * (out_w // 2), np.uint16)
    oops = C.c_longlong(0)
    rc = lib().pfo_solve_depth_all(_p(np.ascontiguousarray(emap, np.float32)), ew, eh, ec,
                                   tiles, len(tiles), _p(tile_data), out_w, out_w // 2,
                                   zr[0], zr[1], _p(out, C.c_uint16), C.byref(oops))
    if rc != 0:
        raise ValueError(f"pfo_solve_depth_all rc={rc}")
    return out.reshape(out_w // 2, out_w), oops.value


def solve_smoothing(tiles, tile_data, out_w, out_h, zr):
    """SolveDepthBySmoothing (Depth.cpp:1773-1878) -> u16 [out_h, out_w]."""
    out = np.zeros(out_w * out_h, np.uint16)
    rc = lib().pfo_solve_smoothing(tiles, len(tiles), _p(tile_data), out_w, out_h, zr[0], zr[1],
                                   _p(out, C.c_uint16))
    if rc != 0:
        raise ValueError(f"pfo_solve_smoothing rc={rc}")
    return out.reshape(out_h, out_w)


SOLVERS = {"normal": 0, "lm": 1}  # PFO_SOLVER_*; "lm" (the reference's Ceres LM) is the default


def register_tile(tile, tile_data, emap, zr, degree=3, solver="lm"):
    """SolveDepthToDepth for one tile from the fixed-order moment sums: (c64, abcd, degree)."""
    eh, ew = emap.shape[:2]
    ec = emap.shape[2] if emap.ndim == 3 else 1
    c64 = np.zeros(4, np.float64)
    abcd = np.zeros(4, np.float32)
    d = lib().pfo_register_tile_solver(C.byref(tile), _p(tile_data),
                                       _p(np.ascontiguousarray(emap, np.float32)), ew, eh, ec,
                                       zr[0], zr[1], degree, SOLVERS[solver],
                                       _p(c64, C.c_double), _p(abcd))
    return c64, abcd, d


def lm_moments(S):
    """Moment-form LM (the HIP kernel's form) on 15 sums: (coef[4], summary dict)."""
    S = np.ascontiguousarray(S, np.float64)
    c = np.zeros(4, np.float64)
    s = LmSummary()
    lib().pfo_lm_moments(_p(S, C.c_double), _p(c, C.c_double), C.byref(s))
    return c, _lm_dict(s)


def reg_samples(tile, tile_data, emap, zr):
    eh, ew = emap.shape[:2]
    ec = emap.shape[2] if emap.ndim == 3 else 1
    cols, rows = C.c_int(0), C.c_int(0)
    zt, zd = C.c_float(0), C.c_float(0)
    lib().pfo_reg_grid(C.byref(tile), zr[0], zr[1], C.byref(cols), C.byref(rows),
                       C.byref(zt), C.byref(zd))
    ns = (cols.value + 1) * (rows.value + 1)
    xs = np.zeros(ns, np.float64)
    ys = np.zeros(ns, np.float64)
    lib().pfo_reg_samples(C.byref(tile), _p(tile_data), _p(np.ascontiguousarray(emap, np.float32)),
                          ew, eh, ec, zr[0], zr[1], _p(xs, C.c_double), _p(ys, C.c_double))
    return xs, ys, cols.value, rows.value


def lm_fit(xs, ys):
    """Ceres-LM restatement (pf_oracle_lm.c) on samples: (coef[4] fp64, summary dict)."""
    xs = np.ascontiguousarray(xs, np.float64)
    ys = np.ascontiguousarray(ys, np.float64)
    c = np.zeros(4, np.float64)
    s = LmSummary()
    if lib().pfo_lm_fit(_p(xs, C.c_double), _p(ys, C.c_double), xs.size, _p(c, C.c_double),
                        C.byref(s)) != 0:
        raise ValueError("pfo_lm_fit failed")
    return c, _lm_dict(s)


def _lm_dict(s):
    return {"iterations": s.iterations, "successful": s.successful,
            "unsuccessful": s.unsuccessful, "termination": LM_TERMINATION[s.termination],
            "initial_cost": s.initial_cost, "final_cost": s.final_cost}


def register_tile_lm(tile, tile_data, emap, zr):
    """SolveDepthToDepth for one tile with the Ceres-LM restatement: (c64, abcd f32, summary)."""
    eh, ew = emap.shape[:2]
    ec = emap.shape[2] if emap.ndim == 3 else 1
    c64 = np.zeros(4, np.float64)
    abcd = np.zeros(4, np.float32)
    s = LmSummary()
    if lib().pfo_register_tile_lm(C.byref(tile), _p(tile_data),
                                  _p(np.ascontiguousarray(emap, np.float32)), ew, eh, ec, zr[0],
                                  zr[1], _p(c64, C.c_double), _p(abcd), C.byref(s)) != 0:
        raise ValueError("pfo_register_tile_lm failed")
    return c64, abcd, _lm_dict(s)


def merge_lm(emap, tiles, tile_data, out_w, zr):
    """MergeDepthMaps core with the Ceres-LM registration; tile_data is transformed in place."""
    eh, ew = emap.shape[:2]
    ec = emap.shape[2] if emap.ndim == 3 else 1
    out = np.zeros(out_w * (out_w // 2), np.uint16)
    abcd = np.zeros(4 * len(tiles), np.float32)
    rc = lib().pfo_merge_lm(_p(np.ascontiguousarray(emap, np.float32)), ew, eh, ec, tiles,
                            len(tiles), _p(tile_data), out_w, zr[0], zr[1],
                            _p(out, C.c_uint16), _p(abcd))
    if rc != 0:
        raise ValueError(f"pfo_merge_lm rc={rc}")
    return out.reshape(out_w // 2, out_w), abcd.reshape(-1, 4)


def depth_to_depth(tile, tile_data, abcd):
    lib().pfo_depth_to_depth(C.byref(tile), _p(tile_data), _p(np.asarray(abcd, np.float32)))


def merge(emap, tiles, tile_data, out_w, zr, degree=3, solver="lm"):
    """MergeDepthMaps core; tile_data is transformed in place."""
    eh, ew = emap.shape[:2]
    ec = emap.shape[2] if emap.ndim == 3 else 1
    out = np.zeros(out_w * (out_w // 2), np.uint16)
    abcd = np.zeros(4 * len(tiles), np.float32)
    rc = lib().pfo_merge(_p(np.ascontiguousarray(emap, np.float32)), ew, eh, ec, tiles,
                         len(tiles), _p(tile_data), out_w, zr[0], zr[1], degree,
                         SOLVERS[solver], _p(out, C.c_uint16), _p(abcd))
    if rc != 0:
        raise ValueError(f"pfo_merge rc={rc}")
    return out.reshape(out_w // 2, out_w), abcd.reshape(-1, 4)


def responses(params):
    """params: (n,5) array-like of (alpha, kappa, beta, sigma, seed)."""
    n = len(params)
    arr = (Response * n)()
    for i, p in enumerate(params):
        arr[i].alpha, arr[i].kappa, arr[i].beta, arr[i].sigma = (float(p[0]), float(p[1]),
                                                                  float(p[2]), float(p[3]))
        arr[i].seed = int(p[4]) & 0xFFFFFFFF
    return arr


def warp_depth(pano, tiles, total, resp=None):
    ph, pw = pano.shape
    out = np.zeros(total, np.float32)
    lib().pfo_warp_depth(_p(np.ascontiguousarray(pano, np.float32)), pw, ph, tiles, len(tiles),
                         resp, _p(out))
    return out


def warp_coords(tile, pw, ph):
    """The depth warp's map of one tile: (wxy uint32 [h*w] = x0 | y0 << 16, wfxy float32
    [h*w, 2] = (fx, fy))."""
    n = tile.width * tile.height
    wxy = np.zeros(n, np.uint32)
    wf = np.zeros((n, 2), np.float32)
    lib().pfo_warp_coords(C.byref(tile), pw, ph, _p(wxy, C.c_uint32), _p(wf))
    return wxy, wf


def rgb_taps(tiles, pw, ph):
    """The RGB warp's tap map of the layout: uint32 [sum h*w, 4]."""
    total = sum(t.width * t.height for t in tiles)
    taps = np.zeros((total, 4), np.uint32)
    lib().pfo_rgb_taps(pw, ph, tiles, len(tiles), _p(taps, C.c_uint32))
    return taps


def warp_rgb(pano_u8, tiles):
    ph, pw, _ = pano_u8.shape
    total = sum(t.width * t.height * 3 for t in tiles)
    out = np.zeros(total, np.uint8)
    lib().pfo_warp_rgb(_p(np.ascontiguousarray(pano_u8, np.uint8), C.c_uint8), pw, ph, tiles,
                       len(tiles), _p(out, C.c_uint8))
    return out


def set_threads(n):
    lib().pfo_set_threads(int(n))


def probe_taps(tiles, lv):
    out = np.zeros(lv.w * lv.h * 5, np.int32)
    L = lib()
    L.pfo_probe_taps.argtypes = [C.POINTER(Tile), C.c_int, C.POINTER(Level), C.POINTER(C.c_int32)]
    if L.pfo_probe_taps(tiles, len(tiles), C.byref(lv), _p(out, C.c_int32)) != 0:
        raise ValueError("degenerate box")
    return out.reshape(lv.h, lv.w, 5)


def targets_subset(tiles, t0, t1, tile_data, lv):
    """pfo_targets over tiles [t0, t1) only (the per-rank share of a sharded panorama)."""
    Lsum = np.zeros(lv.w * lv.h, np.float32)
    cnt = np.zeros(lv.w * lv.h, np.int32)
    oops, oob = C.c_longlong(0), C.c_longlong(0)
    sub = C.cast(C.byref(tiles, t0 * C.sizeof(Tile)), C.POINTER(Tile))
    rc = lib().pfo_targets(sub, t1 - t0, _p(tile_data), C.byref(lv), _p(Lsum),
                           _p(cnt, C.c_int32), C.byref(oops), C.byref(oob))
    if rc != 0:
        raise ValueError(f"pfo_targets rc={rc}")
    return Lsum.reshape(lv.h, lv.w), cnt.reshape(lv.h, lv.w)


METRIC_KEYS = ("mse", "mae", "mre", "mselog", "delta1", "delta2", "delta3", "median_shift",
               "ls_s", "ls_o", "gt_median", "given_median")


def error_metrics(gt, given, zr, align_way=1, cap_depth=True):
    """ErrorData (given: uint16 [h][w]) / ErrorEmap (given: float [h][w] or [h][w][c]);
    gt: float [gh][gw] or [gh][gw][gc].  Returns a dict of METRIC_KEYS + n, nlog."""
    gt = np.ascontiguousarray(gt, np.float32)
    gh, gw = gt.shape[:2]
    gc = gt.shape[2] if gt.ndim == 3 else 1
    h, w = given.shape[:2]
    out = np.zeros(12, np.float32)
    cnt = np.zeros(2, np.int32)
    if given.dtype == np.uint16:
        g16 = np.ascontiguousarray(given)
        lib().pfo_error_metrics(_p(gt), gw, gh, gc, None, _p(g16, C.c_uint16), w, h, 1,
                                zr[0], zr[1], align_way, int(cap_depth), _p(out),
                                _p(cnt, C.c_int))
    else:
        gf = np.ascontiguousarray(given, np.float32)
        c = gf.shape[2] if gf.ndim == 3 else 1
        lib().pfo_error_metrics(_p(gt), gw, gh, gc, _p(gf), None, w, h, c, zr[0], zr[1],
                                align_way, int(cap_depth), _p(out), _p(cnt, C.c_int))
    d = {k: float(out[i]) for i, k in enumerate(METRIC_KEYS)}
    d["n"], d["nlog"] = int(cnt[0]), int(cnt[1])
    return d
