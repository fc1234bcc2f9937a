"""Python host binding of libpanofuse (include/panofuse.h) over ctypes.

This is the host-side mirror of the reference's DepthNamespace entry points for the fused path
(``Depth.h:286-307``): ``Fuser.register`` ~ SolveDepthToDepth + Depth2DepthTransform,
``Fuser.fuse`` ~ SolveDepthAll, ``Fuser.merge`` ~ MergeDepthMaps' compute core.  Tensors are
torch device tensors (PyTorch is used only for device memory and streams); the compute is the
hand-written HIP in csrc/.  There is no CPU fallback: if lib/libpanofuse.so is missing or no GPU
is present, every call raises.
"""
import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# PANOFUSE_LIB selects another build of the same library (A/B tuning runs, tools/gpu_round.sh (ab step))
LIB_PATH = os.environ.get("PANOFUSE_LIB") or os.path.join(HERE, "lib", "libpanofuse.so")

PF_OK, PF_EINVAL, PF_ENOMEM, PF_EHIP, PF_ESTATE, PF_EDEGENERATE = 0, -1, -2, -3, -4, -5
PF_ETIMEOUT = -6  # a resident-kernel hand-off wait timed out: that fusion's output is invalid

# Every symbol declared in include/panofuse.h.
EXPORTS = [
    "pf_create", "pf_destroy", "pf_last_error", "pf_set_stream", "pf_synchronize",
    "pf_version", "pf_set_tiles", "pf_register", "pf_fuse", "pf_merge", "pf_warp_depth",
    "pf_warp_rgb", "pf_level_info", "pf_fuse_partial", "pf_fuse_seed", "pf_fuse_finish_level",
    "pf_probe_taps", "pf_profile_enable", "pf_profile_read", "pf_error_metrics",
    "pf_depth_transform", "pf_register_joint", "pf_set_solver", "pf_fuse_normalize",
    "pf_fuse_border", "pf_fuse_band_plan", "pf_fuse_band_pass", "pf_fuse_multicover",
    "pf_fuse_multicover_patch", "pf_solve_smoothing", "pf_set_metrics_order",
    "pf_jres_errors", "pf_set_jacobi_engine", "pf_stream_wait_level", "pf_debug_jres_fault",
    "pf_probe_warp_coords", "pf_probe_rgb_taps", "pf_debug_smooth_fault",
    "pf_fuse_partial_rows", "pf_fuse_coverage_rows", "pf_fuse_normalize_rows",
    "pf_fuse_tile_rows", "pf_rows_add", "pf_fuse_level", "pf_fuse_targets",
    "pf_rows_add_batch", "pf_set_jacobi_share",
]
NEW_R4 = {"pf_debug_jres_fault", "pf_probe_warp_coords", "pf_probe_rgb_taps",
          "pf_debug_smooth_fault", "pf_fuse_partial_rows", "pf_fuse_coverage_rows",
          "pf_fuse_normalize_rows", "pf_fuse_tile_rows", "pf_rows_add", "pf_fuse_level",
          "pf_fuse_targets", "pf_rows_add_batch", "pf_set_jacobi_share"}
METRICS_ORDERS = {"tree": 0, "sequential": 1}  # PF_METRICS_*; "sequential" = the reference's
SOLVERS = {"normal": 0, "lm": 1}  # PF_SOLVER_*; "lm" = the reference's Ceres LM (default)

STAGES = ["warp", "register", "seed", "targets", "jacobi", "quantize", "metrics"]


class PanofuseError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"panofuse error {code}: {msg}")
        self.code = code


class Window(C.Structure):
    _fields_ = [("az_left", C.c_float), ("az_right", C.c_float),
                ("zen_top", C.c_float), ("zen_down", C.c_float)]


class Response(C.Structure):
    _fields_ = [("alpha", C.c_float), ("kappa", C.c_float), ("beta", C.c_float),
                ("sigma", C.c_float), ("seed", C.c_uint32), ("pad", C.c_uint32)]


_lib = None


def load():
    """Load libpanofuse.so; raises if it was not built (no fallback path exists)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise RuntimeError(f"libpanofuse.so not built at {LIB_PATH}: run "
                           f"`python -c 'import __graft_entry__ as g; g.build()'`")
    L = C.CDLL(LIB_PATH)
    vp, fp, ip = C.c_void_p, C.c_float, C.c_int
    L.pf_create.argtypes = [ip, C.POINTER(vp)]
    L.pf_destroy.argtypes = [vp]
    L.pf_destroy.restype = None
    L.pf_last_error.argtypes = [vp]
    L.pf_last_error.restype = C.c_char_p
    L.pf_set_stream.argtypes = [vp, vp]
    L.pf_synchronize.argtypes = [vp]
    L.pf_version.restype = C.c_char_p
    L.pf_set_tiles.argtypes = [vp, C.POINTER(Window), C.POINTER(Window), ip,
                               C.POINTER(C.c_int), C.POINTER(C.c_int), ip, ip]
    L.pf_register.argtypes = [vp, vp, ip, ip, ip, vp, ip, fp, fp, ip, ip, vp, vp]
    L.pf_fuse.argtypes = [vp, vp, ip, ip, ip, vp, vp, ip, ip, ip, fp, fp, vp]
    L.pf_merge.argtypes = [vp, vp, ip, ip, ip, vp, ip, ip, fp, fp, vp, vp]
    L.pf_warp_depth.argtypes = [vp, vp, ip, ip, ip, vp, vp]
    L.pf_warp_rgb.argtypes = [vp, vp, ip, ip, ip, vp]
    L.pf_solve_smoothing.argtypes = [vp, vp, vp, ip, ip, ip, fp, fp, vp]
    L.pf_set_metrics_order.argtypes = [vp, ip]
    L.pf_level_info.argtypes = [ip, ip, fp, fp, ip] + [C.POINTER(C.c_int)] * 6
    L.pf_fuse_partial.argtypes = [vp, vp, vp, ip, ip, ip, ip, fp, fp, ip, vp, vp]
    L.pf_fuse_seed.argtypes = [vp, vp, ip, ip, ip, vp, ip, ip, fp, fp, ip, vp]
    L.pf_fuse_finish_level.argtypes = [vp, vp, vp, ip, ip, fp, fp, ip, vp, vp]
    L.pf_probe_taps.argtypes = [vp, ip, ip, fp, fp, ip, vp]
    L.pf_depth_transform.argtypes = [vp, vp, C.c_longlong, ip, vp]
    L.pf_register_joint.argtypes = [vp, vp, ip, ip, ip, vp, ip, fp, fp, ip, vp, vp, vp]
    L.pf_error_metrics.argtypes = [vp, vp, ip, ip, ip, vp, vp, ip, ip, ip, ip, fp, fp, ip, ip,
                                   vp]
    L.pf_set_solver.argtypes = [vp, ip]
    L.pf_fuse_normalize.argtypes = [vp, vp, vp, ip, ip, fp, fp, ip, vp]
    L.pf_fuse_multicover.argtypes = [vp, vp, vp, ip, ip, ip, ip, fp, fp, ip, vp,
                                     C.POINTER(C.c_int)]
    L.pf_fuse_multicover_patch.argtypes = [vp, ip, ip, fp, fp, ip, vp, vp]
    L.pf_fuse_border.argtypes = [vp, vp, ip, ip, fp, fp, ip, vp, vp, vp]
    L.pf_fuse_band_plan.argtypes = [vp, ip, ip, fp, fp, ip, ip, C.POINTER(C.c_int), ip]
    L.pf_fuse_band_pass.argtypes = [vp, vp, ip, ip, ip, vp, vp, ip, vp, vp, vp, ip, ip, fp, fp,
                                    ip, ip, ip, ip]
    L.pf_profile_enable.argtypes = [vp, ip]
    L.pf_jres_errors.argtypes = [vp]
    # (entry points added after round 3: an A/B variant built from older sources may lack them)
    for name, at in (("pf_debug_jres_fault", [vp, ip]), ("pf_debug_smooth_fault", [vp, ip]),
                     ("pf_fuse_partial_rows", [vp, vp, vp, ip, ip, ip, ip, fp, fp, ip, ip, ip,
                                               vp, vp]),
                     ("pf_fuse_coverage_rows", [vp, ip, ip, fp, fp, ip, ip, ip, vp]),
                     ("pf_fuse_normalize_rows", [vp, vp, vp, ip, ip, fp, fp, ip, ip, ip, vp]),
                     ("pf_fuse_tile_rows", [vp, ip, ip, fp, fp, ip, ip, ip,
                                            C.POINTER(C.c_int), C.POINTER(C.c_int)]),
                     ("pf_rows_add", [vp, vp, vp, C.c_longlong]),
                     ("pf_rows_add_batch", [vp, vp, vp, vp, ip]),
                     ("pf_fuse_level", [vp, vp, ip, ip, ip, vp, vp, vp, ip, ip, fp, fp, ip, vp,
                                        vp]),
                     ("pf_fuse_targets", [vp, vp, vp, ip, ip, fp, fp, ip, vp]),
                     ("pf_probe_warp_coords", [C.POINTER(Window), ip, ip, ip, ip, vp, vp]),
                     ("pf_probe_rgb_taps", [C.POINTER(Window), ip, ip, ip, ip, vp])):
        if hasattr(L, name):
            getattr(L, name).argtypes = at
    L.pf_set_jacobi_engine.argtypes = [vp, ip, ip]
    L.pf_set_jacobi_share.argtypes = [vp, C.c_double]
    L.pf_stream_wait_level.argtypes = [vp, ip, vp]
    L.pf_profile_read.argtypes = [vp, C.POINTER(C.c_double), C.POINTER(C.c_double),
                                  C.POINTER(C.c_longlong)]
    variant = os.environ.get("PANOFUSE_LIB") is not None
    for name in EXPORTS:
        if not hasattr(L, name) and not (variant and name in NEW_R4):
            raise RuntimeError(f"libpanofuse.so lacks {name}")
    _lib = L
    return L


def level_info(out_w, out_h, zr, level):
    """(w, h, h0, h1, iters, nlevels) of a fusion level (Depth.cpp:1420-1437, 1650-1675)."""
    vals = [C.c_int(0) for _ in range(6)]
    rc = load().pf_level_info(out_w, out_h, float(zr[0]), float(zr[1]), level,
                              *[C.byref(v) for v in vals])
    if rc != PF_OK:
        raise PanofuseError(rc, "pf_level_info")
    return tuple(v.value for v in vals)


def _ptr(t):
    if t is None:
        return None
    if not t.is_cuda:
        raise ValueError("panofuse takes device tensors only")
    if not t.is_contiguous():
        raise ValueError("panofuse takes contiguous tensors")
    return C.c_void_p(t.data_ptr())


def _emap_dims(emap):
    # emap: [B, eh, ew] or [B, eh, ew, ec]
    if emap.dim() == 3:
        return emap.shape[2], emap.shape[1], 1
    return emap.shape[2], emap.shape[1], emap.shape[3]


# pf_metrics field order (include/panofuse.h)
METRIC_KEYS = ("mse", "mae", "mre", "mselog", "delta1", "delta2", "delta3", "median_shift",
               "ls_s", "ls_o", "gt_median", "given_median")


class Fuser:
    """One context = one device + one stream (pf_ctx)."""

    def __init__(self, device=0, stream=None):
        import torch
        if not torch.cuda.is_available():
            raise RuntimeError("panofuse needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.L = load()
        self.device = device
        h = C.c_void_p()
        rc = self.L.pf_create(device, C.byref(h))
        if rc != PF_OK:
            raise PanofuseError(rc, "pf_create failed")
        self.h = h
        self.layout = None
        self.set_stream(stream)

    def set_stream(self, stream=None):
        import torch
        if stream is None:
            stream = torch.cuda.current_stream(self.device)
        self.stream = stream
        self._check(self.L.pf_set_stream(self.h, C.c_void_p(stream.cuda_stream)))

    def close(self):
        if getattr(self, "h", None):
            self.L.pf_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != PF_OK:
            raise PanofuseError(rc, self.L.pf_last_error(self.h).decode())

    def set_tiles(self, layout, channels=1, cap_ranges=True):
        n = layout.ntiles
        fov = (Window * n)(*[Window(*map(float, layout.fovs[i])) for i in range(n)])
        rng = (Window * n)(*[Window(*map(float, layout.ranges[i])) for i in range(n)])
        tw = (C.c_int * n)(*[int(v) for v in layout.tile_w])
        th = (C.c_int * n)(*[int(v) for v in layout.tile_h])
        self._check(self.L.pf_set_tiles(self.h, fov, rng, n, tw, th, channels,
                                        1 if cap_ranges else 0))
        self.layout = layout
        self.channels = channels
        self.tile_elems = int(sum(int(layout.tile_w[i]) * int(layout.tile_h[i])
                                  for i in range(n))) * channels

    def set_solver(self, solver):
        """Degree-3 registration solver: "lm" (the reference's Ceres LM, default) or "normal"."""
        self._check(self.L.pf_set_solver(self.h, SOLVERS[solver]))

    def register(self, emap, tiles, zr, degree=3, apply=True, coeffs=None, coeffs64=None):
        ew, eh, ec = _emap_dims(emap)
        B = emap.shape[0]
        self._check(self.L.pf_register(self.h, _ptr(emap), ew, eh, ec, _ptr(tiles), B,
                                       float(zr[0]), float(zr[1]), degree, 1 if apply else 0,
                                       _ptr(coeffs), _ptr(coeffs64)))

    def fuse(self, emap, tiles, out, zr, coeffs=None):
        ew, eh, ec = _emap_dims(emap)
        B, oh, ow = out.shape
        self._check(self.L.pf_fuse(self.h, _ptr(emap), ew, eh, ec, _ptr(tiles), _ptr(coeffs),
                                   B, ow, oh, float(zr[0]), float(zr[1]), _ptr(out)))

    def merge(self, emap, tiles, out, zr, coeffs=None):
        ew, eh, ec = _emap_dims(emap)
        B, oh, ow = out.shape
        if oh != ow // 2:
            raise ValueError("MergeDepthMaps output height is out_w/2")
        self._check(self.L.pf_merge(self.h, _ptr(emap), ew, eh, ec, _ptr(tiles), B, ow,
                                    float(zr[0]), float(zr[1]), _ptr(coeffs), _ptr(out)))

    def set_metrics_order(self, order):
        """"tree" (the context's default): fp64 partial sums (fast, means within 1e-5 of exact
        sums); "sequential": the reference's float summation order, bit-exact means (~7.4 ms per
        64-panorama call at C3; the facade and panofuse_main default to it)."""
        self._check(self.L.pf_set_metrics_order(self.h, METRICS_ORDERS[order]))

    def solve_smoothing(self, tiles, out, zr, coeffs=None):
        """SolveDepthBySmoothing (Depth.cpp:1773-1878) into out [B, out_h, out_w] (int16 view
        of u16); coeffs: None or [B, ntiles, 4], applied as Depth2DepthTransform on the fly."""
        B, oh, ow = out.shape
        self._check(self.L.pf_solve_smoothing(self.h, _ptr(tiles), _ptr(coeffs), B, ow, oh,
                                              float(zr[0]), float(zr[1]), _ptr(out)))

    def warp_depth(self, pano, tiles, resp=None):
        B, ph, pw = pano.shape
        self._check(self.L.pf_warp_depth(self.h, _ptr(pano), pw, ph, B, _ptr(resp),
                                         _ptr(tiles)))

    def warp_rgb(self, pano, tiles):
        B, ph, pw, _ = pano.shape
        self._check(self.L.pf_warp_rgb(self.h, _ptr(pano), pw, ph, B, _ptr(tiles)))

    def register_joint(self, emap, tiles, zr, active, degree=3, coeffs=None, coeffs64=None):
        """SolveDepthToDepth with the tiles of `active` (list of tile indices) in one problem;
        coeffs / coeffs64: [B, 4] device tensors."""
        ew, eh, ec = _emap_dims(emap)
        B = emap.shape[0]
        mask = (C.c_int * self.layout.ntiles)(*[1 if i in set(active) else 0
                                                 for i in range(self.layout.ntiles)])
        self._check(self.L.pf_register_joint(self.h, _ptr(emap), ew, eh, ec, _ptr(tiles), B,
                                             float(zr[0]), float(zr[1]), int(degree), mask,
                                             _ptr(coeffs), _ptr(coeffs64)))

    def error_metrics_async(self, gt, given, zr, out, align_way=1, cap_depth=True):
        """pf_error_metrics into out (int32 [B,16] device tensor = B pf_metrics), no sync."""
        import torch
        gw, gh, gc = _emap_dims(gt)
        B, h, w = given.shape[:3]
        if given.dtype in (torch.int16, torch.uint16):
            self._check(self.L.pf_error_metrics(self.h, _ptr(gt), gw, gh, gc, None, _ptr(given),
                                                w, h, 1, B, float(zr[0]), float(zr[1]),
                                                int(align_way), int(cap_depth), _ptr(out)))
        else:
            gvc = given.shape[3] if given.dim() == 4 else 1
            self._check(self.L.pf_error_metrics(self.h, _ptr(gt), gw, gh, gc, _ptr(given), None,
                                                w, h, gvc, B, float(zr[0]), float(zr[1]),
                                                int(align_way), int(cap_depth), _ptr(out)))

    def error_metrics(self, gt, given, zr, align_way=1, cap_depth=True):
        """ErrorData (given: int16/uint16 [B,h,w] result bits) or ErrorEmap (given: float32
        [B,h,w] or [B,h,w,c]) against gt float32 [B,gh,gw] or [B,gh,gw,gc]
        (Depth.cpp:1980-2458).  Returns a list (one per panorama) of dicts of METRIC_KEYS +
        n, nlog."""
        import torch
        B = given.shape[0]
        out = torch.zeros((B, 16), dtype=torch.int32, device=gt.device)
        self.error_metrics_async(gt, given, zr, out, align_way, cap_depth)
        self.synchronize()
        o = out.cpu()
        f = o[:, :12].view(torch.float32)
        res = []
        for b in range(B):
            d = {k: float(f[b, i]) for i, k in enumerate(METRIC_KEYS)}
            d["n"], d["nlog"] = int(o[b, 12]), int(o[b, 13])
            res.append(d)
        return res

    def probe_taps(self, out_w, zr, level):
        import torch
        w, h = level_info(out_w, out_w // 2, zr, level)[:2]
        out = torch.empty((h, w, 5), dtype=torch.int32, device=f"cuda:{self.device}")
        self._check(self.L.pf_probe_taps(self.h, out_w, out_w // 2, float(zr[0]), float(zr[1]),
                                         level, _ptr(out)))
        return out

    def fuse_partial(self, tiles, coeffs, t0, t1, out_w, zr, level, lsum, cnt):
        self._check(self.L.pf_fuse_partial(self.h, _ptr(tiles), _ptr(coeffs), t0, t1, out_w,
                                           out_w // 2, float(zr[0]), float(zr[1]), level,
                                           _ptr(lsum), _ptr(cnt)))

    def fuse_partial_rows(self, tiles, coeffs, t0, t1, out_w, zr, level, row0, row1, lsum, cnt):
        """pf_fuse_partial on rows [row0, row1) only (no zeroing elsewhere)."""
        self._check(self.L.pf_fuse_partial_rows(self.h, _ptr(tiles), _ptr(coeffs), t0, t1, out_w,
                                                out_w // 2, float(zr[0]), float(zr[1]), level,
                                                int(row0), int(row1), _ptr(lsum), _ptr(cnt)))

    def fuse_coverage_rows(self, out_w, zr, level, row0, row1, cnt):
        """Coverage count of every tile on rows [row0, row1) (layout-only)."""
        self._check(self.L.pf_fuse_coverage_rows(self.h, out_w, out_w // 2, float(zr[0]),
                                                 float(zr[1]), level, int(row0), int(row1),
                                                 _ptr(cnt)))

    def fuse_normalize_rows(self, lsum, cnt, out_w, zr, level, row0, row1, lnorm):
        self._check(self.L.pf_fuse_normalize_rows(self.h, _ptr(lsum), _ptr(cnt), out_w,
                                                  out_w // 2, float(zr[0]), float(zr[1]), level,
                                                  int(row0), int(row1), _ptr(lnorm)))

    def fuse_tile_rows(self, out_w, zr, level, t0, t1):
        """(ymin, ymax): rows where tiles [t0, t1) have non-zero partial sums (ymin > ymax: none)."""
        lo, hi = C.c_int(), C.c_int()
        self._check(self.L.pf_fuse_tile_rows(self.h, out_w, out_w // 2, float(zr[0]),
                                             float(zr[1]), level, int(t0), int(t1), C.byref(lo),
                                             C.byref(hi)))
        return lo.value, hi.value

    def rows_add(self, dst, src):
        """dst += src (same-size fp32 device tensors), on the context's stream."""
        assert dst.numel() == src.numel()
        self._check(self.L.pf_rows_add(self.h, _ptr(dst), _ptr(src), dst.numel()))

    def rows_add_batch(self, pairs):
        """dst += src for every (dst, src) pair of same-size fp32 device tensors, one launch
        (pf_rows_add_batch); the destinations must not overlap."""
        k = len(pairs)
        if not k:
            return
        dst = (C.c_void_p * k)(*[_ptr(d).value for d, _ in pairs])
        src = (C.c_void_p * k)(*[_ptr(s).value for _, s in pairs])
        n = (C.c_longlong * k)()
        for i, (d, s) in enumerate(pairs):
            assert d.numel() == s.numel()
            n[i] = d.numel()
        self._check(self.L.pf_rows_add_batch(self.h, dst, src, n, k))

    def fuse_seed(self, emap, prev, out_w, zr, level, buf):
        ew, eh, ec = _emap_dims(emap) if emap is not None else (0, 0, 0)
        self._check(self.L.pf_fuse_seed(self.h, _ptr(emap), ew, eh, ec, _ptr(prev), out_w,
                                        out_w // 2, float(zr[0]), float(zr[1]), level,
                                        _ptr(buf)))

    def fuse_finish_level(self, lsum, cnt, out_w, zr, level, buf, out=None):
        self._check(self.L.pf_fuse_finish_level(self.h, _ptr(lsum), _ptr(cnt), out_w,
                                                out_w // 2, float(zr[0]), float(zr[1]), level,
                                                _ptr(buf), _ptr(out)))

    def fuse_level(self, emap, prev, lsum, cnt, out_w, zr, level, buf, out=None):
        """pf_fuse_level: fuse_seed + fuse_finish_level with the seed inside the first pass."""
        ew, eh, ec = _emap_dims(emap) if emap is not None else (0, 0, 0)
        self._check(self.L.pf_fuse_level(self.h, _ptr(emap), ew, eh, ec, _ptr(prev), _ptr(lsum),
                                         _ptr(cnt), out_w, out_w // 2, float(zr[0]),
                                         float(zr[1]), level, _ptr(buf), _ptr(out)))

    def fuse_targets(self, tiles, coeffs, out_w, zr, level, lnorm):
        """pf_fuse_targets: one level's normalised targets of one panorama from every tile."""
        self._check(self.L.pf_fuse_targets(self.h, _ptr(tiles), _ptr(coeffs), out_w, out_w // 2,
                                           float(zr[0]), float(zr[1]), level, _ptr(lnorm)))

    def multicover_count(self, out_w, zr, level):
        n = C.c_int(0)
        self._check(self.L.pf_fuse_multicover(self.h, None, None, 0, 0, out_w, out_w // 2,
                                              float(zr[0]), float(zr[1]), level, None,
                                              C.byref(n)))
        return n.value

    def multicover(self, tiles, coeffs, t0, t1, out_w, zr, level, contrib):
        n = C.c_int(0)
        self._check(self.L.pf_fuse_multicover(self.h, _ptr(tiles), _ptr(coeffs), t0, t1, out_w,
                                              out_w // 2, float(zr[0]), float(zr[1]), level,
                                              _ptr(contrib), C.byref(n)))

    def multicover_patch(self, out_w, zr, level, contrib, lsum):
        self._check(self.L.pf_fuse_multicover_patch(self.h, out_w, out_w // 2, float(zr[0]),
                                                    float(zr[1]), level, _ptr(contrib),
                                                    _ptr(lsum)))

    # ---- row-band sharding of a level's sweeps (pf_dist.fuse_row_sharded) ----
    def fuse_normalize(self, lsum, cnt, out_w, zr, level, lnorm):
        self._check(self.L.pf_fuse_normalize(self.h, _ptr(lsum), _ptr(cnt), out_w, out_w // 2,
                                             float(zr[0]), float(zr[1]), level, _ptr(lnorm)))

    def fuse_border(self, prev, out_w, zr, level, a=None, b=None, out=None):
        self._check(self.L.pf_fuse_border(self.h, _ptr(prev), out_w, out_w // 2, float(zr[0]),
                                          float(zr[1]), level, _ptr(a), _ptr(b), _ptr(out)))

    def fuse_band_plan(self, out_w, zr, level, nbands):
        """Sweep depths of the level's passes (identical on every rank for the same nbands)."""
        T = (C.c_int * 256)()
        n = self.L.pf_fuse_band_plan(self.h, out_w, out_w // 2, float(zr[0]), float(zr[1]),
                                     level, nbands, T, 256)
        if n < 0:
            self._check(n)
        return [T[i] for i in range(n)]

    def fuse_band_pass(self, lnorm, src_mode, out_w, zr, level, T, row0, row1, src=None,
                       dst=None, prev=None, emap=None, out=None):
        ew, eh, ec = _emap_dims(emap) if emap is not None else (0, 0, 0)
        self._check(self.L.pf_fuse_band_pass(self.h, _ptr(emap), ew, eh, ec, _ptr(prev),
                                             _ptr(lnorm), int(src_mode), _ptr(src), _ptr(dst),
                                             _ptr(out), out_w, out_w // 2, float(zr[0]),
                                             float(zr[1]), level, int(T), int(row0), int(row1)))

    def profile(self, on=True):
        """Enable/disable per-stage hipEvent timing (resets the accumulators)."""
        self._check(self.L.pf_profile_enable(self.h, 1 if on else 0))

    def profile_read(self):
        """{stage: (ms, algorithmic_bytes, launches)} accumulated since the last read."""
        n = len(STAGES)
        ms, by, ln = (C.c_double * n)(), (C.c_double * n)(), (C.c_longlong * n)()
        self._check(self.L.pf_profile_read(self.h, ms, by, ln))
        return {STAGES[i]: (ms[i], by[i], ln[i]) for i in range(n)}

    def synchronize(self):
        """Wait for the context stream; raises PanofuseError(PF_ETIMEOUT) if a fusion enqueued
        since the last report had a resident-kernel wait time out (its output is invalid)."""
        self._check(self.L.pf_synchronize(self.h))

    def stream_wait_level(self, level, stream):
        """Make torch `stream` wait for level `level` of this context's last enqueued fusion."""
        self._check(self.L.pf_stream_wait_level(self.h, int(level), C.c_void_p(stream.cuda_stream)))

    def set_jacobi_engine(self, resident=True, row_blocks=0):
        """Jacobi engine of the fusion levels: the resident one-launch kernel where it applies
        (default) or the streaming passes; row_blocks forces its blocks per panorama."""
        self._check(self.L.pf_set_jacobi_engine(self.h, 1 if resident else 0, int(row_blocks)))

    def set_jacobi_share(self, share):
        """Fraction of the GPU this context's Jacobi pass plans count on (0 < share <= 1): for
        fusions that run concurrently with others on the same device (pf_set_jacobi_share)."""
        self._check(self.L.pf_set_jacobi_share(self.h, float(share)))

    def jres_errors(self):
        """Timed-out hand-off waits of the resident level kernel so far (0 = every resident
        level result is valid); synchronises."""
        n = self.L.pf_jres_errors(self.h)
        if n < 0:
            self._check(n)
        return n

    def debug_jres_fault(self, spin_log2=10):
        """Test hook: the next resident launch withholds row block 0's hand-off flag with waits
        bounded at 2^spin_log2 polls, so that fusion must report PF_ETIMEOUT."""
        self._check(self.L.pf_debug_jres_fault(self.h, int(spin_log2)))

    def debug_smooth_fault(self, spin_log2=10):
        """Test hook: in the next row-band smoothing, row block 0 never publishes its steps and
        the waits give up after 2^spin_log2 polls, so that call must report PF_ETIMEOUT."""
        self._check(self.L.pf_debug_smooth_fault(self.h, int(spin_log2)))


def warp_coords(fov, tile_w, tile_h, pw, ph):
    """The depth warp's cached map of one tile (host code, no GPU): (wxy uint32 [h*w] =
    x0 | y0 << 16, wfxy float32 [h*w, 2] = (fx, fy))."""
    n = int(tile_w) * int(tile_h)
    wxy = np.zeros(n, np.uint32)
    wf = np.zeros((n, 2), np.float32)
    rc = load().pf_probe_warp_coords(C.byref(Window(*map(float, fov))), int(tile_w), int(tile_h),
                                     int(pw), int(ph), wxy.ctypes.data, wf.ctypes.data)
    if rc != PF_OK:
        raise PanofuseError(rc, "pf_probe_warp_coords")
    return wxy, wf


def rgb_taps(fov, tile_w, tile_h, pw, ph):
    """The RGB warp's cached tap map of one tile (host code, no GPU): uint32 [h*w, 4]."""
    taps = np.zeros((int(tile_w) * int(tile_h), 4), np.uint32)
    rc = load().pf_probe_rgb_taps(C.byref(Window(*map(float, fov))), int(tile_w), int(tile_h),
                                  int(pw), int(ph), taps.ctypes.data)
    if rc != PF_OK:
        raise PanofuseError(rc, "pf_probe_rgb_taps")
    return taps


def make_responses(params, device):
    """[B, ntiles] pf_response array on the device from (alpha, kappa, beta, sigma, seed)."""
    import torch
    p = np.asarray(params, dtype=np.float64).reshape(-1, 5)
    raw = np.zeros((p.shape[0], 6), np.uint32)
    raw[:, 0:4] = p[:, 0:4].astype(np.float32).view(np.uint32)
    raw[:, 4] = p[:, 4].astype(np.uint64).astype(np.uint32)
    return torch.from_numpy(raw.view(np.int32).copy()).to(device)
