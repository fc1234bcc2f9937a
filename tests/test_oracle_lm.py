"""The registration solver restated: Ceres 1.13 Levenberg-Marquardt (oracle/pf_oracle_lm.c).

SolveDepthToDepth solves its cubic fit with Ceres LM from (1,1,1,1) and stops on
function_tolerance 1e-6 (Depth.cpp:1270-1274, 1399-1404; ceres solver.h:62-128), i.e. before the
exact least-squares minimiser.  The oracle carries two restatements of that run:

* pfo_lm_fit / merge_lm -- sample-wise, as Ceres evaluates it (one residual per sample, Jacobi
  scaling, DENSE_SCHUR with `a` eliminated, Eigen LLT); parity anchor for the reference solver;
* pfo_lm_moments / merge(solver="lm") -- the same run from the 15 moment sums, the form the HIP
  kernel executes (bit-identical to it, tests/test_gpu_parity.py).

Stated tolerances, checked here on the CPU and on the GPU in
tests/test_gpu_lm.py:
  LM coefficients, moment vs sample-wise form   relative <= 1e-5 (ill-conditioned solve: the
                                                 fp64 rounding of each step is amplified)
  fused u16, moment LM (HIP default) vs sample  max <= 2 LSB, <= 0.1 % of pixels differ
  fused u16, normal equations vs sample LM      max <= 8 LSB, >= 99 % of pixels within 1 LSB
"""
import numpy as np
import pytest

import pf_layouts as PL
import pf_synth
import pyoracle as O

ZR = PL.ZENITH_RANGE
CFGS = {"C1": (512, 128), "C2": (2048, 512)}


def _inputs(cfg, seed):
    out_w, ew = CFGS[cfg]
    lay = PL.config_layout(cfg)
    tiles, total = O.make_tiles(lay)
    seeds = pf_synth.seeds_for(1, 20261015 + 1000 * seed)
    emap = pf_synth.baseline_emap(seeds, ew, ew // 2)[0].numpy()
    gt = pf_synth.scene_depth(seeds, out_w, out_w // 2)[0].numpy()
    data = O.warp_depth(gt, tiles, total, O.responses(pf_synth.responses(seeds, lay.ntiles)))
    return lay, tiles, emap, data, out_w


def test_lm_recovers_exact_cubic():
    """Noise-free samples of a cubic: LM converges to it (fitted values within 1e-6)."""
    rs = np.random.RandomState(1)
    x = np.sort(rs.uniform(0.1, 0.6, 3000))
    truth = np.array([0.8, -0.9, 1.2, 0.05])
    y = ((truth[0] * x + truth[1]) * x + truth[2]) * x + truth[3]
    c, s = O.lm_fit(x, y)
    A = np.stack([x ** 3, x ** 2, x, np.ones_like(x)], 1)
    assert np.max(np.abs(A @ c - y)) < 1e-6
    assert s["termination"] in ("function_tolerance", "gradient_tolerance", "parameter_tolerance")
    assert 1 <= s["iterations"] <= 50 and s["final_cost"] <= s["initial_cost"]
    cm, sm = O.lm_moments(_moments(x, y))
    assert np.max(np.abs(A @ cm - y)) < 1e-6


def _moments(x, y):
    X2, X3 = x * x, x * x * x
    return np.array([np.sum(X3 * X3), np.sum(X3 * X2), np.sum(X3 * x), np.sum(X3),
                     np.sum(X2 * X2), np.sum(X2 * x), np.sum(X2), np.sum(x * x), np.sum(x),
                     float(x.size), np.sum(X3 * y), np.sum(X2 * y), np.sum(x * y), np.sum(y),
                     np.sum(y * y)])


def test_lm_stops_before_the_minimiser():
    """Ceres stops on function_tolerance: its fit is near, not at, the least-squares minimiser
    (coefficients ~1 % apart, fitted values ~1e-5)."""
    lay, tiles, emap, data, _ = _inputs("C2", 0)
    far = 0
    for p in range(lay.ntiles):
        xs, ys, _, _ = O.reg_samples(tiles[p], data, emap, ZR)
        c_lm, s = O.lm_fit(xs, ys)
        c_ne, _, _ = O.register_tile(tiles[p], data, emap, ZR, solver="normal")
        A = np.stack([xs ** 3, xs ** 2, xs, np.ones_like(xs)], 1)
        assert s["termination"] == "function_tolerance", (p, s)
        assert 2 <= s["iterations"] <= 50
        fit = np.max(np.abs(A @ c_lm - A @ c_ne))
        assert fit < 1e-3, p
        # the LM cost is within a relative 1e-5 of the minimum (function_tolerance 1e-6/step)
        cost = lambda c: 0.5 * np.sum((A @ c - ys) ** 2)  # noqa: E731
        assert cost(c_lm) >= cost(c_ne) * (1 - 1e-12) and cost(c_lm) <= cost(c_ne) * (1 + 1e-4)
        far += int(np.max(np.abs(c_lm - c_ne) / np.abs(c_ne)) > 1e-4)
    assert far > 0  # the two solvers really differ


@pytest.mark.parametrize("cfg", ["C1", "C2"])
def test_lm_moment_form_matches_samplewise(cfg):
    lay, tiles, emap, data, _ = _inputs(cfg, 1)
    for p in range(lay.ntiles):
        cm, am, deg = O.register_tile(tiles[p], data, emap, ZR, solver="lm")
        cs, as_, s = O.register_tile_lm(tiles[p], data, emap, ZR)
        assert deg == 3
        rel = np.max(np.abs(cm - cs) / np.maximum(np.abs(cs), 1e-12))
        assert rel <= 1e-5, (p, rel)


@pytest.mark.parametrize("cfg", ["C1", "C2"])
def test_fused_u16_tolerances(cfg):
    """The stated end-to-end tolerances against the sample-wise Ceres restatement."""
    O.set_threads(4)
    for seed in (0, 3):
        lay, tiles, emap, data, out_w = _inputs(cfg, seed)
        ref, _ = O.merge_lm(emap, tiles, data.copy(), out_w, ZR)
        mom, _ = O.merge(emap, tiles, data.copy(), out_w, ZR, solver="lm")
        ne, _ = O.merge(emap, tiles, data.copy(), out_w, ZR, solver="normal")
        d = np.abs(mom.astype(np.int64) - ref)
        assert d.max() <= 2 and (d > 0).mean() <= 1e-3, (seed, d.max(), (d > 0).mean())
        d = np.abs(ne.astype(np.int64) - ref)
        assert d.max() <= 8 and (d <= 1).mean() >= 0.99, (seed, d.max(), (d <= 1).mean())


# ------------------------------------------------------------------------------------------------
# Reference-held pins for the LM restatement: Ceres 1.13's own unit tests of the strategy that
# SolveDepthToDepth's Solve runs (vendored in the reference as
# ceres-solver/internal/ceres/levenberg_marquardt_strategy_test.cc), replayed against the
# oracle's factored-out strategy (pfo_lms_*), which both LM forms -- and, through the moment form
# it is bit-identical to, the HIP kernel -- use.
import ctypes as C  # noqa: E402


class _Lms(C.Structure):
    _fields_ = [("radius", C.c_double), ("max_radius", C.c_double), ("decrease", C.c_double),
                ("min_diag", C.c_double), ("max_diag", C.c_double), ("reuse_diag", C.c_int),
                ("diag", C.c_double * 4)]


def _lms(initial_radius, max_radius, min_diag, max_diag):
    L = O.lib()
    L.pfo_lms_init.argtypes = [C.POINTER(_Lms)] + [C.c_double] * 4
    for f in (L.pfo_lms_accepted, L.pfo_lms_rejected):
        f.argtypes = [C.POINTER(_Lms), C.c_double]
    L.pfo_lms_regularizer.argtypes = [C.POINTER(_Lms), C.POINTER(C.c_double), C.c_int,
                                      C.POINTER(C.c_double)]
    s = _Lms()
    L.pfo_lms_init(C.byref(s), initial_radius, max_radius, min_diag, max_diag)
    return L, s


def test_ceres_lm_strategy_accept_reject_radius_scaling():
    """levenberg_marquardt_strategy_test.cc:81-110 (AcceptRejectStepRadiusScaling), with its
    exact EXPECT_EQs on the radius after each accept/reject."""
    L, s = _lms(2.0, 20.0, 1e-8, 1e8)
    assert s.radius == 2.0
    L.pfo_lms_rejected(C.byref(s), 0.0)
    assert s.radius == 1.0
    L.pfo_lms_rejected(C.byref(s), -1.0)
    assert s.radius == 0.25
    for q, expect in ((1.0, 0.25 * 3.0), (1.0, 0.25 * 3.0 * 3.0), (0.25, 0.25 * 3.0 * 3.0 / 1.125),
                      (1.0, 0.25 * 3.0 * 3.0 / 1.125 * 3.0),
                      (1.0, 0.25 * 3.0 * 3.0 / 1.125 * 3.0 * 3.0)):
        L.pfo_lms_accepted(C.byref(s), q)
        assert s.radius == expect, (q, s.radius, expect)
    L.pfo_lms_accepted(C.byref(s), 1.0)
    assert s.radius == 20.0  # capped at max_radius
    # a rejection after acceptances restarts the decrease factor at 2
    L.pfo_lms_rejected(C.byref(s), 0.0)
    assert s.radius == 10.0 and s.decrease == 4.0


def test_ceres_lm_strategy_correct_diagonal_to_linear_solver():
    """levenberg_marquardt_strategy_test.cc:113-160 (CorrectDiagonalToLinearSolver): for the
    Jacobian [[0, 1, 100], [0, 1, 0]] with min/max LM diagonal 1e-2/1e2 and radius 2, the D
    handed to the linear solver is sqrt({1e-2, 2, 1e2} / 2) -- the squared column norms
    {0, 2, 1e4} clamped.  Also: the diagonal is reused after a rejection (only D's radius
    changes) and recomputed after an acceptance."""
    L, s = _lms(2.0, 20.0, 1e-2, 1e2)
    J = np.array([[0.0, 1.0, 100.0], [0.0, 1.0, 0.0]])
    colsq = np.ascontiguousarray((J * J).sum(0))
    D = np.zeros(3)
    dp = C.POINTER(C.c_double)
    L.pfo_lms_regularizer(C.byref(s), colsq.ctypes.data_as(dp), 3, D.ctypes.data_as(dp))
    expect = np.sqrt(np.array([1e-2, 2.0, 1e2]) / 2.0)
    assert np.allclose(D, expect, rtol=0, atol=1e-16), (D, expect)
    L.pfo_lms_rejected(C.byref(s), 0.0)  # radius 1, diagonal reused even for new norms
    other = np.array([5.0, 5.0, 5.0])
    L.pfo_lms_regularizer(C.byref(s), other.ctypes.data_as(dp), 3, D.ctypes.data_as(dp))
    assert np.allclose(D, np.sqrt(np.array([1e-2, 2.0, 1e2]) / 1.0), rtol=0, atol=1e-16)
    L.pfo_lms_accepted(C.byref(s), 1.0)  # radius 3, diagonal recomputed
    L.pfo_lms_regularizer(C.byref(s), other.ctypes.data_as(dp), 3, D.ctypes.data_as(dp))
    assert np.allclose(D, np.sqrt(other / 3.0), rtol=0, atol=1e-16)
