"""CPU checks of the metrics oracle (ErrorData/ErrorEmap restatement, Depth.cpp:1980-2458)
against an independent numpy statement of the same definitions: medians are the element at
index n//2 of the sorted compare values, counts are exact, the means agree to fp32 summation
rounding.  (Parity with the reference itself is unpinned: it ships no metric fixtures.)"""
import numpy as np
import pytest

import pf_layouts as PL
import pyoracle as O

MYPI = 3.14159265359


def _np_metrics(gt, given, zr, align_way, cap):
    h, w = given.shape[:2]
    gh, gw = gt.shape[:2]
    g0 = gt if gt.ndim == 2 else gt[..., 0]
    v = given.astype(np.float32) / np.float32(65535.0) if given.dtype == np.uint16 else (
        given if given.ndim == 2 else given[..., 0])
    h0, h1 = int(float(zr[0]) / MYPI * h), int(float(zr[1]) / MYPI * h)
    rx, ry = np.float32(gw) / np.float32(w), np.float32(gh) / np.float32(h)
    xs = np.minimum((np.arange(w, dtype=np.float32) * rx).astype(np.int64), gw - 1)
    ys = np.minimum((np.arange(h0, h1 + 1, dtype=np.float32) * ry).astype(np.int64), gh - 1)
    a = g0[ys][:, xs].astype(np.float32)
    b = v[h0:h1 + 1].astype(np.float32)
    m = a.astype(np.float64) >= 1e-4
    a, b = a[m], b[m]
    if cap:
        dm = np.float32(10.0) / (np.float32(65535.0) / np.float32(4000.0))
        a, b = np.minimum(a, dm), np.minimum(b, dm)
    r = {"n": a.size}
    if align_way == 1:
        r["gt_median"] = float(np.sort(a)[a.size // 2])
        r["given_median"] = float(np.sort(b)[b.size // 2])
        b = b * np.float32(r["gt_median"] / np.float32(r["given_median"]))
    d = (a - b).astype(np.float64)
    r["mse"], r["mae"] = float((d * d).mean()), float(np.abs(d).mean())
    pos = (a > 0) & (b > 0)
    rm = np.maximum(a[pos] / b[pos], b[pos] / a[pos])
    r["delta1"] = float(np.float32(a.size - int((rm >= 1.25).sum())) / np.float32(a.size))
    return r


@pytest.mark.parametrize("align_way", [0, 1])
@pytest.mark.parametrize("given_kind", ["u16", "f32"])
def test_metrics_oracle_vs_numpy(align_way, given_kind):
    rng = np.random.default_rng(3)
    gt = rng.uniform(0, 0.4, (300, 600)).astype(np.float32)
    gt[rng.random(gt.shape) < 0.1] = 0
    if given_kind == "u16":
        given = (np.clip(gt[::2, ::2] * 1.2 + rng.normal(0, .02, (150, 300)), 0, 1) * 65535
                 ).astype(np.uint16)
    else:
        given = (gt[::2, ::2] * 0.9 + rng.normal(0, .02, (150, 300))).astype(np.float32)
    ref = _np_metrics(gt, given, PL.ZENITH_RANGE, align_way, True)
    got = O.error_metrics(gt, given, PL.ZENITH_RANGE, align_way, True)
    assert got["n"] == ref["n"]
    if align_way == 1:
        assert got["gt_median"] == ref["gt_median"]
        assert got["given_median"] == ref["given_median"]
    assert got["delta1"] == pytest.approx(ref["delta1"], abs=2e-7)
    assert got["mse"] == pytest.approx(ref["mse"], rel=1e-4)
    assert got["mae"] == pytest.approx(ref["mae"], rel=1e-4)


def test_metrics_oracle_empty_is_nan():
    got = O.error_metrics(np.zeros((64, 128), np.float32), np.ones((32, 64), np.uint16),
                          PL.ZENITH_RANGE, 1, True)
    assert got["n"] == 0 and np.isnan(got["mse"]) and np.isnan(got["median_shift"])


def test_u16_unit_reciprocal_form_is_exact():
    """The metrics kernel's u16_unit (x * rcp refined by one fma, pf_metrics.hip) equals the
    correctly rounded (float)u / 65535.0f for every u16: emulated here with fp64 (the fma
    products are exact in fp64, the single roundings are np.float32 casts)."""
    u = np.arange(65536, dtype=np.float64)
    rcp = np.float64(np.float32(1.0) / np.float32(65535.0))
    q = np.float32(u * rcp).astype(np.float64)
    r = np.float32(u - q * 65535.0).astype(np.float64)
    q2 = np.float32(r * rcp + q)
    ref = u.astype(np.float32) / np.float32(65535.0)
    assert np.array_equal(q2, ref)
