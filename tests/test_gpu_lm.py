"""GPU registration against the reference's solver.

The HIP registration runs the reference's Ceres LM (PF_SOLVER_LM, the default) from the fp64
moment sums; pf_set_solver(PF_SOLVER_NORMAL) gives the exact least-squares minimiser instead.
Both are held to the tolerances stated in DESIGN.md section 4 against the oracle's sample-wise
restatement of Ceres 1.13 LM (oracle/pf_oracle_lm.c, merge_lm):

  HIP LM (default) vs Ceres-LM restatement       fused u16 max <= 2 LSB, <= 0.1 % pixels differ;
                                                  coefficients relative <= 1e-5
  HIP normal equations vs Ceres-LM restatement   fused u16 max <= 8 LSB, >= 99 % within 1 LSB
  HIP LM vs the oracle's moment-form LM           bit-exact (coefficients fp64 and u16)
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import panofuse  # noqa: E402
import pf_layouts as PL  # noqa: E402
import pf_synth  # noqa: E402
import pyoracle as O  # noqa: E402

ZR = PL.ZENITH_RANGE
DEV = "cuda:0"
CFGS = {"C1": (512, 128), "C2": (2048, 512)}


@pytest.fixture(scope="module")
def fuser():
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a host without a GPU")
    return panofuse.Fuser(0)


def _inputs(cfg, seed):
    out_w, ew = CFGS[cfg]
    lay = PL.config_layout(cfg)
    tiles, total = O.make_tiles(lay)
    seeds = pf_synth.seeds_for(1, 20261015 + 1000 * seed)
    emap = pf_synth.baseline_emap(seeds, ew, ew // 2)[0].numpy()
    gt = pf_synth.scene_depth(seeds, out_w, out_w // 2)[0].numpy()
    data = O.warp_depth(gt, tiles, total, O.responses(pf_synth.responses(seeds, lay.ntiles)))
    return lay, tiles, emap, data, out_w


def _merge(fuser, lay, emap, data, out_w, solver):
    fuser.set_tiles(lay)
    fuser.set_solver(solver)
    try:
        out = torch.zeros((1, out_w // 2, out_w), dtype=torch.int16, device=DEV)
        coeffs = torch.zeros((1, lay.ntiles, 4), dtype=torch.float32, device=DEV)
        fuser.merge(torch.from_numpy(emap)[None].to(DEV), torch.from_numpy(data)[None].to(DEV),
                    out, ZR, coeffs=coeffs)
        return out.cpu().numpy().view(np.uint16)[0].astype(np.int64), coeffs.cpu().numpy()[0]
    finally:
        fuser.set_solver("lm")


@pytest.mark.parametrize("cfg,seed", [("C1", 0), ("C1", 3), ("C2", 0), ("C2", 3)])
def test_merge_vs_ceres_lm_restatement(fuser, cfg, seed):
    lay, tiles, emap, data, out_w = _inputs(cfg, seed)
    ref, ref_abcd = O.merge_lm(emap, tiles, data.copy(), out_w, ZR)
    lm, lm_abcd = _merge(fuser, lay, emap, data, out_w, "lm")
    d = np.abs(lm - ref)
    assert d.max() <= 2 and (d > 0).mean() <= 1e-3, (d.max(), (d > 0).mean())
    rel = np.abs(lm_abcd.astype(np.float64) - ref_abcd) / np.maximum(np.abs(ref_abcd), 1e-6)
    assert rel.max() <= 1e-5
    ne, _ = _merge(fuser, lay, emap, data, out_w, "normal")
    d = np.abs(ne - ref)
    assert d.max() <= 8 and (d <= 1).mean() >= 0.99, (d.max(), (d <= 1).mean())
    # and the HIP LM is the oracle's moment-form LM bit for bit
    mom, mom_abcd = O.merge(emap, tiles, data.copy(), out_w, ZR, solver="lm")
    assert np.array_equal(lm_abcd, mom_abcd)
    assert int((lm != mom).sum()) == 0


def test_register_lm_fp64_bit_exact(fuser):
    """coeffs64 of the HIP LM == the oracle's moment-form LM, every tile of C2."""
    lay, tiles, emap, data, _ = _inputs("C2", 5)
    fuser.set_tiles(lay)
    c64 = torch.zeros((1, lay.ntiles, 4), dtype=torch.float64, device=DEV)
    fuser.register(torch.from_numpy(emap)[None].to(DEV), torch.from_numpy(data)[None].to(DEV),
                   ZR, apply=False, coeffs64=c64)
    got = c64.cpu().numpy()[0]
    for p in range(lay.ntiles):
        r64, _, _ = O.register_tile(tiles[p], data, emap, ZR, solver="lm")
        assert np.array_equal(got[p], r64), p
