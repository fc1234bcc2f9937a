"""SolveDepthBySmoothing (Depth.cpp:1773-1878) on the GPU against the oracle.

pf_solve_smoothing reproduces the reference's lexicographic in-place Gauss-Seidel with a
wavefront schedule (pf_smooth.hip); bar: bit-exact u16 output.  Parity against the reference
itself is unpinned (pf_oracle.h), as for every path here.
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
CFGS = {"C1": 512, "C2": 2048, "LERES": 1024}


@pytest.fixture(scope="module")
def fuser():
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a host without a GPU")
    return panofuse.Fuser(0)


def _tiles(cfg, seed, n=1):
    out_w = CFGS[cfg]
    lay = PL.config_layout(cfg)
    tiles, total = O.make_tiles(lay)
    datas = []
    for k in range(n):
        seeds = pf_synth.seeds_for(1, 20261015 + 97 * seed + k)
        gt = pf_synth.scene_depth(seeds, out_w, out_w // 2)[0].numpy()
        resp = pf_synth.responses(seeds, lay.ntiles)
        datas.append(O.warp_depth(gt, tiles, total, O.responses(resp)))
    return lay, tiles, np.stack(datas), out_w


@pytest.mark.parametrize("cfg,batch", [("C1", 3), ("C2", 2), ("LERES", 1)])
def test_smoothing_bit_exact(fuser, cfg, batch):
    lay, tiles, data, out_w = _tiles(cfg, 1, batch)
    fuser.set_tiles(lay)
    out = torch.zeros((batch, out_w // 2, out_w), dtype=torch.int16, device=DEV)
    fuser.solve_smoothing(torch.from_numpy(data).to(DEV), out, ZR)
    got = out.cpu().numpy().view(np.uint16)
    for b in range(batch):
        ref = O.solve_smoothing(tiles, np.ascontiguousarray(data[b]), out_w, out_w // 2, ZR)
        bad = int((got[b] != ref).sum())
        assert bad == 0, f"{cfg} panorama {b}: {bad} pixels differ (max |d| " \
                         f"{int(np.abs(got[b].astype(np.int64) - ref).max())})"
        assert int((ref != 0).sum()) > out_w  # non-trivial output


def test_smoothing_with_transform_equals_pretransformed(fuser):
    """coeffs applied on the fly == Depth2DepthTransform applied to the tiles first."""
    lay, tiles, data, out_w = _tiles("C1", 2, 2)
    rng = np.random.default_rng(5)
    coeffs = np.zeros((2, lay.ntiles, 4), np.float32)
    coeffs[:, :, 0] = rng.uniform(-0.3, 0.3, (2, lay.ntiles))
    coeffs[:, :, 1] = rng.uniform(-0.3, 0.3, (2, lay.ntiles))
    coeffs[:, :, 2] = rng.uniform(0.8, 1.2, (2, lay.ntiles))
    coeffs[:, :, 3] = rng.uniform(-0.05, 0.05, (2, lay.ntiles))
    fuser.set_tiles(lay)
    out = torch.zeros((2, out_w // 2, out_w), dtype=torch.int16, device=DEV)
    fuser.solve_smoothing(torch.from_numpy(data).to(DEV), out, ZR,
                          coeffs=torch.from_numpy(coeffs).to(DEV))
    got = out.cpu().numpy().view(np.uint16)
    for b in range(2):
        d = np.ascontiguousarray(data[b]).copy()
        for p in range(lay.ntiles):
            O.depth_to_depth(tiles[p], d, coeffs[b, p])
        ref = O.solve_smoothing(tiles, d, out_w, out_w // 2, ZR)
        assert int((got[b] != ref).sum()) == 0


def test_smoothing_rejects_stencil_outside(fuser):
    lay, tiles, data, out_w = _tiles("C1", 3, 1)
    fuser.set_tiles(lay)
    out = torch.zeros((1, out_w // 2, out_w), dtype=torch.int16, device=DEV)
    with pytest.raises(RuntimeError):
        fuser.solve_smoothing(torch.from_numpy(data).to(DEV), out, (0.0, ZR[1]))


@pytest.mark.parametrize("nb", ["0", "2", "3", "7", "64"])
def test_smoothing_row_blocks_equal(fuser, nb, monkeypatch):
    """The row-band form (k_smooth_band: a panorama's Gauss-Seidel steps spread over nb
    workgroups with a step hand-off between neighbouring row blocks) equals the one-workgroup
    form (PF_SMOOTH_BAND=0) bit for bit, for several block counts; then the oracle at one."""
    lay, tiles, data, out_w = _tiles("C2", 4, 2)
    fuser.set_tiles(lay)
    t = torch.from_numpy(data).to(DEV)
    monkeypatch.setenv("PF_SMOOTH_BAND", "0")
    ref = torch.zeros((2, out_w // 2, out_w), dtype=torch.int16, device=DEV)
    fuser.solve_smoothing(t, ref, ZR)
    monkeypatch.setenv("PF_SMOOTH_BAND", nb)
    got = torch.zeros_like(ref)
    fuser.solve_smoothing(t, got, ZR)
    fuser.synchronize()  # PF_ETIMEOUT if a step hand-off timed out
    assert torch.equal(got, ref)
    if nb == "7":
        r0 = O.solve_smoothing(tiles, np.ascontiguousarray(data[0]), out_w, out_w // 2, ZR)
        assert np.array_equal(got.cpu().numpy().view(np.uint16)[0], r0)


def test_smoothing_timeout_is_reported(fuser, monkeypatch):
    """a row-band hand-off wait that times out must surface as PF_ETIMEOUT on the
    smoothing call's own report (pf_synchronize, or the next call), not as a silently wrong
    output or a later fusion's failure.  The fault hook makes row block 0 withhold its step
    flags in one launch, waits bounded at 2^10 polls; after a timeout a workgroup stops waiting,
    so the faulty launch still ends quickly.  The launches after it are bit-exact again."""
    lay, tiles, data, out_w = _tiles("C2", 4, 2)
    fuser.set_tiles(lay)
    t = torch.from_numpy(data).to(DEV)
    monkeypatch.setenv("PF_SMOOTH_BAND", "7")
    ref = torch.zeros((2, out_w // 2, out_w), dtype=torch.int16, device=DEV)
    fuser.solve_smoothing(t, ref, ZR)
    fuser.synchronize()
    # 1. reported by pf_synchronize
    got = torch.zeros_like(ref)
    fuser.debug_smooth_fault(10)
    fuser.solve_smoothing(t, got, ZR)
    with pytest.raises(panofuse.PanofuseError) as e:
        fuser.synchronize()
    assert e.value.code == panofuse.PF_ETIMEOUT and "timed out" in str(e.value)
    # 2. the next launch runs normally and is bit-exact
    fuser.solve_smoothing(t, got, ZR)
    fuser.synchronize()
    assert torch.equal(got, ref)
    # 3. reported by the next smoothing call once the faulty one has finished
    fuser.debug_smooth_fault(10)
    fuser.solve_smoothing(t, got, ZR)
    torch.cuda.synchronize()
    with pytest.raises(panofuse.PanofuseError) as e:
        fuser.solve_smoothing(t, got, ZR)
    assert e.value.code == panofuse.PF_ETIMEOUT
    fuser.solve_smoothing(t, got, ZR)
    fuser.synchronize()
    assert torch.equal(got, ref)
