"""GPU parity: the HIP path (through the C-ABI) against the CPU oracle on identical inputs.

Bars: bit-exact for everything -- tile index maps, level seeds, Laplacian
targets, Jacobi buffers, registration coefficients, the u16 output, and the E->P warps (depth
tiles and RGB tiles: their coordinate maps are built on the host with glibc atan2f / atan2, as
the reference and the oracle call them, so the warped tiles are array_equal to the oracle's).
Oracle parity against the reference itself is unpinned (pf_oracle.h).
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


def _inputs(cfg, seed=0):
    out_w, ew = CFGS[cfg]
    lay = PL.config_layout(cfg)
    seeds = pf_synth.seeds_for(1, 20261015 + 101 * seed)
    emap = pf_synth.baseline_emap(seeds, ew, ew // 2)[0].numpy()
    gt = pf_synth.scene_depth(seeds, out_w, out_w // 2)[0].numpy()
    tiles, total = O.make_tiles(lay)
    resp = pf_synth.responses(seeds, lay.ntiles)
    data = O.warp_depth(gt, tiles, total, O.responses(resp))
    return lay, emap, gt, tiles, total, data, resp


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


@pytest.mark.parametrize("cfg", ["C1", "C2", "LERES"])
def test_tap_index_maps_bit_exact(fuser, cfg):
    lay = PL.config_layout(cfg)
    out_w = 2048 if cfg != "C1" else 512
    fuser.set_tiles(lay)
    tiles, _ = O.make_tiles(lay)
    for level in range(O.num_levels(out_w)):
        got = fuser.probe_taps(out_w, ZR, level).cpu().numpy()
        ref = O.probe_taps(tiles, O.level_dims(out_w, out_w // 2, ZR, level))
        assert got.shape == ref.shape
        bad = int((got != ref).sum())
        assert bad == 0, f"{cfg} level {level}: {bad} tap indices differ"


@pytest.mark.parametrize("cfg", ["C1", "C2"])
def test_level_internals_bit_exact(fuser, cfg):
    lay, emap, gt, tiles, total, data, _ = _inputs(cfg)
    out_w = CFGS[cfg][0]
    fuser.set_tiles(lay)
    t_tiles = _dev(data)
    t_emap = _dev(emap)[None]
    prev_gpu = None
    prev_ref = None
    for level in range(O.num_levels(out_w)):
        lv = O.level_dims(out_w, out_w // 2, ZR, level)
        buf = torch.zeros(lv.h * lv.w, dtype=torch.float32, device=DEV)
        fuser.fuse_seed(t_emap if level == 0 else None, prev_gpu, out_w, ZR, level, buf)
        ref_seed = O.seed_level0(emap, lv) if level == 0 else O.upsample(prev_ref, lv)
        assert np.array_equal(buf.cpu().numpy().reshape(lv.h, lv.w), ref_seed), f"seed L{level}"
        lsum = torch.zeros(lv.h * lv.w, dtype=torch.float32, device=DEV)
        cnt = torch.zeros_like(lsum)
        fuser.fuse_partial(t_tiles, None, 0, lay.ntiles, out_w, ZR, level, lsum, cnt)
        rL, rn, oops, _ = O.targets(tiles, data, lv)
        assert oops == 0
        band = slice(lv.h0, lv.h1 + 1)
        g_l = lsum.cpu().numpy().reshape(lv.h, lv.w)[band]
        g_n = cnt.cpu().numpy().reshape(lv.h, lv.w)[band]
        assert np.array_equal(g_n, rn[band].astype(np.float32)), f"coverage L{level}"
        assert np.array_equal(g_l.view(np.uint32), rL[band].view(np.uint32)), f"targets L{level}"
        fuser.fuse_finish_level(lsum, cnt, out_w, ZR, level, buf)
        ref_buf = O.jacobi(ref_seed, O.normalize(rL, rn, lv), lv, lv.iters)
        got = buf.cpu().numpy().reshape(lv.h, lv.w)
        bad = int((got.view(np.uint32) != ref_buf.view(np.uint32)).sum())
        assert bad == 0, f"{cfg} level {level}: {bad} Jacobi values differ"
        prev_gpu, prev_ref = buf, ref_buf


@pytest.mark.parametrize("cfg", ["C1", "C2"])
def test_register_bit_exact(fuser, cfg):
    lay, emap, gt, tiles, total, data, _ = _inputs(cfg)
    fuser.set_tiles(lay)
    t_tiles = _dev(data)[None].contiguous()
    coeffs = torch.zeros((1, lay.ntiles, 4), dtype=torch.float32, device=DEV)
    c64 = torch.zeros((1, lay.ntiles, 4), dtype=torch.float64, device=DEV)
    fuser.register(_dev(emap)[None], t_tiles, ZR, degree=3, apply=True, coeffs=coeffs,
                   coeffs64=c64)
    ref = data.copy()
    for p in range(lay.ntiles):
        r64, rabcd, deg = O.register_tile(tiles[p], data, emap, ZR)
        assert deg == 3
        assert np.array_equal(c64.cpu().numpy()[0, p], r64), f"tile {p} fp64 solution"
        assert np.array_equal(coeffs.cpu().numpy()[0, p], rabcd), f"tile {p} abcd"
        O.depth_to_depth(tiles[p], ref, rabcd)
    assert np.array_equal(t_tiles.cpu().numpy()[0].view(np.uint32), ref.view(np.uint32))


def test_register_degree1_and_lstsq(fuser):
    """Scale/shift mode (north_star's 2x2 system) and agreement with an fp64 lstsq (the
    normal-equation solver; the default LM solver is checked in test_gpu_lm.py)."""
    lay, emap, gt, tiles, total, data, _ = _inputs("C1")
    fuser.set_tiles(lay)
    fuser.set_solver("normal")
    for degree in (1, 2, 3):
        coeffs = torch.zeros((1, lay.ntiles, 4), dtype=torch.float32, device=DEV)
        c64 = torch.zeros((1, lay.ntiles, 4), dtype=torch.float64, device=DEV)
        fuser.register(_dev(emap)[None], _dev(data)[None].contiguous(), ZR, degree=degree,
                       apply=False, coeffs=coeffs, coeffs64=c64)
        for p in range(lay.ntiles):
            xs, ys, _, _ = O.reg_samples(tiles[p], data, emap, ZR)
            A = np.stack([xs ** k for k in range(degree, -1, -1)], 1)
            sol, *_ = np.linalg.lstsq(A, ys, rcond=None)
            got = c64.cpu().numpy()[0, p][3 - degree:]
            assert np.max(np.abs(A @ got - A @ sol)) < 1e-6
    fuser.set_solver("lm")


@pytest.mark.parametrize("cfg", ["C1", "C2"])
def test_fuse_bit_exact(fuser, cfg):
    lay, emap, gt, tiles, total, data, _ = _inputs(cfg, seed=3)
    out_w = CFGS[cfg][0]
    fuser.set_tiles(lay)
    out = torch.zeros((1, out_w // 2, out_w), dtype=torch.int16, device=DEV)
    fuser.fuse(_dev(emap)[None], _dev(data)[None].contiguous(), out, ZR)
    ref, _ = O.solve_depth_all(emap, tiles, data, out_w, ZR)
    got = out.cpu().numpy().view(np.uint16)[0]
    assert int((got != ref).sum()) == 0


@pytest.mark.parametrize("cfg", ["C1", "C2"])
def test_merge_bit_exact_batched(fuser, cfg):
    """MergeDepthMaps core for a batch of 3 panoramas == the oracle per panorama."""
    out_w, ew = CFGS[cfg]
    lay = PL.config_layout(cfg)
    fuser.set_tiles(lay)
    tiles, total = O.make_tiles(lay)
    seeds = pf_synth.seeds_for(3, 777)
    emaps = pf_synth.baseline_emap(seeds, ew, ew // 2).numpy()
    gts = pf_synth.scene_depth(seeds, out_w, out_w // 2).numpy()
    resp = pf_synth.responses(seeds, lay.ntiles)
    datas = np.stack([O.warp_depth(gts[b], tiles, total,
                                   O.responses(resp[b * lay.ntiles:(b + 1) * lay.ntiles]))
                      for b in range(3)])
    out = torch.zeros((3, out_w // 2, out_w), dtype=torch.int16, device=DEV)
    coeffs = torch.zeros((3, lay.ntiles, 4), dtype=torch.float32, device=DEV)
    t_tiles = _dev(datas)
    fuser.merge(_dev(emaps), t_tiles, out, ZR, coeffs=coeffs)
    got = out.cpu().numpy().view(np.uint16)
    assert np.array_equal(t_tiles.cpu().numpy(), datas), "merge must not modify the tiles"
    for b in range(3):
        ref, abcd = O.merge(emaps[b], tiles, datas[b].copy(), out_w, ZR)
        assert np.array_equal(coeffs.cpu().numpy()[b], abcd)
        assert int((got[b] != ref).sum()) == 0, f"pano {b}"


@pytest.mark.parametrize("cfg", ["C1", "C2"])
def test_warp_depth_bit_exact(fuser, cfg):
    """The coordinate map is built on the host with glibc atan2f (tests/test_warp_maps.py pins
    it to the oracle), the bilinear blend and the response run in the oracle's fp32 order: every
    tile pixel equals the oracle's bit for bit."""
    lay, emap, gt, tiles, total, data, resp = _inputs(cfg)
    fuser.set_tiles(lay)
    out = torch.zeros((2, total), dtype=torch.float32, device=DEV)
    r = panofuse.make_responses(np.concatenate([resp, resp]), DEV)
    fuser.warp_depth(_dev(np.stack([gt, gt])), out, r)
    got = out.cpu().numpy()
    assert np.array_equal(got[0], data)
    assert np.array_equal(got[0], got[1])
    # without the response: plain bilinear E->P gather
    out2 = torch.zeros((1, total), dtype=torch.float32, device=DEV)
    fuser.warp_depth(_dev(gt)[None], out2)
    ref2 = O.warp_depth(gt, tiles, total, None)
    assert np.array_equal(out2.cpu().numpy()[0], ref2)


def test_warp_depth_ragged_batch_and_resize(fuser):
    """Batch 19 (one full 16-panorama chunk + a ragged one), distinct responses per panorama,
    then other panorama sizes on the same context (the cached warp map must follow): 300 wide
    stages 16-B quads, 302 wide (not a multiple of 4) the 4-B staging path."""
    lay = PL.config_layout("C1")
    fuser.set_tiles(lay)
    tiles, total = O.make_tiles(lay)
    B = 19
    seeds = pf_synth.seeds_for(B, 777)
    resp = pf_synth.responses(seeds, lay.ntiles)
    for (pw, ph) in ((512, 256), (300, 150), (302, 151)):
        gt = pf_synth.scene_depth(seeds, pw, ph).numpy()
        out = torch.zeros((B, total), dtype=torch.float32, device=DEV)
        fuser.warp_depth(_dev(gt), out, panofuse.make_responses(resp, DEV))
        got = out.cpu().numpy()
        for b in (0, 15, 16, 18):
            nt = lay.ntiles
            ref = O.warp_depth(gt[b], tiles, total, O.responses(resp[b * nt:(b + 1) * nt]))
            assert np.array_equal(got[b], ref), (pw, b)


def test_warp_rgb_bit_exact(fuser):
    lay = PL.config_layout("C1")
    fuser.set_tiles(lay)
    tiles, _ = O.make_tiles(lay)
    rs = np.random.RandomState(5)
    h, w = 256, 512
    yy, xx = np.mgrid[0:h, 0:w]
    pano = np.stack([(xx * 255 // (w - 1)), (yy * 255 // (h - 1)),
                     rs.randint(0, 256, size=(h, w))], -1).astype(np.uint8)
    ref = O.warp_rgb(pano, tiles)
    out = torch.zeros((1, ref.size), dtype=torch.uint8, device=DEV)
    fuser.warp_rgb(_dev(pano)[None], out)
    got = out.cpu().numpy()[0].astype(np.int32)
    d = np.abs(got - ref.astype(np.int32))
    assert d.max() == 0  # host-built taps (glibc atan2), fp32 GL_LINEAR as the oracle


@pytest.mark.parametrize("pw,ph,B", [(2048, 1024, 18), (1000, 500, 3), (1024, 512, 1)])
def test_warp_rgb_staged_bit_exact(pw, ph, B, monkeypatch):
    """The RGB warp at the C2/C3 layout (20 tiles of 512^2): the LDS-staged kernel
    (k_warp_rgb_box; 64x16 patches, 16 panoramas per block, so batch 18 crosses a block's
    panorama chunk) equals the oracle's GL-camera restatement for every byte, and equals the
    per-pixel kernel (PF_WARP_RGB_NAIVE=1) on the whole batch.  pw = 1000 (3*pw not a multiple
    of 16) takes the per-pixel kernel; both must agree with the oracle."""
    lay = PL.config_layout("C2")
    tiles, _ = O.make_tiles(lay)
    rs = np.random.RandomState(pw + B)
    pano = rs.randint(0, 256, size=(B, ph, pw, 3)).astype(np.uint8)
    pano[0, :, :, 0] = (np.arange(pw) * 255 // (pw - 1)).astype(np.uint8)[None, :]
    outs = []
    for naive in ("0", "1"):
        monkeypatch.setenv("PF_WARP_RGB_NAIVE", naive)
        f = panofuse.Fuser(0)  # a new context rebuilds the taps under this setting
        f.set_tiles(lay)
        n = sum(int(lay.tile_w[i]) * int(lay.tile_h[i]) * 3 for i in range(lay.ntiles))
        out = torch.zeros((B, n), dtype=torch.uint8, device=DEV)
        f.warp_rgb(_dev(pano), out)
        torch.cuda.synchronize()
        outs.append(out.cpu().numpy())
        f.close()
    assert np.array_equal(outs[0], outs[1])
    for b in sorted({0, B - 1}):
        ref = O.warp_rgb(pano[b], tiles)
        assert np.array_equal(outs[0][b], ref), b


def test_sharded_partial_sum_equals_full(fuser):
    """C5-style tile sharding: per-shard (sum L, n) grids summed == all tiles at once."""
    lay, emap, gt, tiles, total, data, _ = _inputs("C2")
    fuser.set_tiles(lay)
    t_tiles = _dev(data)
    lv = O.level_dims(2048, 1024, ZR, 2)
    full_l = torch.zeros(lv.h * lv.w, dtype=torch.float32, device=DEV)
    full_n = torch.zeros_like(full_l)
    fuser.fuse_partial(t_tiles, None, 0, lay.ntiles, 2048, ZR, 2, full_l, full_n)
    acc_l = torch.zeros_like(full_l)
    acc_n = torch.zeros_like(full_l)
    for t0 in range(0, lay.ntiles, 5):
        l = torch.zeros_like(full_l)
        n = torch.zeros_like(full_l)
        fuser.fuse_partial(t_tiles, None, t0, t0 + 5, 2048, ZR, 2, l, n)
        acc_l += l
        acc_n += n
    assert torch.equal(acc_n, full_n)
    assert torch.equal(acc_l.view(torch.int32), full_l.view(torch.int32))


def test_error_paths(fuser):
    lay = PL.config_layout("C1")
    fuser.set_tiles(lay)
    emap = torch.zeros((1, 64, 128), dtype=torch.float32, device=DEV)
    tiles = torch.zeros((1, fuser.tile_elems), dtype=torch.float32, device=DEV)
    out = torch.zeros((1, 251, 502), dtype=torch.int16, device=DEV)
    with pytest.raises(panofuse.PanofuseError) as e:
        fuser.fuse(emap, tiles, out, ZR)  # 502 does not halve twice (levels 125/251/502)
    assert e.value.code == panofuse.PF_EINVAL
    with pytest.raises(panofuse.PanofuseError) as e:
        fuser.register(emap, tiles, ZR, degree=7)
    assert e.value.code == panofuse.PF_EINVAL
    # a tile whose range collapses to one column at level 0 is rejected, not looped on
    bad = PL.Layout("bad", lay.fovs[:1].copy(), lay.ranges[:1].copy(), lay.tile_w[:1],
                    lay.tile_h[:1])
    bad.ranges[0, 1] = bad.ranges[0, 0] - np.float32(1e-4)
    fuser.set_tiles(bad)
    out = torch.zeros((1, 256, 512), dtype=torch.int16, device=DEV)
    with pytest.raises(panofuse.PanofuseError) as e:
        fuser.fuse(emap, tiles[:, : 256 * 256].contiguous(), out, ZR)
    assert e.value.code == panofuse.PF_EDEGENERATE


@pytest.mark.parametrize("zr_deg", [(3.0, 177.0), (12.0, 150.0)])
def test_fuse_bit_exact_wide_zenith(fuser, zr_deg):
    """Zenith bands reaching near the poles: levels whose band leaves too little room for the
    streaming engine's halo rows take the per-sweep kernel; both must match the oracle."""
    zr = (np.float32(PL.D2R(zr_deg[0])), np.float32(PL.D2R(zr_deg[1])))
    lay = PL.band_layout(5, 4, 256, 256, 3, 12, "wide", z_lo=zr_deg[0] + 1, z_hi=zr_deg[1] - 1)
    fuser.set_tiles(lay)
    tiles, total = O.make_tiles(lay)
    rs = np.random.RandomState(11)
    data = rs.rand(total).astype(np.float32)
    emap = rs.rand(128, 256).astype(np.float32)
    out = torch.zeros((1, 512, 1024), dtype=torch.int16, device=DEV)
    fuser.fuse(_dev(emap)[None], _dev(data)[None].contiguous(), out, zr)
    ref, _ = O.solve_depth_all(emap, tiles, data, 1024, zr)
    assert int((out.cpu().numpy().view(np.uint16)[0] != ref).sum()) == 0


def test_fuse_bit_exact_coverage_holes(fuser):
    """A layout with uncovered band pixels (two tiles dropped from C2) has no standard-coverage
    certificate, so every level takes the general (scalar, marker-masked) Jacobi form; the full
    C2 layout takes the packed form (test_fuse_bit_exact).  Both must match the oracle."""
    full = PL.config_layout("C2")
    keep = [i for i in range(full.ntiles) if i not in (6, 13)]
    lay = PL.Layout("C2-holes", full.fovs[keep], full.ranges[keep], full.tile_w[keep],
                    full.tile_h[keep])
    fuser.set_tiles(lay)
    tiles, total = O.make_tiles(lay)
    rs = np.random.RandomState(5)
    data = rs.rand(total).astype(np.float32)
    emap = rs.rand(256, 512).astype(np.float32)
    out = torch.zeros((1, 1024, 2048), dtype=torch.int16, device=DEV)
    fuser.fuse(_dev(emap)[None], _dev(data)[None].contiguous(), out, ZR)
    ref, _ = O.solve_depth_all(emap, tiles, data, 2048, ZR)
    assert int((out.cpu().numpy().view(np.uint16)[0] != ref).sum()) == 0


def test_merge_batch16_staggered_halves(fuser):
    """A batch of 16: every panorama equals the oracle, and the run with the stage timers on
    (events between stages) equals the run without."""
    out_w, ew = CFGS["C1"]
    lay = PL.config_layout("C1")
    fuser.set_tiles(lay)
    tiles, total = O.make_tiles(lay)
    B = 16
    seeds = pf_synth.seeds_for(B, 4242)
    emaps = pf_synth.baseline_emap(seeds, ew, ew // 2).numpy()
    gts = pf_synth.scene_depth(seeds, out_w, out_w // 2).numpy()
    resp = pf_synth.responses(seeds, lay.ntiles)
    datas = np.stack([O.warp_depth(gts[b], tiles, total,
                                   O.responses(resp[b * lay.ntiles:(b + 1) * lay.ntiles]))
                      for b in range(B)])
    out = torch.zeros((B, out_w // 2, out_w), dtype=torch.int16, device=DEV)
    fuser.merge(_dev(emaps), _dev(datas), out, ZR)
    got = out.cpu().numpy().view(np.uint16)
    for b in range(B):
        ref, _ = O.merge(emaps[b], tiles, datas[b].copy(), out_w, ZR)
        assert int((got[b] != ref).sum()) == 0, f"pano {b}"
    fuser.profile(True)
    out2 = torch.zeros_like(out)
    fuser.merge(_dev(emaps), _dev(datas), out2, ZR)
    fuser.profile_read()
    fuser.profile(False)
    assert torch.equal(out, out2)


def test_merge_c2_batch16_profiled_equals_plain(fuser):
    out_w, ew = CFGS["C2"]
    lay = PL.config_layout("C2")
    fuser.set_tiles(lay)
    B = 16
    seeds = pf_synth.seeds_for(B, 99)
    dev = torch.device(DEV)
    gt = pf_synth.scene_depth(seeds, out_w, out_w // 2, dev).contiguous()
    emap = pf_synth.baseline_emap(seeds, ew, ew // 2, dev).contiguous()
    tiles = torch.empty((B, fuser.tile_elems), dtype=torch.float32, device=dev)
    fuser.warp_depth(gt, tiles, panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), dev))
    outs = []
    for prof in (False, True):
        fuser.profile(prof)
        o = torch.zeros((B, out_w // 2, out_w), dtype=torch.int16, device=dev)
        fuser.merge(emap, tiles, o, ZR)
        if prof:
            fuser.profile_read()
        outs.append(o)
    fuser.profile(False)
    assert torch.equal(outs[0], outs[1])


def test_tile_sharded_pipeline_equals_fuse(fuser):
    """C5 decomposition on one GPU: sub-layout warps into slices of the full tile block, then
    pf_dist.fuse_tile_sharded over two simulated ranks (per-rank partials summed, as the RCCL
    reduce would) == the whole-layout warp + fuse, bit for bit."""
    import pf_dist
    out_w, ew = CFGS["C2"]
    lay = PL.config_layout("C2")
    seeds = pf_synth.seeds_for(1, 20261015 + 7)
    gt = pf_synth.scene_depth(seeds, out_w, out_w // 2, DEV).contiguous()
    emap = pf_synth.baseline_emap(seeds, ew, ew // 2, DEV).contiguous()
    resp_all = pf_synth.responses(seeds, lay.ntiles)
    fuser.set_tiles(lay)
    full = torch.zeros((1, fuser.tile_elems), dtype=torch.float32, device=DEV)
    fuser.warp_depth(gt, full, panofuse.make_responses(resp_all, DEV))
    ref = torch.zeros((1, out_w // 2, out_w), dtype=torch.int16, device=DEV)
    fuser.fuse(emap, full, ref, ZR)

    world = 2
    tiles = torch.zeros_like(full)
    off = 0
    for rank in range(world):
        t0, t1 = pf_dist.shard_range(lay.ntiles, rank, world)
        sub = PL.Layout("sub", lay.fovs[t0:t1], lay.ranges[t0:t1], lay.tile_w[t0:t1],
                        lay.tile_h[t0:t1])
        fs = panofuse.Fuser(0)
        fs.set_tiles(sub)
        fs.warp_depth(gt, tiles[:, off:off + fs.tile_elems],
                      panofuse.make_responses(resp_all[t0:t1], DEV))
        off += fs.tile_elems
        fs.close()
    assert torch.equal(tiles.view(torch.int32), full.view(torch.int32))

    out = torch.zeros_like(ref)
    fz = panofuse.Fuser(0)
    fz.set_tiles(lay)
    be = pf_dist.HipTileShardBackend(fz, emap, tiles, None, out_w, ZR, out)

    class SumBackend:
        """Rank 0's view: partial() returns the sum over every simulated rank's shard."""
        def partial(self, level, t0, t1):
            acc = None
            for r in range(world):
                l, n = be.partial(level, *pf_dist.shard_range(lay.ntiles, r, world))
                acc = (l, n) if acc is None else (acc[0] + l, acc[1] + n)
            return acc

        seed, finish = be.seed, be.finish

    nlev = panofuse.level_info(out_w, out_w // 2, ZR, 0)[5]
    pf_dist.fuse_tile_sharded(SumBackend(), nlev, lay.ntiles, 0, 1)
    torch.cuda.synchronize()
    assert int((out != ref).sum().item()) == 0


def test_layout_reuse_and_switch_bit_exact(fuser):
    """pf_set_tiles with the same layout again keeps the per-layout caches; switching layouts
    (C1 -> C2 -> C1, and the same windows with other ranges) rebuilds them.  Every merge stays
    bit-exact against the oracle."""
    def run(cfg, lay=None):
        out_w, ew = CFGS[cfg]
        lay = lay or PL.config_layout(cfg)
        fuser.set_tiles(lay)
        tiles, total = O.make_tiles(lay)
        seeds = pf_synth.seeds_for(1, 4242)
        emap = pf_synth.baseline_emap(seeds, ew, ew // 2).numpy()
        gt = pf_synth.scene_depth(seeds, out_w, out_w // 2).numpy()
        data = O.warp_depth(gt[0], tiles, total, O.responses(pf_synth.responses(seeds, lay.ntiles)))
        out = torch.zeros((1, out_w // 2, out_w), dtype=torch.int16, device=DEV)
        fuser.merge(_dev(emap), _dev(data[None]), out, ZR)
        ref, _ = O.merge(emap[0], tiles, data.copy(), out_w, ZR)
        assert int((out.cpu().numpy().view(np.uint16)[0] != ref).sum()) == 0, cfg

    for cfg in ("C1", "C1", "C2", "C1"):
        run(cfg)
    lay = PL.config_layout("C1")
    shifted = PL.Layout(lay.name, lay.fovs.copy(), lay.ranges.copy(), lay.tile_w, lay.tile_h)
    shifted.ranges[:, 2] += np.float32(0.02)  # same windows, other valid zenith ranges
    run("C1", shifted)
    run("C1")


def test_register_joint_matches_lstsq(fuser):
    """SolveDepthToDepth with several active maps (Depth.cpp:1274-1376): the samples of every
    active tile in one problem.  Against an fp64 lstsq over the concatenated samples (the fitted
    values within 1e-6, the bar of test_register_degree1_and_lstsq); a single active tile equals
    pf_register's per-tile solve bit for bit."""
    lay, emap, gt, tiles, total, data, _ = _inputs("C1")
    fuser.set_tiles(lay)
    fuser.set_solver("normal")
    t_emap, t_data = _dev(emap)[None], _dev(data)[None].contiguous()
    for active in ([0, 2], [1, 3, 4], list(range(lay.ntiles))):
        c64 = torch.zeros((1, 4), dtype=torch.float64, device=DEV)
        fuser.register_joint(t_emap, t_data, ZR, active, coeffs64=c64)
        xs, ys = [], []
        for p in active:
            x, y, _, _ = O.reg_samples(tiles[p], data, emap, ZR)
            xs.append(x)
            ys.append(y)
        xs, ys = np.concatenate(xs), np.concatenate(ys)
        A = np.stack([xs ** k for k in range(3, -1, -1)], 1)
        sol, *_ = np.linalg.lstsq(A, ys, rcond=None)
        assert np.max(np.abs(A @ c64.cpu().numpy()[0] - A @ sol)) < 1e-6, active
    fuser.set_solver("lm")
    per = torch.zeros((1, lay.ntiles, 4), dtype=torch.float32, device=DEV)
    fuser.register(t_emap, t_data, ZR, apply=False, coeffs=per)
    one = torch.zeros((1, 4), dtype=torch.float32, device=DEV)
    fuser.register_joint(t_emap, t_data, ZR, [3], coeffs=one)
    assert torch.equal(one[0], per[0, 3])
