"""GPU parity at the BASELINE configurations beyond C1/C2 ("test the configs that have
never run").

* the 4-level path (out_w >= 4096: max_level 4, 200/150/100/50 sweeps, Depth.cpp:1423-1424,
  1665-1675) at 4096 and at the C5 layout (8192x4096, 80 tiles of 1024^2, 10x8), bit-exact against
  the oracle run live on the same inputs AND against the committed checksums of
  tests/golden/large_merge.npz (tools/make_golden_large.py: SHA-256 + strided subsample, SURVEY.md
  8c G3);
* the C5 tile-sharded pipeline (pf_dist.fuse_tile_sharded, 4 levels) on one GPU == pf_fuse;
* C3 (batch 64 of C2) end to end on the GPU (warp -> register -> fuse): every panorama equals its
  own batch-1 run, and sampled panoramas equal the oracle on the same tiles.
"""
import hashlib
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import panofuse  # noqa: E402
import pf_layouts as PL  # noqa: E402
import pf_synth  # noqa: E402
import pyoracle as O  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ZR = PL.ZENITH_RANGE
DEV = "cuda:0"
GOLDEN = os.path.join(ROOT, "tests", "golden", "large_merge.npz")


@pytest.fixture(scope="module")
def fuser():
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a host without a GPU")
    O.set_threads(min(16, os.cpu_count() or 1))
    return panofuse.Fuser(0)


def _dev(a):
    return torch.from_numpy(np.ascontiguousarray(a)).to(DEV)


def _sha(a):
    return np.frombuffer(hashlib.sha256(np.ascontiguousarray(a).tobytes()).digest(), np.uint8)


def _large_inputs(name):
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import make_golden_large as G
    return G.case_inputs(name)


@pytest.mark.parametrize("name", ["W4096", "C5"])
def test_merge_4level_bit_exact(fuser, name):
    """MergeDepthMaps core (registration + 4-level fusion) at out_w 4096 / 8192."""
    gold = np.load(GOLDEN)
    lay, tiles, emap, data, out_w = _large_inputs(name)
    assert O.num_levels(out_w) == 4
    assert np.array_equal(_sha(np.concatenate([emap.ravel(), data.ravel()])),
                          gold[f"{name}_in_sha256"]), "synthetic inputs drifted"
    fuser.set_tiles(lay)
    out = torch.zeros((1, out_w // 2, out_w), dtype=torch.int16, device=DEV)
    coeffs = torch.zeros((1, lay.ntiles, 4), dtype=torch.float32, device=DEV)
    fuser.merge(_dev(emap)[None], _dev(data)[None], out, ZR, coeffs=coeffs)
    got = out.cpu().numpy().view(np.uint16)[0]
    # the committed checksums (oracle output generated in the build container)
    assert np.array_equal(coeffs.cpu().numpy()[0], gold[f"{name}_abcd"])
    sub = got.ravel()[::int(gold["stride"])]
    assert int((sub != gold[f"{name}_out_sub"]).sum()) == 0, "strided subsample differs"
    assert np.array_equal(_sha(got), gold[f"{name}_out_sha256"]), "SHA-256 of the u16 output"
    # and the oracle run live on this host
    ref, abcd = O.merge(emap, tiles, data.copy(), out_w, ZR)
    assert np.array_equal(coeffs.cpu().numpy()[0], abcd)
    assert int((got != ref).sum()) == 0


def test_fuse_4level_level_internals(fuser):
    """Every level's seed, (sum L, n) targets and post-Jacobi buffer at 4096 (4 levels)."""
    lay = PL.band_layout(5, 4, 1024, 1024, 3, 12, "C2@4096")
    out_w = 4096
    tiles, total = O.make_tiles(lay)
    rs = np.random.RandomState(17)
    data = rs.rand(total).astype(np.float32)
    emap = rs.rand(512, 1024).astype(np.float32)
    fuser.set_tiles(lay)
    t_tiles, t_emap = _dev(data), _dev(emap)[None]
    prev_gpu = prev_ref = None
    for level in range(4):
        lv = O.level_dims(out_w, out_w // 2, ZR, level)
        assert lv.iters == (200, 150, 100, 50)[level]
        buf = torch.zeros(lv.h * lv.w, dtype=torch.float32, device=DEV)
        fuser.fuse_seed(t_emap if level == 0 else None, prev_gpu, out_w, ZR, level, buf)
        ref_seed = O.seed_level0(emap, lv) if level == 0 else O.upsample(prev_ref, lv)
        assert np.array_equal(buf.cpu().numpy().reshape(lv.h, lv.w), ref_seed), f"seed L{level}"
        lsum = torch.zeros(lv.h * lv.w, dtype=torch.float32, device=DEV)
        cnt = torch.zeros_like(lsum)
        fuser.fuse_partial(t_tiles, None, 0, lay.ntiles, out_w, ZR, level, lsum, cnt)
        rL, rn, oops, _ = O.targets(tiles, data, lv)
        band = slice(lv.h0, lv.h1 + 1)
        assert np.array_equal(cnt.cpu().numpy().reshape(lv.h, lv.w)[band],
                              rn[band].astype(np.float32)), f"coverage L{level}"
        g_l = lsum.cpu().numpy().reshape(lv.h, lv.w)[band]
        assert np.array_equal(g_l.view(np.uint32), rL[band].view(np.uint32)), f"targets L{level}"
        fuser.fuse_finish_level(lsum, cnt, out_w, ZR, level, buf)
        ref_buf = O.jacobi(ref_seed, O.normalize(rL, rn, lv), lv, lv.iters)
        got = buf.cpu().numpy().reshape(lv.h, lv.w)
        bad = int((got.view(np.uint32) != ref_buf.view(np.uint32)).sum())
        assert bad == 0, f"level {level}: {bad} Jacobi values differ"
        prev_gpu, prev_ref = buf, ref_buf


def test_c5_tile_sharded_pipeline_equals_fuse(fuser):
    """C5 (8192x4096, 80 tiles, 4 levels): per-rank tile shards warped into slices of the tile
    block, (sum L, n) partials summed over 8 simulated ranks (as the RCCL reduce does), rank 0
    sweeps -- bit-identical to the one-context warp + fuse."""
    import pf_dist
    lay = PL.config_layout("C5")
    out_w, ew = PL.CONFIGS["C5"]
    seeds = pf_synth.seeds_for(1, 20261015 + 3)
    gt = pf_synth.scene_depth(seeds, out_w, out_w // 2, DEV).contiguous()
    emap = pf_synth.baseline_emap(seeds, ew, ew // 2, DEV).contiguous()
    resp_all = pf_synth.responses(seeds, lay.ntiles)
    fuser.set_tiles(lay)
    full = torch.zeros((1, fuser.tile_elems), dtype=torch.float32, device=DEV)
    fuser.warp_depth(gt, full, panofuse.make_responses(resp_all, DEV))
    coeffs = torch.zeros((1, lay.ntiles, 4), dtype=torch.float32, device=DEV)
    fuser.register(emap, full, ZR, apply=False, coeffs=coeffs)
    ref = torch.zeros((1, out_w // 2, out_w), dtype=torch.int16, device=DEV)
    fuser.fuse(emap, full, ref, ZR, coeffs=coeffs)

    world = 8
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
    be = pf_dist.HipTileShardBackend(fz, emap, tiles, coeffs[0], out_w, ZR, out)

    class SumBackend:
        """Rank 0's view of the 8-rank reduce: partials summed over the simulated ranks, then the
        pixels covered by 3+ tiles (7 per level at this layout) re-added in tile order from the
        per-rank contributions, as fuse_tile_sharded does at world > 1."""
        def partial(self, level, t0, t1):
            acc = None
            contrib = None
            for r in range(world):
                q0, q1 = pf_dist.shard_range(lay.ntiles, r, world)
                l, n = be.partial(level, q0, q1)
                acc = (l, n) if acc is None else (acc[0] + l, acc[1] + n)
                c = be.multicover(level, q0, q1)
                contrib = c if contrib is None else contrib + c
            assert be.multicover_count(level) == 4 * 7  # 7 pixels x 4 tiles (tests/test_oracle.py)
            be.multicover_patch(level, contrib, acc[0])
            return acc

        seed, finish = be.seed, be.finish

    nlev = panofuse.level_info(out_w, out_w // 2, ZR, 0)[5]
    assert nlev == 4
    pf_dist.fuse_tile_sharded(SumBackend(), nlev, lay.ntiles, 0, 1)
    torch.cuda.synchronize()
    assert int((out != ref).sum().item()) == 0


def test_c3_batch64_end_to_end(fuser):
    """C3: 64 panoramas of C2 through warp -> register -> fuse in one call chain (the bench
    step).  Every panorama equals its own batch-1 run on the same tiles; panoramas 0, 21, 42
    and 63 equal the oracle's MergeDepthMaps on those tiles."""
    out_w, ew = 2048, 512
    lay = PL.config_layout("C2")
    B = 64
    seeds = pf_synth.seeds_for(B, 20261015)
    dev = torch.device(DEV)
    gt = pf_synth.scene_depth(seeds, out_w, out_w // 2, dev).contiguous()
    emap = pf_synth.baseline_emap(seeds, ew, ew // 2, dev).contiguous()
    fuser.set_tiles(lay)
    tiles = torch.empty((B, fuser.tile_elems), dtype=torch.float32, device=dev)
    fuser.warp_depth(gt, tiles, panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), dev))
    out = torch.zeros((B, out_w // 2, out_w), dtype=torch.int16, device=dev)
    coeffs = torch.zeros((B, lay.ntiles, 4), dtype=torch.float32, device=dev)
    fuser.merge(emap, tiles, out, ZR, coeffs=coeffs)
    one = torch.zeros((1, out_w // 2, out_w), dtype=torch.int16, device=dev)
    c1 = torch.zeros((1, lay.ntiles, 4), dtype=torch.float32, device=dev)
    for b in range(B):
        fuser.merge(emap[b:b + 1], tiles[b:b + 1], one, ZR, coeffs=c1)
        assert torch.equal(c1[0], coeffs[b]), f"pano {b}: coefficients differ from batch-1"
        assert torch.equal(one[0], out[b]), f"pano {b}: batch-64 != batch-1"
    otiles, _ = O.make_tiles(lay)
    got = out.cpu().numpy().view(np.uint16)
    for b in (0, 21, 42, 63):
        ref, abcd = O.merge(emap[b].cpu().numpy(), otiles, tiles[b].cpu().numpy().copy(), out_w,
                            ZR)
        assert np.array_equal(coeffs[b].cpu().numpy(), abcd), f"pano {b} abcd"
        assert int((got[b] != ref).sum()) == 0, f"pano {b}"
