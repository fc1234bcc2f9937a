"""Row-band sharded fusion on the GPU: pf_dist.fuse_row_sharded over the HIP band
entry points (pf_fuse_band_plan / pf_fuse_band_pass / pf_fuse_border / pf_fuse_normalize).

The ranks are simulated on one GPU: one thread and one panofuse context per rank, all on the
same stream, with an in-process communicator standing in for RCCL (all-reduce, halo exchange,
band broadcast).  The result of every rank must equal the one-GPU pf_fuse bit for bit, at C2
(3 levels, 2 and 3 bands) and at the C5 layout (8192x4096, 4 levels, 4 bands, tiles sharded
too, including the pixels covered by four tiles), and likewise the tiles-only flow
(fuse_tile_sharded, 8 ranks).  Rank 0 holds the gathered u16 result.  The collectives
themselves are covered over gloo in tests/test_dist.py.
"""
import threading

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import panofuse  # noqa: E402
import pf_dist  # noqa: E402
import pf_layouts as PL  # noqa: E402
import pf_synth  # noqa: E402

ZR = PL.ZENITH_RANGE
DEV = "cuda:0"


class ThreadComm:
    """In-process stand-in for pf_dist.TorchComm among `world` threads."""

    def __init__(self, world):
        self.world = world
        self.bar = threading.Barrier(world, timeout=120)
        self.box = {}

    def rank(self, r):
        outer = self

        class RankComm:
            def all_reduce_sum(self, t):
                outer.box[("ar", r)] = t
                torch.cuda.current_stream().synchronize()
                outer.bar.wait()
                if r == 0:
                    acc = outer.box[("ar", 0)].clone()
                    for k in range(1, outer.world):
                        acc += outer.box[("ar", k)]
                    outer.box["ar"] = acc
                torch.cuda.current_stream().synchronize()
                outer.bar.wait()
                t.copy_(outer.box["ar"])
                torch.cuda.current_stream().synchronize()
                outer.bar.wait()

            def reduce_sum(self, t, dst):
                self.all_reduce_sum(t)

            def exchange(self, sends, recvs):
                # several messages per pair arrive in the order they were sent (as batched
                # isend/irecv pairs match); the clones are complete before another thread's
                # stream reads them (a rank may exchange on its side stream)
                for peer, t in sends:
                    outer.box.setdefault(("x", r, peer), []).append(t.clone())
                torch.cuda.current_stream().synchronize()
                outer.bar.wait()
                for peer, t in recvs:
                    t.copy_(outer.box[("x", peer, r)].pop(0))
                outer.bar.wait()

            def broadcast(self, t, src):
                if r == src:
                    outer.box["bc"] = t.clone()
                torch.cuda.current_stream().synchronize()
                outer.bar.wait()
                if r != src:
                    t.copy_(outer.box["bc"])
                outer.bar.wait()

        return RankComm()


def _run(cfg, world, seed, flow="rows", rep=0, side=False):
    lay = PL.config_layout(cfg)
    out_w, ew = PL.CONFIGS["C5" if cfg == "C5" else "C2"]
    seeds = pf_synth.seeds_for(1, seed)
    gt = pf_synth.scene_depth(seeds, out_w, out_w // 2, DEV).contiguous()
    emap = pf_synth.baseline_emap(seeds, ew, ew // 2, DEV).contiguous()
    fz = panofuse.Fuser(0)
    fz.set_tiles(lay)
    tiles = torch.zeros((1, fz.tile_elems), dtype=torch.float32, device=DEV)
    fz.warp_depth(gt, tiles, panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), DEV))
    coeffs = torch.zeros((1, lay.ntiles, 4), dtype=torch.float32, device=DEV)
    fz.register(emap, tiles, ZR, apply=False, coeffs=coeffs)
    ref = torch.zeros((1, out_w // 2, out_w), dtype=torch.int16, device=DEV)
    fz.fuse(emap, tiles, ref, ZR, coeffs=coeffs)
    torch.cuda.synchronize()

    comm = ThreadComm(world)
    outs, errs = [None] * world, []

    def rank_main(r):
        try:
            f = panofuse.Fuser(0)
            f.set_tiles(lay)
            out = torch.zeros(out_w * (out_w // 2), dtype=torch.int16, device=DEV)
            if flow == "rows":
                be = pf_dist.HipRowShardBackend(f, emap, tiles, coeffs[0], out_w, ZR, out)
                if side:  # the row-sharded levels' tile sums on a second stream
                    fs = panofuse.Fuser(0, stream=torch.cuda.Stream(DEV))
                    fs.set_tiles(lay)
                    be.enable_side(fs)
                pf_dist.fuse_row_sharded(be, be.nlevels, lay.ntiles, r, world, comm.rank(r),
                                         rep_levels=rep)
            else:  # tiles only: rank 0 sweeps
                be = pf_dist.HipTileShardBackend(f, emap, tiles, coeffs[0], out_w, ZR,
                                                 out.view(out_w // 2, out_w))
                nlev = panofuse.level_info(out_w, out_w // 2, ZR, 0)[5]
                pf_dist.fuse_tile_sharded(be, nlev, lay.ntiles, r, world, comm.rank(r))
            torch.cuda.synchronize()
            outs[r] = out
            f.close()
        except BaseException as e:  # surfaced by the main thread
            errs.append(e)
            comm.bar.abort()

    th = [threading.Thread(target=rank_main, args=(r,)) for r in range(world)]
    for t in th:
        t.start()
    for t in th:
        t.join(300)
    assert not errs, errs
    for r in range(1):  # the u16 result is gathered to rank 0 (both flows)
        diff = (outs[r].view(out_w // 2, out_w) != ref[0]).sum(1)
        rows = torch.nonzero(diff).flatten().tolist()
        assert not rows, (f"rank {r}: {int(diff.sum())} pixels differ from the one-GPU fusion in "
                          f"rows {rows[:20]} (bands {[pf_dist.band_rows(*panofuse.level_info(out_w, out_w // 2, ZR, 0)[2:4], q, world) for q in range(world)]})")


@pytest.mark.parametrize("world", [2, 3])
def test_row_sharded_c2_equals_fuse(world):
    _run("C2", world, 20261015 + 11)


def test_row_sharded_c5_equals_fuse():
    _run("C5", 4, 20261015 + 12)


def test_row_sharded_c5_eight_ranks_coarse_levels_replicated():
    """C5's 8-rank shape with the 1024- and 2048-wide levels replicated on every rank (the
    all-gather of partial target rows) and the two finer levels row-sharded: rank 0's u16 ==
    the one-GPU fusion (8 threads on one GPU)."""
    _run("C5", 8, 20261015 + 14, rep=2)


def test_row_sharded_c5_eight_ranks_side_stream():
    """The same with each rank's row-sharded levels' tile sums, their exchange and adds on a
    second stream beside the replicated levels' sweeps (HipRowShardBackend.enable_side, the
    bench's C5 flow), and rank 0's own border rows standing in for the last rank's rows below
    the band (pf_dist.border_local_from)."""
    _run("C5", 8, 20261015 + 17, rep=2, side=True)


def test_tile_sharded_c5_threads_equals_fuse():
    """fuse_tile_sharded at world 8 (reduce to rank 0, the 7 pixels per level covered by four
    tiles re-added in tile order): rank 0's u16 == the one-GPU fusion."""
    _run("C5", 8, 20261015 + 13, flow="tiles")


@pytest.mark.parametrize("cfg", ["C2", "C5"])
def test_row_sharded_world1_equals_fuse(cfg):
    """World 1: every level through pf_fuse_targets + pf_fuse_level (no partial sums, the seed
    inside the first pass) equals the one-GPU pf_fuse bit for bit."""
    _run(cfg, 1, 20261015 + 15)


def test_fuse_level_forms_agree():
    """The three ways to one level at C2, plane by plane and bit for bit: pf_fuse_seed +
    pf_fuse_finish_level, pf_fuse_level on (lsum, cnt), and pf_fuse_level on pf_fuse_targets'
    normalised plane; and pf_fuse_targets == pf_fuse_normalize_rows of the all-tile partial
    sums (pf_fuse_partial_rows), sNaN markers included."""
    lay = PL.config_layout("C2")
    out_w, ew = PL.CONFIGS["C2"]
    seeds = pf_synth.seeds_for(1, 20261015 + 16)
    gt = pf_synth.scene_depth(seeds, out_w, out_w // 2, DEV).contiguous()
    emap = pf_synth.baseline_emap(seeds, ew, ew // 2, DEV).contiguous()
    fz = panofuse.Fuser(0)
    fz.set_tiles(lay)
    tiles = torch.zeros((1, fz.tile_elems), dtype=torch.float32, device=DEV)
    fz.warp_depth(gt, tiles, panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), DEV))
    coeffs = torch.zeros((1, lay.ntiles, 4), dtype=torch.float32, device=DEV)
    fz.register(emap, tiles, ZR, apply=False, coeffs=coeffs)
    nlev = panofuse.level_info(out_w, out_w // 2, ZR, 0)[5]
    prev = {k: None for k in ("a", "b", "c")}
    outs = {k: torch.zeros(out_w * (out_w // 2), dtype=torch.int16, device=DEV)
            for k in ("a", "b", "c")}
    for lv in range(nlev):
        w, h, h0, h1 = panofuse.level_info(out_w, out_w // 2, ZR, lv)[:4]
        last = lv == nlev - 1
        lsum = torch.zeros(h * w, dtype=torch.float32, device=DEV)
        cnt = torch.zeros_like(lsum)
        lnorm = torch.zeros_like(lsum)
        tgt = torch.zeros_like(lsum)
        fz.fuse_partial_rows(tiles, coeffs[0], 0, lay.ntiles, out_w, ZR, lv, h0, h1 + 1, lsum, cnt)
        fz.fuse_normalize_rows(lsum, cnt, out_w, ZR, lv, h0, h1 + 1, lnorm)
        fz.fuse_targets(tiles, coeffs[0], out_w, ZR, lv, tgt)
        band = slice(h0 * w, (h1 + 1) * w)
        assert torch.equal(lnorm[band].view(torch.int32), tgt[band].view(torch.int32)), lv
        bufs = {k: torch.zeros(h * w, dtype=torch.float32, device=DEV) for k in ("a", "b", "c")}
        e = emap if lv == 0 else None
        fz.fuse_seed(e, prev["a"], out_w, ZR, lv, bufs["a"])
        fz.fuse_finish_level(lsum, cnt, out_w, ZR, lv, bufs["a"],
                             outs["a"].view(h, w) if last else None)
        fz.fuse_level(e, prev["b"], lsum, cnt, out_w, ZR, lv, bufs["b"],
                      outs["b"].view(h, w) if last else None)
        fz.fuse_level(e, prev["c"], tgt, None, out_w, ZR, lv, bufs["c"],
                      outs["c"].view(h, w) if last else None)
        torch.cuda.synchronize()
        if not last:
            assert torch.equal(bufs["a"], bufs["b"]) and torch.equal(bufs["a"], bufs["c"]), lv
        prev = bufs
    assert torch.equal(outs["a"], outs["b"]) and torch.equal(outs["a"], outs["c"])
    ref = torch.zeros((1, out_w // 2, out_w), dtype=torch.int16, device=DEV)
    fz.fuse(emap, tiles, ref, ZR, coeffs=coeffs)
    torch.cuda.synchronize()
    assert torch.equal(outs["a"].view(out_w // 2, out_w), ref[0])
    fz.close()
