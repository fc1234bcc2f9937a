"""World-size-2 gloo tests (CPU) of the multi-GPU decompositions in pf_dist.py.

The per-rank compute here is the CPU oracle (no GPU in this container); on the GPU box the same
driver runs with the HIP backend over RCCL (bench.py --mode c5)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
import torch.distributed as dist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import pf_dist  # noqa: E402


def test_shard_range_partitions():
    for n in (1, 5, 20, 80, 81):
        for world in (1, 2, 3, 8):
            seen = []
            for r in range(world):
                lo, hi = pf_dist.shard_range(n, r, world)
                seen.extend(range(lo, hi))
            assert seen == list(range(n))


def test_panorama_blocks_disjoint():
    a = pf_dist.panorama_block(64, 0)
    b = pf_dist.panorama_block(64, 1)
    assert len(set(a) | set(b)) == 128


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class OracleBackend:
    """CPU stand-in for the GPU backend: the oracle computes each rank's share."""

    def __init__(self, O, PL, out_w, emap, tiles, data):
        self.O, self.PL, self.out_w = O, PL, out_w
        self.emap, self.tiles, self.data = emap, tiles, data
        self.zr = PL.ZENITH_RANGE

    def _lv(self, level):
        return self.O.level_dims(self.out_w, self.out_w // 2, self.zr, level)

    def partial(self, level, t0, t1):
        lv = self._lv(level)
        if t1 > t0:
            Ls, n = self.O.targets_subset(self.tiles, t0, t1, self.data, lv)
        else:
            Ls = np.zeros((lv.h, lv.w), np.float32)
            n = np.zeros((lv.h, lv.w), np.int32)
        return torch.from_numpy(Ls.copy()), torch.from_numpy(n.astype(np.float32))

    def multicover_count(self, level):
        # the C1 layout covers every pixel at most twice (tests/test_oracle.py); the GPU backend
        # handles 3+ (tests/test_gpu_rowshard.py at the C5 layout)
        return 0

    def seed(self, level, prev):
        lv = self._lv(level)
        if level == 0:
            return self.O.seed_level0(self.emap, lv)
        return self.O.upsample(prev, lv)

    def finish(self, level, lsum, cnt, buf, last):
        lv = self._lv(level)
        Ln = self.O.normalize(lsum.numpy(), cnt.numpy().astype(np.int32), lv)
        return self.O.jacobi(buf, Ln, lv, lv.iters)


def _worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pf_layouts as PL
        import pf_synth
        import pyoracle as O
        lay = PL.config_layout("C1")
        tiles, total = O.make_tiles(lay)
        seeds = pf_synth.seeds_for(1, 31337)
        emap = pf_synth.baseline_emap(seeds, 128, 64)[0].numpy()
        data = np.random.RandomState(2).rand(total).astype(np.float32)
        be = OracleBackend(O, PL, 512, emap, tiles, data)
        final = pf_dist.fuse_tile_sharded(be, 3, lay.ntiles, rank, world, pf_dist.TorchComm(dist))
        # every rank also checks the reduced level-2 targets against the single-rank sums
        lv = be._lv(2)
        ls, n = be.partial(2, *pf_dist.shard_range(lay.ntiles, rank, world))
        dist.all_reduce(ls)
        dist.all_reduce(n)
        full_l, full_n = O.targets_subset(tiles, 0, lay.ntiles, data, lv)
        ok_targets = bool(np.array_equal(ls.numpy().view(np.uint32), full_l.view(np.uint32))
                          and np.array_equal(n.numpy(), full_n.astype(np.float32)))
        if rank == 0:
            ref, _ = O.solve_depth_all(emap, tiles, data, 512, PL.ZENITH_RANGE)
            got = O.quantize(final)
            q.put(("final", bool(np.array_equal(got, ref))))
        q.put(("targets", ok_targets))
        # batch sharding: the timing reduction is a MAX over ranks
        t = torch.tensor([1.0 + rank], dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        q.put(("max", float(t.item())))
    finally:
        dist.destroy_process_group()


def test_tile_sharded_fusion_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0
    res = []
    while not q.empty():
        res.append(q.get())
    assert ("final", True) in res
    assert res.count(("targets", True)) == 2
    assert res.count(("max", 2.0)) == 2


class OracleRowBackend(OracleBackend):
    """CPU stand-in of pf_dist.HipRowShardBackend: each rank holds full-level planes (torch CPU
    tensors) but only its band rows stay current; a band pass of depth T is T oracle sweeps of
    the whole plane, of which only rows [row0, row1) are kept (they depend on rows row0-T-1 ..
    row1+T only, the halo the orchestration refreshed)."""

    def __init__(self, *args):
        super().__init__(*args)
        lv = self._lv(2)
        self.out = torch.zeros(lv.w * lv.h, dtype=torch.int16)

    def dims(self, level):
        lv = self._lv(level)
        return lv.w, lv.h, lv.h0, lv.h1

    def plane(self, level):
        lv = self._lv(level)
        return torch.zeros(lv.w * lv.h, dtype=torch.float32)

    def scratch(self, n):
        return torch.zeros(n, dtype=torch.float32)

    def seed(self, level, prev):  # a replicated level (flat torch planes, as the GPU backend)
        lv = self._lv(level)
        if level == 0:
            base = self.O.seed_level0(self.emap, lv)
        else:
            plv = self._lv(level - 1)
            base = self.O.upsample(prev.numpy().reshape(plv.h, plv.w), lv)
        return torch.from_numpy(np.ascontiguousarray(base).ravel().copy())

    def finish(self, level, lsum, cnt, buf, last):
        lv = self._lv(level)
        Ln = self.O.normalize(lsum.numpy().reshape(lv.h, lv.w),
                              cnt.numpy().astype(np.int32).reshape(lv.h, lv.w), lv)
        res = self.O.jacobi(buf.numpy().reshape(lv.h, lv.w), Ln, lv, lv.iters)
        if last:
            self.out.copy_(torch.from_numpy(self.O.quantize(res).view(np.int16).ravel()))
        return torch.from_numpy(np.ascontiguousarray(res).ravel().copy())

    def level(self, level, prev, lsum, cnt, last):  # pf_fuse_level's contract
        buf = self.seed(level, prev)
        if cnt is None:  # lsum holds the normalised targets (pf_fuse_targets)
            lv = self._lv(level)
            res = self.O.jacobi(buf.numpy().reshape(lv.h, lv.w), lsum.numpy().reshape(lv.h, lv.w),
                                lv, lv.iters)
            if last:
                self.out.copy_(torch.from_numpy(self.O.quantize(res).view(np.int16).ravel()))
                return None
            return torch.from_numpy(np.ascontiguousarray(res).ravel().copy())
        res = self.finish(level, lsum, cnt, buf, last)
        return None if last else res

    def targets(self, level):  # pf_fuse_targets: every tile, normalised
        lv = self._lv(level)
        Ls, n = self._subset(level, 0, len(self.tiles))
        Ln = self.O.normalize(Ls.reshape(lv.h, lv.w), n.reshape(lv.h, lv.w).astype(np.int32), lv)
        return torch.from_numpy(np.ascontiguousarray(Ln, dtype=np.float32).ravel().copy())

    def _subset(self, level, t0, t1):
        key = (level, t0, t1)
        if not hasattr(self, "_sub"):
            self._sub = {}
        if key not in self._sub:
            lv = self._lv(level)
            if t1 > t0:
                Ls, n = self.O.targets_subset(self.tiles, t0, t1, self.data, lv)
            else:
                Ls, n = np.zeros((lv.h, lv.w), np.float32), np.zeros((lv.h, lv.w), np.int32)
            self._sub[key] = (np.ascontiguousarray(Ls).ravel(), np.ascontiguousarray(n).ravel())
        return self._sub[key]

    def _rows(self, level, row0, row1):
        lv = self._lv(level)
        a, b = max(row0, lv.h0), min(row1, lv.h1 + 1)
        return slice(a * lv.w, max(a, b) * lv.w)

    def tile_rows(self, level, t0, t1):
        lv = self._lv(level)
        rows = np.nonzero(self._subset(level, t0, t1)[1].reshape(lv.h, lv.w).any(1))[0]
        return (int(rows[0]), int(rows[-1])) if rows.size else (0, -1)

    def partial_rows(self, level, t0, t1, row0, row1, lsum, cnt):
        Ls, n = self._subset(level, t0, t1)
        sl = self._rows(level, row0, row1)
        lsum[sl] = torch.from_numpy(Ls[sl].copy())
        cnt[sl] = torch.from_numpy(n[sl].astype(np.float32))

    def coverage_plane(self, level):
        _, n = self._subset(level, 0, len(self.tiles))
        return torch.from_numpy(n.astype(np.float32))

    def rows_add(self, dst, src):
        dst += src

    def normalize_rows(self, level, lsum, cnt, row0, row1, lnorm):
        lv = self._lv(level)
        Ln = np.ascontiguousarray(self.O.normalize(lsum.numpy().reshape(lv.h, lv.w),
                                                   cnt.numpy().astype(np.int32).reshape(lv.h, lv.w),
                                                   lv)).ravel()
        sl = self._rows(level, row0, row1)
        lnorm[sl] = torch.from_numpy(Ln[sl].copy())

    def plan(self, level, nbands):
        it = self._lv(level).iters
        return [10] * (it // 10) + ([it % 10] if it % 10 else [])

    def _base(self, level, prev):
        lv = self._lv(level)
        if level == 0:
            return self.O.seed_level0(self.emap, lv)
        plv = self._lv(level - 1)
        return self.O.upsample(prev.numpy().reshape(plv.h, plv.w), lv)

    def border(self, level, prev, a, b):
        base = torch.from_numpy(np.ascontiguousarray(self._base(level, prev)).ravel().copy())
        if level == 2:
            self.out.copy_(torch.from_numpy(self.O.quantize(base.numpy()).view(np.int16)))
        else:
            a.copy_(base)
            b.copy_(base)

    def band_pass(self, level, lnorm, src_mode, src, dst, T, row0, row1, last, prev):
        lv = self._lv(level)
        base = src.numpy().reshape(lv.h, lv.w) if src_mode == 0 else self._base(level, prev)
        res = self.O.jacobi(base, lnorm.numpy().reshape(lv.h, lv.w), lv, T).ravel()
        sl = slice(row0 * lv.w, row1 * lv.w)
        if last:
            self.out[sl] = torch.from_numpy(self.O.quantize(res[sl]).view(np.int16))
        else:
            dst[sl] = torch.from_numpy(res[sl].copy())


def _row_worker(rank, world, port, q, rep=0):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import pf_layouts as PL
        import pf_synth
        import pyoracle as O
        lay = PL.config_layout("C1")
        tiles, total = O.make_tiles(lay)
        seeds = pf_synth.seeds_for(1, 4711)
        emap = pf_synth.baseline_emap(seeds, 128, 64)[0].numpy()
        data = np.random.RandomState(9).rand(total).astype(np.float32)
        be = OracleRowBackend(O, PL, 512, emap, tiles, data)
        log = pf_dist.ExchangeLog()
        pf_dist.fuse_row_sharded(be, 3, lay.ntiles, rank, world, pf_dist.TorchComm(dist), log,
                                 rep_levels=rep)
        # the bytes this rank sent are those of the exchange model
        dims = [be.dims(lv) for lv in range(3)]
        plans = [be.plan(lv, 1 if lv < rep else world) for lv in range(3)]
        ext = [[be.tile_rows(lv, *pf_dist.shard_range(lay.ntiles, r, world))
                for r in range(world)] for lv in range(3)]
        model = pf_dist.exchange_model(dims, plans, ext, world, rep_levels=rep)[rank]
        same = all(model.get(k, 0) == v for k, v in log.sent.items()) and \
            all(log.sent.get(k, 0) == v for k, v in model.items())
        ok = True
        if rank == 0:  # the u16 result is gathered to rank 0 only
            ref, _ = O.solve_depth_all(emap, tiles, data, 512, PL.ZENITH_RANGE)
            ok = bool(np.array_equal(be.out.numpy().view(np.uint16).reshape(256, 512), ref))
        q.put((rank, ok and same, log.sent, model))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,rep", [(1, 0), (2, 0), (3, 1), (2, 3)])
def test_row_sharded_fusion_gloo(world, rep):
    """tiles and rows sharded, halo rows exchanged between passes; rank 0 ends
    with the u16 panorama of the unsharded oracle fusion, bit for bit.  rep = the coarse levels
    replicated on every rank instead (an all-gather of the partial target rows, no pass halos):
    none, the first, all three.  World 1: every level from pf_fuse_targets + pf_fuse_level."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_row_worker, args=(r, world, port, q, rep))
             for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(240)
        assert p.exitcode == 0
    res = sorted((q.get() for _ in range(world)), key=lambda x: x[0])
    assert [(r, ok) for r, ok, _, _ in res] == [(r, True) for r in range(world)], res
    # world 2 deals the C1 layout band by band (tiles 0-2 = the upper zenith band), so only
    # halo-sized rows travel: per rank the target rows it sends are at most its neighbour's halo
    # plus the shared boundary row (K + 1 rows of <= 512 floats, 3 levels; K = halo_rows(plan):
    # 11 for passes of 10 with one exchange each, more with grouped passes), far below a plane.
    # (World 3 deals 2 tiles per rank across the bands: the bands fall back to an even split and
    # more rows travel -- still exactly the model's bytes.)
    if world == 2 and rep == 0:
        K = pf_dist.halo_rows([10] * 5, max(pf_dist.PASS_GROUP, 2))
        for _, _, sent, _ in res:
            assert 0 < sent.get("targets", 0) <= 3 * (K + 1) * 512 * 4, sent


def test_pass_groups_pair_the_exchanges():
    """Grouped passes (round 6): one exchange per run of G passes after the first, sum(T + 1)
    rows, each pass of a run computing the rows past the band the rest of its run reads; G = 1:
    T + 1 before every pass but the first."""
    plan = [10, 10, 10, 8, 8, 5]
    assert pf_dist.pass_groups(plan, 1) == [(0, 0), (11, 0), (11, 0), (9, 0), (9, 0), (6, 0)]
    assert pf_dist.pass_groups(plan, 2) == [(0, 0), (22, 11), (0, 0), (18, 9), (0, 0), (6, 0)]
    assert pf_dist.pass_groups(plan, 3) == [(0, 0), (31, 20), (0, 9), (0, 0), (15, 6), (0, 0)]
    assert pf_dist.halo_rows(plan, 2) == 22 and pf_dist.halo_rows(plan, 1) == 11
    assert pf_dist.pass_groups([10], 4) == [(0, 0)]
    # the group a level gets: the largest whose halo every band supplies
    g, K, b = pf_dist.level_geometry(0, 99, 4, None, [10] * 9, gmax=4)
    assert (g, K) == (2, 22) and min(b[r + 1] - b[r] for r in range(4)) >= K
    g, K, _ = pf_dist.level_geometry(0, 999, 4, None, [10] * 9, gmax=4)
    assert (g, K) == (4, 44)


@pytest.mark.parametrize("world", [2, 3])
def test_row_sharded_fusion_gloo_one_exchange_per_pass(world, monkeypatch):
    """The one-exchange-per-pass flow (PF_C5_GROUP=1, pf_dist.PASS_GROUP) stays bit-exact with its
    own byte model."""
    monkeypatch.setenv("PF_C5_GROUP", "1")  # the spawned workers import pf_dist afresh
    test_row_sharded_fusion_gloo(world, 0)
