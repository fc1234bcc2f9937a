"""Multi-GPU decomposition of the fusion path.

* Batch sharding (configs C3/C4): panoramas are independent, so rank r simply processes its own
  contiguous block of panoramas; no collective touches the data path (`panorama_block`).
* Tile sharding of one huge panorama (config C5): per fusion level every rank scatters the
  Laplacian targets of its contiguous share of the tiles into full-level (sum L, n) grids, the
  grids are summed over ranks (RCCL reduce over xGMI; gloo in the CPU tests), and rank 0
  normalises and runs the damped Jacobi sweeps (`fuse_tile_sharded`).  The reference adds the
  covering tiles' Laplacians to a pixel one at a time (Depth.cpp:1609-1617); a sum of per-rank
  partials is that same value for pixels covered by at most two tiles (adding zeros is exact,
  a + b commutes), not always for the few covered by three or more (sector corners on shared
  band rows: 7 pixels per level in the C5 layout).  Those pixels are recomputed exactly: every
  rank contributes its tiles' terms of their (pixel, tile) pairs, the terms are summed over
  ranks (one non-zero per pair: exact), and the pixels are re-added in tile order
  (`_exact_multicover`, pf_fuse_multicover).  The result is bit-identical to one GPU's.
* Row-band sharding of the sweeps as well (`fuse_row_sharded`, below).

The reference has no distributed code; this replaces its single-process OpenMP tile loop
(Depth.cpp:1492-1624).
"""
import os


def shard_range(n, rank, world):
    """Contiguous [lo, hi) share of n items for `rank` (first n % world ranks get one more)."""
    base, extra = divmod(n, world)
    lo = rank * base + min(rank, extra)
    return lo, lo + base + (1 if rank < extra else 0)


def panorama_block(batch_per_rank, rank, base_seed=20261015):
    """Seeds of the panoramas rank `rank` owns in a batch-sharded run."""
    return [base_seed + rank * batch_per_rank + i for i in range(batch_per_rank)]


class HipTileShardBackend:
    """GPU backend of `fuse_tile_sharded` for one rank (pf_fuse_partial / pf_fuse_seed /
    pf_fuse_finish_level on a panofuse.Fuser bound to this rank's GPU).  tiles: [1, tile_elems]
    of the full layout (only [t0, t1) is read); coeffs: [ntiles, 4] or None; out: the int16
    [out_h, out_w] result written by the last level on rank 0."""

    def __init__(self, fuser, emap, tiles, coeffs, out_w, zr, out=None):
        import panofuse
        self.fz, self.emap, self.tiles, self.coeffs = fuser, emap, tiles, coeffs
        self.out_w, self.zr, self.out = out_w, zr, out
        n = panofuse.level_info(out_w, out_w // 2, zr, 0)[5]
        self.levels = [panofuse.level_info(out_w, out_w // 2, zr, lv) for lv in range(n)]

    def _plane(self, level):
        import torch
        w, h = self.levels[level][:2]
        return torch.empty(h * w, dtype=torch.float32, device=self.tiles.device)

    def partial(self, level, t0, t1):
        lsum, cnt = self._plane(level), self._plane(level)
        self.fz.fuse_partial(self.tiles, self.coeffs, t0, t1, self.out_w, self.zr, level,
                             lsum, cnt)
        return lsum, cnt

    def multicover_count(self, level):
        return self.fz.multicover_count(self.out_w, self.zr, level)

    def multicover(self, level, t0, t1):
        import torch
        c = torch.zeros(max(1, self.multicover_count(level)), dtype=torch.float32,
                        device=self.tiles.device)
        self.fz.multicover(self.tiles, self.coeffs, t0, t1, self.out_w, self.zr, level, c)
        return c

    def multicover_patch(self, level, contrib, lsum):
        self.fz.multicover_patch(self.out_w, self.zr, level, contrib, lsum)

    def seed(self, level, prev):
        buf = self._plane(level)
        self.fz.fuse_seed(self.emap if level == 0 else None, prev, self.out_w, self.zr, level,
                          buf)
        return buf

    def finish(self, level, lsum, cnt, buf, last):
        self.fz.fuse_finish_level(lsum, cnt, self.out_w, self.zr, level, buf,
                                  self.out if last else None)
        return buf


def fuse_tile_sharded(backend, nlevels, ntiles, rank, world, comm=None):
    """Tile-sharded fusion of one panorama.

    backend: object with
      partial(level, t0, t1) -> (lsum, cnt) tensors of the level (zeros outside the band),
      multicover_count(level) / multicover(level, t0, t1) / multicover_patch(level, contrib,
        lsum) -> the exact fix-up of pixels covered by three or more tiles,
      seed(level, prev) -> buf tensor (level 0 from the baseline, else upsampled prev),
      finish(level, lsum, cnt, buf, last) -> buf after the sweeps (u16 written when last).
    comm: TorchComm (reduce to rank 0) or a stand-in; None for world == 1.
    Returns rank 0's final level buffer (None on other ranks).
    """
    t0, t1 = shard_range(ntiles, rank, world)
    prev = None
    for level in range(nlevels):
        lsum, cnt = backend.partial(level, t0, t1)
        if world > 1:
            comm.reduce_sum(lsum, 0)
            comm.reduce_sum(cnt, 0)
            if backend.multicover_count(level):
                contrib = backend.multicover(level, t0, t1)
                comm.all_reduce_sum(contrib)
                if rank == 0:
                    backend.multicover_patch(level, contrib, lsum)
        if rank == 0:
            buf = backend.seed(level, prev)
            prev = backend.finish(level, lsum, cnt, buf, level == nlevels - 1)
    return prev if rank == 0 else None


# ---------------------------------------------------------------------------------------------
# Row-band sharding of the sweeps: removes the Amdahl ceiling of
# fuse_tile_sharded, whose Jacobi runs on rank 0 alone.  Every rank sweeps its own contiguous band
# of rows; before every pass but a level's first, the T+1 rows nearest each band edge are
# exchanged with the neighbouring ranks (a pass of depth T reads rows row0-T-1 .. row1+T).  Each
# band row is computed exactly as in the one-GPU fusion (the kernels are the same; the band is just
# the row range of the chunks), so the result is bit-identical.
#
# Round 5: every exchange carries only the rows its receiver reads.
#  * Targets: a sparse reduce-scatter by band rows.  The tiles are dealt to the ranks in layout
#    order, which for the band layouts is zenith band by zenith band, and the row bands start at
#    the first row of each rank's tiles (band_bounds), so a rank's tiles feed its own rows plus the
#    one boundary row its neighbour shares.  A rank computes its tiles' partial sums only on the
#    rows it needs (its band + halo) and the rows it sends (pf_fuse_partial_rows); it sends each
#    other rank the rows of that rank's band + halo where its tiles are non-zero -- in practice the
#    K = T+1 halo rows to each neighbour -- and adds what it receives (pf_rows_add).  The targets
#    depend on the tiles alone, so the replicated levels' rows travel in one round and the
#    row-sharded levels' in another (each group's multicover terms in one all-reduce).  The
#    coverage
#    count is layout-only, so every rank counts it itself, once per level and backend
#    (pf_fuse_coverage_rows, coverage_plane): only fp32 sums travel, never counts.
#  * Between levels: no broadcast of the bands.  The next level's first pass reads the 2x
#    upsample of the previous level on its band + halo, i.e. about T/2 + 2 rows of the
#    neighbouring ranks' previous bands, which they send (prev_exchange).
#  * The u16 result is gathered to rank 0 only.
#  * Rank 0 and the last rank own the rows above / below the band (k_border).
#  * The coarsest levels may be replicated (rep_levels, auto_rep_levels): their bands would be a
#    few halos deep, so each of their many short passes would wait on an exchange.  Every rank
#    sends its tile rows to every rank instead and runs the whole level alone (pf_fuse_level);
#    the next level then reads its previous rows locally.  At world 1 every level is replicated,
#    which is the one-GPU path.
# DESIGN.md section 6 tabulates the bytes per rank per panorama at C5.

class TorchComm:
    """The collectives fuse_row_sharded / fuse_tile_sharded need, over torch.distributed (RCCL
    on the GPU box, gloo on CPU).  stage_host=True runs every collective on host copies of
    device tensors (gloo with GPU data: several ranks sharing one GPU, where RCCL refuses a
    duplicate device) -- same values, the copies are exact."""

    def __init__(self, dist, group=None, stage_host=False):
        self.dist, self.group, self.stage = dist, group, stage_host

    def _host(self, t):
        return t.cpu() if self.stage and t.device.type != "cpu" else t

    def _back(self, h, t):
        if h is not t:
            t.copy_(h)

    def all_reduce_sum(self, t):
        h = self._host(t)
        self.dist.all_reduce(h, op=self.dist.ReduceOp.SUM, group=self.group)
        self._back(h, t)

    def reduce_sum(self, t, dst):
        h = self._host(t)
        self.dist.reduce(h, dst=dst, op=self.dist.ReduceOp.SUM, group=self.group)
        self._back(h, t)

    def exchange(self, sends, recvs):
        """sends: [(peer, tensor)], recvs: [(peer, tensor)]; point-to-point, all at once."""
        hs = [(peer, self._host(t)) for peer, t in sends]
        hr = [(peer, self._host(t), t) for peer, t in recvs]
        ops = [self.dist.P2POp(self.dist.isend, t, peer, group=self.group) for peer, t in hs]
        ops += [self.dist.P2POp(self.dist.irecv, h, peer, group=self.group) for peer, h, _ in hr]
        if ops:
            for req in self.dist.batch_isend_irecv(ops):
                req.wait()
        for _, h, t in hr:
            self._back(h, t)

    def broadcast(self, t, src):
        import torch
        if t.dtype == torch.int16:  # the u16 result: as bytes (gloo has no 16-bit integers)
            t = t.view(torch.uint8)
        h = self._host(t)
        self.dist.broadcast(h, src=src, group=self.group)
        self._back(h, t)

    def agree(self, values, src=0, device=None):
        """Rank `src`'s list of small ints on every rank (the pass plan of a level: every rank
        must run the same passes, or the halo exchanges would not pair up)."""
        import torch
        dev = device if (device is not None and not self.stage) else "cpu"
        n = torch.tensor([len(values)], dtype=torch.int64, device=dev)
        self.dist.broadcast(n, src=src, group=self.group)
        v = torch.zeros(int(n.item()), dtype=torch.int64, device=dev)
        if len(values) == v.numel():
            v.copy_(torch.tensor(values, dtype=torch.int64))
        self.dist.broadcast(v, src=src, group=self.group)
        return [int(x) for x in v.tolist()]


def band_rows(h0, h1, rank, world):
    """[row0, row1) of rank's band of the level rows h0..h1 (even split)."""
    lo, hi = shard_range(h1 - h0 + 1, rank, world)
    return h0 + lo, h0 + hi


def band_bounds(h0, h1, world, extents=None, halo=0):
    """Boundaries [b_0 = h0, b_1, .., b_world = h1 + 1] of the row bands: rank r sweeps
    [b_r, b_r+1).  extents[r] = (ymin, ymax), the rows where rank r's tiles have non-zero partial
    sums; when every rank has tiles and their first rows ascend with the rank (a band layout dealt
    in layout order), b_r = rank r's first row, so the partial sums stay local except for the
    boundary row and the halo.  Otherwise, or if a band would be thinner than `halo` + 1 rows, an
    even split.  A function of the layout only: identical on every rank."""
    even = [band_rows(h0, h1, r, world)[0] for r in range(world)] + [h1 + 1]
    if not extents or world == 1:
        return even
    b = [h0] + [extents[r][0] for r in range(1, world)] + [h1 + 1]
    if any(lo > hi for lo, hi in extents) or \
            any(b[r + 1] - b[r] < halo + 1 for r in range(world)):
        return even
    return b


def _span(a, b):
    """Intersection of two half-open row ranges, or None."""
    lo, hi = max(a[0], b[0]), min(a[1], b[1])
    return (lo, hi) if lo < hi else None


def owned_rows(bounds, h, rank):
    """Rows a rank owns at a level: its band, plus all rows above it (rank 0) or below it (the
    last rank) -- the border rows of k_border."""
    world = len(bounds) - 1
    lo = 0 if rank == 0 else bounds[rank]
    hi = h if rank == world - 1 else bounds[rank + 1]
    return lo, hi


def gather_rows(bounds, h, rank, local_from=None):
    """Rows of the last level's u16 result rank `rank` sends to rank 0: its owned rows, except
    that the last rank keeps the rows from `local_from` down, which rank 0's own border pass
    computes exactly (border_local_from)."""
    lo, hi = owned_rows(bounds, h, rank)
    if local_from is not None and rank == len(bounds) - 2:
        hi = max(bounds[-1], min(hi, local_from))
    return lo, hi


def border_local_from(dims, rep_levels):
    """First row of the last level from which rank 0's border pass (k_border: the rows outside
    [h0, h1], the previous level's nearest upsample) is exact by itself.  A level after a
    replicated one: every row below the band (rank 0 holds the previous level whole).  After a
    row-sharded level: border row y reads row y // 2 of the previous level, which rank 0 holds
    exactly from that level's own first exact border row fb on, so fb' = max(h1 + 1, 2 fb).  The
    last rank then sends only the rows above that (fuse_row_sharded's u16 gather)."""
    fb = None
    for lv, (w, h, h0, h1) in enumerate(dims):
        if lv < rep_levels or lv == 0:
            fb = None if lv < rep_levels else h1 + 1  # replicated (whole) / level 0 (zeros)
            continue
        fb = h1 + 1 if fb is None else max(h1 + 1, 2 * fb)
    return fb


def prev_rows_needed(bounds, h0, h1, K, hp, rank):
    """Rows of the previous level (hp rows) a rank's first pass and border read at this level: the
    2x upsample of its band + halo [b_r - K, b_r+1 + K) (a virtual column past a row end reaches
    one row more), all rows above for rank 0 and below for the last rank."""
    world = len(bounds) - 1
    lo = 0 if rank == 0 else max(0, ((max(h0, bounds[rank] - K - 1) - 1) >> 1) - 1)
    hi = hp if rank == world - 1 else min(hp, ((min(h1, bounds[rank + 1] + K) + 1) >> 1) + 2)
    return lo, hi


class ExchangeLog:
    """Bytes each rank sends per kind of exchange (DESIGN.md section 6's model is checked
    against it in tests/test_dist.py), and the number of exchange rounds (each a latency on the
    critical path)."""

    def __init__(self):
        self.sent = {}
        self.rounds = 0

    def add(self, kind, nbytes):
        self.sent[kind] = self.sent.get(kind, 0) + int(nbytes)
        self.rounds += 1


class NullComm:
    """A communicator that moves nothing: every rank's COMPUTE of the sharded flow can be run
    alone on one GPU (bench.py's 8-rank rehearsal times each rank's kernels this way; the values
    are not the sharded result)."""

    def exchange(self, sends, recvs):
        pass

    def all_reduce_sum(self, t):
        pass

    def agree(self, values, src=0, device=None):
        return list(values)


# Communication-avoiding pass halos (round 6): the passes after a level's first go in groups of up
# to PASS_GROUP with one halo exchange per group (PF_C5_GROUP=1: one exchange per pass, the
# round-5 flow).  A level takes the largest group size whose halo its thinnest band can supply.
PASS_GROUP = max(1, int(os.environ.get("PF_C5_GROUP", "4")))


def pass_groups(plan, group=None):
    """Per pass i of a row-sharded level: (k, ext).  k > 0: the halo rows exchanged with each
    neighbour before the pass (0: none); ext: the rows the pass computes past each side of the
    band.  A pass of depth T on rows [r0, r1) reads rows [r0 - T - 1, r1 + T + 1) (T sweeps, plus
    the row a virtual column wraps into).  group 1: every pass but the first exchanges T + 1 rows.
    group G: the passes after the first in runs of G share one exchange of sum(T + 1) rows, and
    each computes the rows past the band that the rest of its run reads (sum of their T + 1):
    1/G of the exchange rounds for the same bytes, some rows computed twice -- by the rank and by
    its neighbour, bit-identically."""
    group = max(1, PASS_GROUP if group is None else group)
    out = [(0, 0)] if plan else []
    for s0 in range(1, len(plan), group):
        run = plan[s0:s0 + group]
        need = [T + 1 for T in run]
        for j in range(len(run)):
            out.append((sum(need) if j == 0 else 0, sum(need[j + 1:])))
    return out


def halo_rows(plan, group=None):
    """The rows past its band a rank's passes read or compute on (targets, previous-level rows):
    the largest exchange of pass_groups, and the first pass's T + 1."""
    return max([plan[0] + 1] + [k for k, _ in pass_groups(plan, group)])


def level_geometry(h0, h1, world, ext, plan, gmax=None):
    """(group, K, bounds) of a row-sharded level: the largest pass group <= gmax whose halo K
    every band can supply (band_bounds' layout-dealt bands if thick enough, else the even split),
    falling back to group 1.  A function of the layout and the plan: identical on every rank and
    in exchange_model."""
    gmax = PASS_GROUP if gmax is None else gmax
    for g in range(max(1, gmax), 0, -1):
        K = halo_rows(plan, g)
        bnd = band_bounds(h0, h1, world, ext, K)
        if g == 1 or min(bnd[r + 1] - bnd[r] for r in range(world)) >= K:
            return g, K, bnd
    raise AssertionError("unreachable")


def fuse_row_sharded(backend, nlevels, ntiles, rank, world, comm=None, log=None, rep_levels=0):
    """One panorama's fusion with tiles AND rows sharded over `world` ranks.

    rep_levels: the first (coarsest) rep_levels levels are REPLICATED instead of row-sharded:
    every rank receives every other rank's partial target rows (an all-gather of the tile rows)
    and sweeps the whole level itself, with no halo exchange per pass; the next level then has
    every previous row locally.  Worth it where a rank's band is thin against the halo (many
    short passes, each an exchange on the critical path): C5's 1024-wide level at 8 ranks.

    backend (one rank's device):
      dims(level) -> (w, h, h0, h1)
      plane(level) -> a new full-level fp32 buffer (flat); scratch(n) -> n fp32
      tile_rows(level, t0, t1) -> (ymin, ymax)   rows with non-zero sums of tiles [t0, t1)
      partial_rows(level, t0, t1, row0, row1, lsum, cnt)   the sums of tiles [t0, t1) on rows
                                               [row0, row1) (cnt: their coverage count)
      coverage_plane(level) -> the coverage count of ALL tiles on the level's band (layout-only;
                                               a backend may count it once and keep it)
      rows_add(dst, src)                       dst += src (device views)
      multicover_count / multicover / multicover_patch   as fuse_tile_sharded
      normalize_rows(level, lsum, cnt, row0, row1, lnorm)
      level(level, prev, lsum, cnt, last) -> the level's plane (None after the last level)
                                               a replicated level: normalise + seeded sweeps
                                               (cnt None: lsum holds normalised targets)
      targets(level) -> the level's normalised targets from every tile (world 1)
      plan(level, nbands) -> [T, ...]          identical on every rank
      border(level, prev, a, b)               rows outside [h0, h1] (u16 `out` on the last level)
      band_pass(level, lnorm, src_mode, src, dst, T, row0, row1, last, prev)
                                               src_mode 0: src, 1: upsample prev, 2: emap seed
      out                                      the u16 result plane (flat); complete on rank 0
    comm: TorchComm (or a stand-in with exchange / all_reduce_sum / agree); None for world 1.
    log: an ExchangeLog, or None.
    Returns the bounds of the last level's bands."""
    t0, t1 = shard_range(ntiles, rank, world)
    prev, pbounds, bounds = None, None, None
    # the per-level geometry is a function of the layout and the plans only: computed (and the
    # plan agreed) once per backend, then reused by every panorama
    geo = getattr(backend, "_row_geo", None)
    if geo is None:
        geo = {}
        try:
            backend._row_geo = geo
        except AttributeError:
            pass
    # per-level geometry (plans agreed once per backend)
    G = []
    for level in range(nlevels):
        # replicated: the whole level on this rank (at world 1, every level: the one-GPU path)
        rep = world == 1 or level < rep_levels
        w, h, h0, h1 = backend.dims(level)
        key = (level, world, rep, ntiles)
        if key not in geo:
            plan = backend.plan(level, 1 if rep else world)
            if world > 1 and hasattr(comm, "agree"):
                # one plan for all ranks: rank 0's (the plan depends on per-process state -- CU
                # count, occupancy, PF_J* overrides -- and mismatched passes would hang the
                # exchanges)
                plan = comm.agree(plan, 0, getattr(backend, "device", None))
            ext = [backend.tile_rows(level, *shard_range(ntiles, r, world)) for r in range(world)]
            group = 1
            if rep:
                K = max(plan) + 1
                bnd = [h0] + [h1 + 1] * world  # rank 0's band is the level; all sweep it
                need = [(h0, h1 + 1)] * world
            else:
                group, K, bnd = level_geometry(h0, h1, world, ext, plan)
                if world > 1 and min(bnd[r + 1] - bnd[r] for r in range(world)) < K:
                    raise ValueError(f"level {level}: {h1 - h0 + 1} band rows over {world} ranks "
                                     f"leave bands thinner than the {K}-row halo")
                need = [(max(h0, bnd[d] - K), min(h1 + 1, bnd[d + 1] + K))
                        for d in range(world)]
            geo[key] = (plan, K, ext, bnd, need, group)
        G.append((rep, geo[key]))
    if world == 1:  # nothing travels: each level's normalised targets from every tile
        for level in range(nlevels):
            prev = backend.level(level, prev, backend.targets(level), None,
                                 level == nlevels - 1)
        return G[-1][1][3]
    # The targets depend on the tiles alone, so several levels' partial rows travel in ONE
    # exchange round and their multicover terms in ONE all-reduce (per-level rounds would each be
    # a latency on the critical path).  Two groups: the replicated levels, then the row-sharded
    # ones -- the second group's host work is queued while the GPU sweeps the first.  A rank sums
    # its tiles only on the rows it needs (its band + halo) and the rows it sends.
    tgt = {}

    # The targets of a group of levels in three phases: allocation (on the calling stream),
    # the tile sums and multicover terms (kernels only), and the exchange + adds.  A backend with
    # a side stream (HipRowShardBackend.side) runs the second phase of the row-sharded levels
    # beside the replicated levels' sweeps and the third when those are queued; the targets
    # depend on the tiles alone.
    def targets_alloc(levels):
        st = {"sends": [], "recvs": [], "bufs": [], "levels": list(levels)}
        for level in levels:
            rep, (plan, K, ext, bounds, need, group) = G[level]
            w = backend.dims(level)[0]
            lsum = backend.plane(level)
            mlo, mhi = ext[rank][0], ext[rank][1] + 1
            for d in range(world):
                if d == rank:
                    continue
                sp = _span(need[d], (mlo, mhi))
                if sp:
                    st["sends"].append((d, lsum[sp[0] * w:sp[1] * w]))
                s_lo, s_hi = ext[d][0], ext[d][1] + 1
                rp = _span(need[rank], (s_lo, s_hi)) if s_lo < s_hi else None
                if rp:
                    buf = backend.scratch((rp[1] - rp[0]) * w)
                    st["recvs"].append((d, buf))
                    st["bufs"].append((level, rp, buf))
            tgt[level] = (lsum, None)
        return st

    def targets_compute(st):
        for level in st["levels"]:
            rep, (plan, K, ext, bounds, need, group) = G[level]
            e0, e1 = need[rank]
            lsum = tgt[level][0]
            mlo, mhi = ext[rank][0], ext[rank][1] + 1
            lo, hi = (min(e0, mlo), max(e1, mhi)) if mlo < mhi else (e0, e1)
            backend.partial_rows(level, t0, t1, lo, hi, lsum, backend.plane(level))
            # every tile's coverage count (layout-only: counted once per backend and level)
            tgt[level] = (lsum, backend.coverage_plane(level))
        st["mcl"] = [lv for lv in st["levels"] if backend.multicover_count(lv)]
        st["parts"] = [backend.multicover(lv, t0, t1) for lv in st["mcl"]]

    def targets_finish(st):
        sends, recvs = st["sends"], st["recvs"]
        comm.exchange(sends, recvs)  # level-major on both sides: the pairs match in order
        if log:
            log.add("targets", sum(4 * t.numel() for _, t in sends))
        # one addend per covering tile: exact up to 2 (3+: below).  The adds go in the order
        # received (a pixel fed by two other ranks' tiles takes them in tile order); a batched
        # launch holds only segments that do not overlap, so an overlapping one starts a new
        # batch after the earlier adds.
        batch, spans = [], []
        for level, (a, b), buf in st["bufs"]:
            w = backend.dims(level)[0]
            dst = tgt[level][0][a * w:b * w]
            if not hasattr(backend, "rows_add_batch"):
                backend.rows_add(dst, buf)
                continue
            if any(lv == level and a < b_ and a_ < b for lv, a_, b_ in spans):
                backend.rows_add_batch(batch)
                batch, spans = [], []
            batch.append((dst, buf))
            spans.append((level, a, b))
        if batch:
            backend.rows_add_batch(batch)
        mcl, parts = st["mcl"], st["parts"]
        if mcl:  # exact sums where 3+ tiles meet, the group's terms in one all-reduce
            import torch
            allc = torch.cat(parts) if len(parts) > 1 else parts[0]
            comm.all_reduce_sum(allc)
            if log:
                log.add("multicover", 4 * allc.numel())
            o = 0
            for lv, part in zip(mcl, parts):
                backend.multicover_patch(lv, allc[o:o + part.numel()], tgt[lv][0])
                o += part.numel()

    def gather_targets(levels):
        st = targets_alloc(levels)
        targets_compute(st)
        targets_finish(st)

    nrep = sum(1 for r_, _ in G if r_)
    if nrep:
        gather_targets(range(nrep))
    side = backend.side if getattr(backend, "has_side", False) else None
    early = None
    if side is not None and 0 < nrep < nlevels:
        # the row-sharded levels' tile sums beside the replicated levels' sweeps
        early = targets_alloc(range(nrep, nlevels))
        with side():
            targets_compute(early)
    for level in range(nlevels):
        last = level == nlevels - 1
        rep, (plan, K, ext, bounds, need, group) = G[level]
        if level == nrep:
            if early is not None:
                # the exchange and adds follow the side stream's tile sums only, not the sweeps
                # queued on the calling stream since
                with side(wait=False):
                    targets_finish(early)
                backend.join()
            else:
                gather_targets(range(nrep, nlevels))
        w, h, h0, h1 = backend.dims(level)
        r0, r1 = (h0, h1 + 1) if rep else (bounds[rank], bounds[rank + 1])
        e0, e1 = need[rank]
        # the previous level's rows this rank's first pass / border read, from their owners
        # (after a replicated level every rank holds all of them)
        if level > 0 and pbounds is not None:
            hp = backend.dims(level - 1)[1]
            wp = backend.dims(level - 1)[0]
            psends, precvs = [], []
            mine = owned_rows(pbounds, hp, rank)
            for d in range(world):
                if d == rank:
                    continue
                sp = _span(prev_rows_needed(bounds, h0, h1, K, hp, d), mine)
                if sp:
                    psends.append((d, prev[sp[0] * wp:sp[1] * wp]))
                rp = _span(prev_rows_needed(bounds, h0, h1, K, hp, rank),
                           owned_rows(pbounds, hp, d))
                if rp:
                    precvs.append((d, prev[rp[0] * wp:rp[1] * wp]))
            comm.exchange(psends, precvs)
            if log:
                log.add("prev_halo", sum(4 * t.numel() for _, t in psends))
        lsum, cnt = tgt[level]
        if rep:  # the whole level on this rank: the one-GPU level (seed, normalise, sweeps)
            prev = backend.level(level, prev, lsum, cnt, last)
            pbounds = None
            continue
        lnorm = backend.plane(level)
        backend.normalize_rows(level, lsum, cnt, e0, e1, lnorm)
        a, b = backend.plane(level), backend.plane(level)
        if rank == 0 or rank == world - 1:  # the rows above / below the band
            backend.border(level, prev, a, b)
        src, dst = None, a
        groups = pass_groups(plan, group)
        for i, T in enumerate(plan):
            k, xt = groups[i]
            if k:
                hsends, hrecvs = [], []
                if rank > 0:
                    lo_ = max(r0 - k, h0)
                    hsends.append((rank - 1, src[r0 * w:min(r0 + k, r1) * w]))
                    hrecvs.append((rank - 1, src[lo_ * w:r0 * w]))
                if rank < world - 1:
                    hi_ = min(r1 + k, h1 + 1)
                    hsends.append((rank + 1, src[max(r1 - k, r0) * w:r1 * w]))
                    hrecvs.append((rank + 1, src[r1 * w:hi_ * w]))
                comm.exchange(hsends, hrecvs)
                if log:
                    log.add("pass_halo", sum(4 * t.numel() for _, t in hsends))
            mode = (2 if level == 0 else 1) if i == 0 else 0
            fin = last and i == len(plan) - 1
            backend.band_pass(level, lnorm, mode, src, dst, T, max(r0 - xt, h0),
                              min(r1 + xt, h1 + 1), fin, prev)
            src, dst = dst, (b if dst is a else a)
        prev, pbounds = (None if last else src), bounds
    bounds = G[-1][1][3]
    # the u16 result: every rank's owned rows to rank 0 (a replicated last level: all local),
    # except the rows below the band that rank 0's border pass computed (border_local_from)
    if pbounds is not None:
        import torch
        w, h = backend.dims(nlevels - 1)[:2]
        loc = border_local_from([backend.dims(lv) for lv in range(nlevels)], nrep)

        def out8(a_, b_):  # as bytes: gloo has no 16-bit integers
            return backend.out[a_ * w:b_ * w].view(torch.uint8)
        if rank == 0:
            recvs = [(s, out8(*gather_rows(bounds, h, s, loc))) for s in range(1, world)]
            comm.exchange([], recvs)
        else:
            snd = out8(*gather_rows(bounds, h, rank, loc))
            comm.exchange([(0, snd)], [])
            if log:
                log.add("gather_u16", snd.numel())
    return bounds


def exchange_model(dims, plans, ext, world, multicover=None, rep_levels=0):
    """Bytes each rank SENDS per panorama in fuse_row_sharded, by kind -- the same row arithmetic
    as the flow, from the layout alone (tests/test_dist.py checks it against
    the bytes a gloo run logs).  dims[l] = (w, h, h0, h1); plans[l] = the pass depths of level l;
    ext[l][r] = (ymin, ymax) of rank r's tiles at level l; multicover[l] = that level's count of
    (pixel, tile) pairs covered three or more times (one fp32 each, all-reduced)."""
    res = [dict() for _ in range(world)]

    def add(r, kind, n):
        if n:
            res[r][kind] = res[r].get(kind, 0) + n
    if world == 1:
        return res
    pb = None
    for lv, (w, h, h0, h1) in enumerate(dims):
        if lv < rep_levels:  # replicated: every rank's tile rows to every other rank
            for r in range(world):
                lo, hi = ext[lv][r][0], ext[lv][r][1] + 1
                if lo < hi:
                    add(r, "targets", 4 * w * (hi - lo) * (world - 1))
                if multicover and multicover[lv]:
                    add(r, "multicover", 4 * multicover[lv])
            pb = None
            continue
        group, K, b = level_geometry(h0, h1, world, ext[lv], plans[lv])
        need = [(max(h0, b[d] - K), min(h1 + 1, b[d + 1] + K)) for d in range(world)]
        for r in range(world):
            if lv > 0 and pb is not None:
                wp, hp = dims[lv - 1][:2]
                for d in range(world):
                    if d != r:
                        sp = _span(prev_rows_needed(b, h0, h1, K, hp, d), owned_rows(pb, hp, r))
                        add(r, "prev_halo", 4 * wp * (sp[1] - sp[0]) if sp else 0)
            lo, hi = ext[lv][r][0], ext[lv][r][1] + 1
            for d in range(world):
                if d != r and lo < hi:
                    sp = _span(need[d], (lo, hi))
                    add(r, "targets", 4 * w * (sp[1] - sp[0]) if sp else 0)
            if multicover and multicover[lv]:
                add(r, "multicover", 4 * multicover[lv])
            r0, r1 = b[r], b[r + 1]
            for k, _ in pass_groups(plans[lv], group):
                if not k:
                    continue
                if r > 0:
                    add(r, "pass_halo", 4 * w * (min(r0 + k, r1) - r0))
                if r < world - 1:
                    add(r, "pass_halo", 4 * w * (r1 - max(r1 - k, r0)))
        pb = b
    if pb is None:  # a replicated last level: no gather
        return res
    w, h = dims[-1][:2]
    loc = border_local_from(dims, rep_levels)
    for r in range(1, world):
        lo, hi = gather_rows(pb, h, r, loc)
        add(r, "gather_u16", 2 * w * (hi - lo))
    return res


def auto_rep_levels(backend, nlevels, world, ratio=10, comm=None):
    """The coarse levels worth replicating at `world` ranks: the leading levels whose band per
    rank is under `ratio` halos deep (each of their many short passes would wait for an exchange).
    The pass plans behind the choice depend on per-process state (CU count, occupancy, PF_J*
    overrides), so with a `comm` every rank takes rank 0's answer: ranks with different rep_levels
    would build different level geometries and their exchanges would not pair up."""
    if world <= 1:
        return 0
    n = 0
    for lv in range(nlevels - 1):  # the finest level stays sharded
        w, h, h0, h1 = backend.dims(lv)
        K = max(backend.plan(lv, world)) + 1
        if (h1 - h0 + 1) / world < ratio * K:
            n = lv + 1
        else:
            break
    if comm is not None and hasattr(comm, "agree"):
        n = comm.agree([n], 0, getattr(backend, "device", None))[0]
    return n


class HipRowShardBackend:
    """GPU backend of `fuse_row_sharded` for one rank: the panofuse band entry points on a
    panofuse.Fuser bound to this rank's GPU.  tiles: [1, tile_elems] of the full layout (only
    [t0, t1) is read); coeffs: [ntiles, 4] or None; out: flat int16 [out_h * out_w]."""

    def __init__(self, fuser, emap, tiles, coeffs, out_w, zr, out):
        import panofuse
        self.fz, self.emap, self.tiles, self.coeffs = fuser, emap, tiles, coeffs
        self.out_w, self.zr, self.out = out_w, zr, out
        n = panofuse.level_info(out_w, out_w // 2, zr, 0)[5]
        self.levels = [panofuse.level_info(out_w, out_w // 2, zr, lv) for lv in range(n)]
        self.nlevels = n

    def dims(self, level):
        w, h, h0, h1 = self.levels[level][:4]
        return w, h, h0, h1

    @property
    def device(self):
        return self.tiles.device

    def plane(self, level):
        import torch
        w, h = self.levels[level][:2]
        return torch.empty(h * w, dtype=torch.float32, device=self.tiles.device)

    def scratch(self, n):
        import torch
        return torch.empty(n, dtype=torch.float32, device=self.tiles.device)

    def tile_rows(self, level, t0, t1):
        return self.fz.fuse_tile_rows(self.out_w, self.zr, level, t0, t1)

    def partial_rows(self, level, t0, t1, row0, row1, lsum, cnt):
        self.fz.fuse_partial_rows(self.tiles, self.coeffs, t0, t1, self.out_w, self.zr, level,
                                  row0, row1, lsum, cnt)

    def coverage_plane(self, level):
        cov = self.__dict__.setdefault("_cov", {})
        if level not in cov:
            w, h, h0, h1 = self.levels[level][:4]
            cov[level] = self.plane(level)
            self.fz.fuse_coverage_rows(self.out_w, self.zr, level, h0, h1 + 1, cov[level])
        return cov[level]

    def rows_add(self, dst, src):
        self.fz.rows_add(dst, src)

    def rows_add_batch(self, pairs):
        self.fz.rows_add_batch(pairs)

    def enable_side(self, fuser):
        """A second panofuse.Fuser of the same layout on its own stream: fuse_row_sharded runs the
        row-sharded levels' tile sums on it beside the replicated levels' sweeps (side / join)."""
        self.fz_side = fuser
        self.has_side = True

    def side(self, wait=True):
        """Context: the backend's kernels go to the side Fuser's stream, which first waits for
        everything queued so far on the calling stream (wait=False: only for its own earlier
        work); torch's current stream is the side stream too (collectives, host copies).
        Tensors the main stream uses later are allocated outside (targets_alloc)."""
        import contextlib
        import torch
        be = self

        @contextlib.contextmanager
        def ctx():
            s = be.fz_side.stream
            if wait:
                s.wait_stream(torch.cuda.current_stream(be.tiles.device))
            fz, be.fz = be.fz, be.fz_side
            try:
                with torch.cuda.stream(s):
                    yield
            finally:
                be.fz = fz
        return ctx()

    def join(self):
        """The calling stream waits for the side stream's work."""
        import torch
        torch.cuda.current_stream(self.tiles.device).wait_stream(self.fz_side.stream)

    multicover_count = HipTileShardBackend.multicover_count
    multicover = HipTileShardBackend.multicover
    multicover_patch = HipTileShardBackend.multicover_patch

    def normalize_rows(self, level, lsum, cnt, row0, row1, lnorm):
        self.fz.fuse_normalize_rows(lsum, cnt, self.out_w, self.zr, level, row0, row1, lnorm)

    def targets(self, level):
        lnorm = self.plane(level)
        self.fz.fuse_targets(self.tiles, self.coeffs, self.out_w, self.zr, level, lnorm)
        return lnorm

    def level(self, level, prev, lsum, cnt, last):
        """A replicated level: the one-GPU level from the summed targets (pf_fuse_level: seeded
        inside the first sweep pass).  Returns the level's plane (None after the last)."""
        buf = self.plane(level)
        self.fz.fuse_level(self.emap if level == 0 else None, prev, lsum, cnt, self.out_w,
                           self.zr, level, buf,
                           self.out.view(self.levels[level][1], -1) if last else None)
        return None if last else buf

    def plan(self, level, nbands):
        return self.fz.fuse_band_plan(self.out_w, self.zr, level, nbands)

    def border(self, level, prev, a, b):
        if level == self.nlevels - 1:
            self.fz.fuse_border(prev, self.out_w, self.zr, level, a=a, b=b, out=self.out)
        else:
            self.fz.fuse_border(prev, self.out_w, self.zr, level, a=a, b=b)

    def band_pass(self, level, lnorm, src_mode, src, dst, T, row0, row1, last, prev):
        self.fz.fuse_band_pass(lnorm, src_mode, self.out_w, self.zr, level, T, row0, row1,
                               src=src if src_mode == 0 else None,
                               dst=None if last else dst,
                               prev=prev if src_mode == 1 else None,
                               emap=self.emap if src_mode == 2 else None,
                               out=self.out if last else None)
