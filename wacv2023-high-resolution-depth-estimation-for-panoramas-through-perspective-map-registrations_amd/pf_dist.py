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
# fuse_tile_sharded, whose Jacobi runs on rank 0 alone.  Every rank scatters its tiles' targets,
# the grids are all-reduced, and each rank sweeps its own contiguous band of rows; before every
# pass but a level's first, the T+1 rows nearest each band edge are exchanged with the
# neighbouring ranks (a pass of depth T reads rows row0-T-1 .. row1+T).  Each band row is
# computed exactly as in the one-GPU fusion (the kernels are the same; the band is just the row
# range of the chunks), so the result is bit-identical.  After a level its bands are broadcast
# so every rank holds the full buffer the next level upsamples; the u16 bands likewise.

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
    """[row0, row1) of rank's band of the level rows h0..h1."""
    lo, hi = shard_range(h1 - h0 + 1, rank, world)
    return h0 + lo, h0 + hi


def fuse_row_sharded(backend, nlevels, ntiles, rank, world, comm=None):
    """One panorama's fusion with tiles AND rows sharded over `world` ranks.

    backend (one rank's device):
      partial(level, t0, t1) -> (lsum, cnt)   the targets of tiles [t0, t1), full-level grids
      multicover_count / multicover / multicover_patch   as fuse_tile_sharded
      dims(level) -> (w, h, h0, h1)
      plane(level) -> a new full-level fp32 buffer (flat)
      normalize(level, lsum, cnt) -> lnorm
      plan(level, nbands) -> [T, ...]          identical on every rank
      border(level, prev, a, b)               rows outside [h0, h1] (u16 `out` on the last level)
      band_pass(level, lnorm, src_mode, src, dst, T, row0, row1, last, prev)
                                               src_mode 0: src, 1: upsample prev, 2: emap seed
      out                                      the u16 result plane (flat), filled on every rank
    comm: TorchComm (or a stand-in with the same methods); None for world == 1.
    Returns the final level's band-assembled buffer (None for the last level, whose result is
    backend.out)."""
    t0, t1 = shard_range(ntiles, rank, world)
    prev = None
    for level in range(nlevels):
        last = level == nlevels - 1
        lsum, cnt = backend.partial(level, t0, t1)
        if world > 1:
            comm.all_reduce_sum(lsum)
            comm.all_reduce_sum(cnt)
            if backend.multicover_count(level):  # exact sums where 3+ tiles meet
                contrib = backend.multicover(level, t0, t1)
                comm.all_reduce_sum(contrib)
                backend.multicover_patch(level, contrib, lsum)
        lnorm = backend.normalize(level, lsum, cnt)
        w, h, h0, h1 = backend.dims(level)
        r0, r1 = band_rows(h0, h1, rank, world)
        plan = backend.plan(level, world)
        if world > 1 and hasattr(comm, "agree"):
            # one plan for all ranks: rank 0's (the plan depends on per-process state -- CU
            # count, occupancy, PF_J* overrides -- and mismatched passes would hang the exchanges)
            plan = comm.agree(plan, 0, getattr(backend, "device", None))
        if world > 1 and (h1 - h0 + 1) // world < max(plan) + 1:
            raise ValueError(f"level {level}: {h1 - h0 + 1} band rows over {world} ranks leave "
                             f"bands thinner than the {max(plan) + 1}-row halo")
        a, b = backend.plane(level), backend.plane(level)
        backend.border(level, prev, a, b)
        src, dst = None, a
        for i, T in enumerate(plan):
            if i > 0 and world > 1:
                k = T + 1
                sends, recvs = [], []
                if rank > 0:
                    lo = max(r0 - k, h0)
                    sends.append((rank - 1, src[r0 * w:min(r0 + k, r1) * w]))
                    recvs.append((rank - 1, src[lo * w:r0 * w]))
                if rank < world - 1:
                    hi = min(r1 + k, h1 + 1)
                    sends.append((rank + 1, src[max(r1 - k, r0) * w:r1 * w]))
                    recvs.append((rank + 1, src[r1 * w:hi * w]))
                comm.exchange(sends, recvs)
            mode = (2 if level == 0 else 1) if i == 0 else 0
            fin = last and i == len(plan) - 1
            backend.band_pass(level, lnorm, mode, src, dst, T, r0, r1, fin, prev)
            src, dst = dst, (b if dst is a else a)
        res = backend.out if last else src
        if world > 1:
            for r in range(world):
                q0, q1 = band_rows(h0, h1, r, world)
                comm.broadcast(res[q0 * w:q1 * w], r)
        prev = None if last else res
    return prev


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

    def partial(self, level, t0, t1):
        lsum, cnt = self.plane(level), self.plane(level)
        self.fz.fuse_partial(self.tiles, self.coeffs, t0, t1, self.out_w, self.zr, level,
                             lsum, cnt)
        return lsum, cnt

    multicover_count = HipTileShardBackend.multicover_count
    multicover = HipTileShardBackend.multicover
    multicover_patch = HipTileShardBackend.multicover_patch

    def normalize(self, level, lsum, cnt):
        lnorm = self.plane(level)
        self.fz.fuse_normalize(lsum, cnt, self.out_w, self.zr, level, lnorm)
        return lnorm

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
