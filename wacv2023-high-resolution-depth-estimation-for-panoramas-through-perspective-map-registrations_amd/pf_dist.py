"""Multi-GPU decomposition of the fusion path.

* Batch sharding (configs C3/C4): panoramas are independent, so rank r simply processes its own
  contiguous block of panoramas; no collective touches the data path (`panorama_block`).
* Tile sharding of one huge panorama (config C5): per fusion level every rank scatters the
  Laplacian targets of its contiguous share of the tiles into full-level (sum L, n) grids, the
  grids are summed over ranks (RCCL reduce over xGMI; gloo in the CPU tests), and rank 0
  normalises and runs the damped Jacobi sweeps (`fuse_tile_sharded`).  With every pixel covered
  by at most two tiles (the reference's layouts) the reduced sums are exactly the single-GPU
  sums: adding zeros is exact and a + b is commutative.

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

    def seed(self, level, prev):
        buf = self._plane(level)
        self.fz.fuse_seed(self.emap if level == 0 else None, prev, self.out_w, self.zr, level,
                          buf)
        return buf

    def finish(self, level, lsum, cnt, buf, last):
        self.fz.fuse_finish_level(lsum, cnt, self.out_w, self.zr, level, buf,
                                  self.out if last else None)
        return buf


def fuse_tile_sharded(backend, nlevels, ntiles, rank, world, dist=None, group=None):
    """Tile-sharded fusion of one panorama.

    backend: object with
      partial(level, t0, t1) -> (lsum, cnt) tensors of the level (zeros outside the band),
      seed(level, prev) -> buf tensor (level 0 from the baseline, else upsampled prev),
      finish(level, lsum, cnt, buf, last) -> buf after the sweeps (u16 written when last).
    Returns rank 0's final level buffer (None on other ranks).
    """
    t0, t1 = shard_range(ntiles, rank, world)
    prev = None
    for level in range(nlevels):
        lsum, cnt = backend.partial(level, t0, t1)
        if dist is not None and world > 1:
            dist.reduce(lsum, dst=0, op=dist.ReduceOp.SUM, group=group)
            dist.reduce(cnt, dst=0, op=dist.ReduceOp.SUM, group=group)
        if rank == 0:
            buf = backend.seed(level, prev)
            prev = backend.finish(level, lsum, cnt, buf, level == nlevels - 1)
    return prev if rank == 0 else None
