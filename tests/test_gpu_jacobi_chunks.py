"""The streamed Jacobi passes under forced row chunkings and sweep depths (round 5: the chunk's
fill and drain are compiled as their own steps, and a chunk too short for both takes the plain
loop).  Every forced plan must give the default fusion's u16 output bit for bit -- C2, two
panoramas, the level-0 kernel switched to streamed passes so that all three levels take the
forced chunkings (PF_JN<w>: row chunks per pass of the level of width w; PF_JT<w>: its largest
sweep depth).  Chunks of 1-7 rows are shorter than the fill (3 groups of 6 steps) plus the drain.
"""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import panofuse  # noqa: E402
import pf_layouts as PL  # noqa: E402
import pf_synth  # noqa: E402

DEV = "cuda:0"
CASES = [
    {"PF_JN1024": "60"},                      # ~6-row chunks at level 1
    {"PF_JN2048": "731"},                     # one row per chunk at level 2
    {"PF_JN2048": "300", "PF_JN1024": "120"},  # 2-3 rows
    {"PF_JN512": "23", "PF_JT512": "4"},      # level 0 streamed at T <= 4, 8-row chunks
    {"PF_JT1024": "8", "PF_JT2048": "5", "PF_JN2048": "7"},
]


@pytest.fixture(scope="module")
def inputs():
    lay = PL.config_layout("C2")
    seeds = pf_synth.seeds_for(2, 20261015 + 21)
    gt = pf_synth.scene_depth(seeds, 2048, 1024, DEV).contiguous()
    emap = pf_synth.baseline_emap(seeds, 512, 256, DEV).contiguous()
    f = panofuse.Fuser(0)
    f.set_tiles(lay)
    tiles = torch.zeros((2, f.tile_elems), dtype=torch.float32, device=DEV)
    f.warp_depth(gt, tiles, panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), DEV))
    coeffs = torch.zeros((2, lay.ntiles, 4), dtype=torch.float32, device=DEV)
    f.register(emap, tiles, PL.ZENITH_RANGE, apply=False, coeffs=coeffs)
    f.set_jacobi_engine(resident=False)
    ref = torch.zeros((2, 1024, 2048), dtype=torch.int16, device=DEV)
    f.fuse(emap, tiles, ref, PL.ZENITH_RANGE, coeffs=coeffs)
    torch.cuda.synchronize()
    yield f, emap, tiles, coeffs, ref
    f.close()


@pytest.mark.parametrize("env", CASES, ids=["-".join(f"{k[3:]}{v}" for k, v in c.items())
                                           for c in CASES])
def test_forced_chunks_bit_exact(inputs, env):
    f, emap, tiles, coeffs, ref = inputs
    old = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        out = torch.zeros_like(ref)
        f.fuse(emap, tiles, out, PL.ZENITH_RANGE, coeffs=coeffs)
        torch.cuda.synchronize()
    finally:
        for k, v in old.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    bad = int((out != ref).sum())
    assert bad == 0, f"{env}: {bad} pixels differ from the default plan's fusion"
    assert np.count_nonzero(out.cpu().numpy()) > 0


@pytest.mark.parametrize("share", [0.75, 0.3, 0.01])
def test_jacobi_share_bit_exact(inputs, share):
    """pf_set_jacobi_share (round 6): a context planning for part of the chip re-cuts its passes
    into fewer, longer row chunks; the output stays the whole-chip plan's bit for bit."""
    f, emap, tiles, coeffs, ref = inputs
    f.set_jacobi_share(share)
    try:
        out = torch.zeros_like(ref)
        f.fuse(emap, tiles, out, PL.ZENITH_RANGE, coeffs=coeffs)
        torch.cuda.synchronize()
    finally:
        f.set_jacobi_share(1.0)
    assert torch.equal(out, ref)


def test_jacobi_share_rejects_out_of_range(inputs):
    f = inputs[0]
    for bad in (0.0, -0.5, 1.5, float("nan")):
        with pytest.raises(panofuse.PanofuseError):
            f.set_jacobi_share(bad)
