"""The resident level kernel (pf_jres.hip) against the streaming Jacobi passes (pf_jacobi.hip).

Both engines restate the same sweeps (Depth.cpp:1649-1718) in the reference's fp32 operand
order, so their u16 outputs must be equal bit for bit, whatever the row blocking of the resident
kernel (blocks per panorama, hence halo depth K and the number of hand-off rounds), the batch
size, or how many resident launches share the chip.  The streaming engine itself is held to the
oracle by test_gpu_parity.py / test_gpu_configs.py, and those tests now run the resident kernel
too (it is the default wherever it applies).
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import panofuse  # noqa: E402
import pf_layouts as PL  # noqa: E402

ZR = PL.ZENITH_RANGE
DEV = "cuda:0"
OUT_W = {"C1": 512, "C2": 2048, "LERES": 2048}
EW = {"C1": 128, "C2": 512, "LERES": 512}


def _inputs(cfg, batch, seed):
    lay = PL.config_layout(cfg)
    ew = EW[cfg]
    g = torch.Generator(device="cpu").manual_seed(seed)
    emap = torch.rand((batch, ew // 2, ew), generator=g).to(DEV)
    total = int(sum(int(lay.tile_w[i]) * int(lay.tile_h[i]) for i in range(lay.ntiles)))
    tiles = torch.rand((batch, total), generator=g).to(DEV)
    return lay, emap, tiles


def _fuse(f, lay, emap, tiles, out_w):
    f.set_tiles(lay)
    out = torch.zeros((emap.shape[0], out_w // 2, out_w), dtype=torch.int16, device=DEV)
    f.fuse(emap, tiles, out, ZR)
    return out


@pytest.fixture(scope="module")
def fusers():
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a host without a GPU")
    a, b = panofuse.Fuser(0), panofuse.Fuser(0)
    a.set_jacobi_engine(resident=False)
    return a, b


@pytest.mark.parametrize("cfg,batch", [("C1", 1), ("C1", 5), ("C2", 1), ("C2", 3), ("C2", 16),
                                       ("LERES", 2)])
def test_resident_equals_streaming(fusers, cfg, batch):
    stream, res = fusers
    lay, emap, tiles = _inputs(cfg, batch, 11 + batch)
    ref = _fuse(stream, lay, emap, tiles, OUT_W[cfg])
    res.set_jacobi_engine(resident=True)
    got = _fuse(res, lay, emap, tiles, OUT_W[cfg])
    torch.cuda.synchronize()
    assert res.jres_errors() == 0
    assert torch.equal(got, ref)


@pytest.mark.parametrize("nb", [2, 3, 4, 5, 8, 13])
def test_resident_row_blockings(fusers, nb):
    """Forced blocks per panorama: K = min(core, (64 - core) / 2) ranges from 4 (nb 3) to
    the core itself (nb 8, 13: a row sits in both published edges when core < 2K)."""
    stream, res = fusers
    lay, emap, tiles = _inputs("C2", 2, 100 + nb)
    ref = _fuse(stream, lay, emap, tiles, 2048)
    res.set_jacobi_engine(resident=True, row_blocks=nb)
    got = _fuse(res, lay, emap, tiles, 2048)
    res.set_jacobi_engine(resident=True)
    assert res.jres_errors() == 0
    assert torch.equal(got, ref)


def test_resident_concurrent_launches(fusers):
    """Two contexts on two streams run full-chip resident launches at once (each grid fills
    every CU): the ticket order keeps them deadlock-free and the results unchanged."""
    stream, res = fusers
    other = panofuse.Fuser(0)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    lay, emap, tiles = _inputs("C2", 64, 7)
    lay2, emap2, tiles2 = _inputs("C2", 64, 8)
    ref1 = _fuse(stream, lay, emap, tiles, 2048)
    ref2 = _fuse(stream, lay2, emap2, tiles2, 2048)
    torch.cuda.synchronize()
    res.set_stream(s1)
    other.set_stream(s2)
    res.set_tiles(lay)
    other.set_tiles(lay2)
    o1 = torch.zeros((64, 1024, 2048), dtype=torch.int16, device=DEV)
    o2 = torch.zeros_like(o1)
    for _ in range(3):
        res.fuse(emap, tiles, o1, ZR)
        other.fuse(emap2, tiles2, o2, ZR)
    torch.cuda.synchronize()
    res.set_stream(None)
    assert res.jres_errors() == 0 and other.jres_errors() == 0
    assert torch.equal(o1, ref1)
    assert torch.equal(o2, ref2)
    other.close()


def test_resident_timeout_is_reported(fusers):
    """VERDICT r3 item 3 / ADVICE r3: a resident hand-off wait that times out must surface as
    PF_ETIMEOUT (pf_synchronize, or the next pf_fuse / pf_merge), not as a silently wrong
    panorama.  The fault hook makes row block 0 withhold its flag in one launch with waits
    bounded at 2^10 polls; the launches after it run normally and stay bit-exact."""
    stream, _ = fusers
    f = panofuse.Fuser(0)
    f.set_jacobi_engine(resident=True, row_blocks=4)  # 4 blocks per panorama: hand-offs happen
    lay, emap, tiles = _inputs("C2", 2, 321)
    ref = _fuse(stream, lay, emap, tiles, 2048)
    torch.cuda.synchronize()
    # 1. reported by pf_synchronize
    f.debug_jres_fault(10)
    _fuse(f, lay, emap, tiles, 2048)
    with pytest.raises(panofuse.PanofuseError) as e:
        f.synchronize()
    assert e.value.code == panofuse.PF_ETIMEOUT and "timed out" in str(e.value)
    assert f.jres_errors() > 0
    # 2. the next launch runs normally: no error, bit-exact
    got = _fuse(f, lay, emap, tiles, 2048)
    f.synchronize()
    assert torch.equal(got, ref)
    # 3. reported by the next pf_fuse once the faulty fusion has finished
    f.debug_jres_fault(10)
    _fuse(f, lay, emap, tiles, 2048)
    torch.cuda.synchronize()
    with pytest.raises(panofuse.PanofuseError) as e:
        _fuse(f, lay, emap, tiles, 2048)
    assert e.value.code == panofuse.PF_ETIMEOUT
    got = _fuse(f, lay, emap, tiles, 2048)
    f.synchronize()
    assert torch.equal(got, ref)
    f.close()
