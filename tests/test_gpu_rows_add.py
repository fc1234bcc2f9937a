"""pf_rows_add_batch (round 6): all of a level's received partial rows added in one launch.

The sharded fusion (pf_dist.fuse_row_sharded) adds the target rows other ranks send into its own
sums.  The batched launch takes any number of (dst, src, n) segments of any length (empty and
odd ones included) whose destinations do not overlap; each must come out exactly as the single
pf_rows_add of the same segment (one fp32 add per element)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

import panofuse  # noqa: E402
import pf_layouts as PL  # noqa: E402

DEV = "cuda:0"


@pytest.fixture(scope="module")
def fuser():
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a host without a GPU")
    f = panofuse.Fuser(0)
    f.set_tiles(PL.config_layout("C1"))  # the row entry points check for a layout, as in the flow
    return f


def test_rows_add_batch_equals_single_adds(fuser):
    rng = np.random.default_rng(5)
    base = torch.from_numpy(rng.normal(0, 1, 1 << 20).astype(np.float32)).to(DEV)
    # disjoint destination segments of mixed lengths (0, 1, odd, multiples of 4, > 64 K), more
    # than one launch's worth (32) with empty ones in between: every segment added exactly once
    lens = [0, 1, 3, 4, 17, 255, 4096, 65537, 100003, 7]
    lens += [0 if i % 5 == 0 else int(rng.integers(1, 3000)) for i in range(70)]
    segs, o = [], 0
    for n in lens:
        segs.append((o, n))
        o += n + int(rng.integers(0, 9))
    srcs = [torch.from_numpy(rng.normal(0, 1, n).astype(np.float32)).to(DEV) for _, n in segs]
    a, b = base.clone(), base.clone()
    fuser.rows_add_batch([(a[s:s + n], src) for (s, n), src in zip(segs, srcs)])
    for (s, n), src in zip(segs, srcs):
        if n:
            fuser.rows_add(b[s:s + n], src)
    torch.cuda.synchronize()
    assert torch.equal(a.view(torch.int32), b.view(torch.int32))
    # and both equal the host's fp32 adds
    ref = base.cpu().numpy().copy()
    for (s, n), src in zip(segs, srcs):
        ref[s:s + n] += src.cpu().numpy()
    assert np.array_equal(a.cpu().numpy().view(np.uint32), ref.view(np.uint32))


def test_rows_add_batch_empty_list_is_a_no_op(fuser):
    fuser.rows_add_batch([])
