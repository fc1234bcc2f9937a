"""The software-pipelined bench steps: bench.pipelined_step (warp of batch k+1 on a second stream
while batch k is registered and fused) and bench.lane_steps (N fusion lanes, batch k on lane
k % N, the default schedule with N = 2).  Every step must produce exactly the serial step's
result (the bench repeats one batch, so each step's output is the same panoramas), and the bench
line of a short pipelined run must carry the contract's fields."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import panofuse  # noqa: E402
import pf_layouts as PL  # noqa: E402
import pf_synth  # noqa: E402


def test_pipelined_steps_equal_serial():
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a host without a GPU")
    dev = torch.device("cuda:0")
    B, zr = 4, PL.ZENITH_RANGE
    lay = PL.config_layout("C2")
    seeds = pf_synth.seeds_for(B, 20261015 + 5)
    gt = pf_synth.scene_depth(seeds, 2048, 1024, dev).contiguous()
    emap = pf_synth.baseline_emap(seeds, 512, 256, dev).contiguous()
    resp = panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), dev)
    fz = panofuse.Fuser(0)
    fz.set_tiles(lay)
    tiles = torch.empty((B, fz.tile_elems), dtype=torch.float32, device=dev)
    # serial reference
    ref = torch.zeros((B, 1024, 2048), dtype=torch.int16, device=dev)
    rc = torch.zeros((B, lay.ntiles, 4), dtype=torch.float32, device=dev)
    fz.warp_depth(gt, tiles, resp)
    fz.merge(emap, tiles, ref, zr, coeffs=rc)
    torch.cuda.synchronize()
    out = torch.zeros_like(ref)
    coeffs = torch.zeros_like(rc)
    step = bench.pipelined_step(fz, lay, 0, dev, gt, emap, resp, tiles, out, coeffs, zr)
    for _ in range(3):
        out.zero_()
        step()
        torch.cuda.synchronize()
        assert torch.equal(out, ref)
        assert torch.equal(coeffs, rc)


def test_lane_steps_equal_serial():
    """Two and three lanes in flight at once (own contexts, streams and buffers; the resident
    level-0 kernels of different lanes run concurrently): every lane's output and coefficients
    equal the serial step's, and no resident hand-off timed out (synchronize() raises)."""
    if not torch.cuda.is_available():
        pytest.fail("GPU test collected on a host without a GPU")
    dev = torch.device("cuda:0")
    B, zr = 8, PL.ZENITH_RANGE
    lay = PL.config_layout("C2")
    seeds = pf_synth.seeds_for(B, 20261015 + 9)
    gt = pf_synth.scene_depth(seeds, 2048, 1024, dev).contiguous()
    emap = pf_synth.baseline_emap(seeds, 512, 256, dev).contiguous()
    resp = panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), dev)
    fz = panofuse.Fuser(0)
    fz.set_tiles(lay)
    tiles = torch.empty((B, fz.tile_elems), dtype=torch.float32, device=dev)
    ref = torch.zeros((B, 1024, 2048), dtype=torch.int16, device=dev)
    rc = torch.zeros((B, lay.ntiles, 4), dtype=torch.float32, device=dev)
    fz.warp_depth(gt, tiles, resp)
    fz.merge(emap, tiles, ref, zr, coeffs=rc)
    torch.cuda.synchronize()
    for n in (2, 3):
        out = torch.zeros_like(ref)
        coeffs = torch.zeros_like(rc)
        step, lanes = bench.lane_steps(fz, lay, 0, dev, gt, emap, resp, tiles, out, coeffs, zr, n)
        assert len(lanes) == n and lanes[0][2] is out
        for _, _, o, c in lanes:
            o.zero_()
            c.zero_()
        for _ in range(2 * n):  # every lane twice, all enqueued before one synchronize
            step()
        torch.cuda.synchronize()
        for f, _, o, c in lanes:
            f.synchronize()
            assert torch.equal(o, ref) and torch.equal(c, rc)


def test_pipelined_bench_line():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup",
                        "1", "--batch", "8", "--no-cpu-baseline", "--prof-steps", "1",
                        "--pipeline", "1"], capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "roofline",
              "config"):
        assert k in d, k
    assert d["steps"] == 3 and d["n_gpus"] == 1 and d["value"] > 0
    assert "warp of batch k+1" in d["config"]["pipeline"]
    assert 0 < d["roofline"]["frac"] <= 1
    assert d["bit_exact_vs_one_process"] is True
    # the other single-GPU configs ride along in the line
    assert d["c2_batch1_ms"] > 0 and d["c2_batch1"]["reps"] >= 5
    assert d["c5_one_gpu"]["value"] > 0 and d["c5_one_gpu"]["bit_exact_vs_one_gpu"] is True


def test_lanes_bench_line():
    """The default schedule (two fusion lanes) end to end: contract fields, bit-exact output."""
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "4", "--warmup",
                        "2", "--batch", "8", "--no-cpu-baseline", "--prof-steps", "1",
                        "--no-extra-configs"], capture_output=True, text=True, timeout=300,
                       cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["steps"] == 4 and d["n_gpus"] == 1 and d["value"] > 0
    assert d["config"]["pipeline"].startswith("2 fusion lanes")
    assert d["bit_exact_vs_one_process"] is True
