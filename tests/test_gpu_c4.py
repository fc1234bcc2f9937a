"""BASELINE config C4 -- a batch of 512 panoramas (2048x1024, 20 tiles each) sharded over 8 ranks,
64 per rank, no collective on the data path -- in the GPU suite.

`bench.py --gpus 8` is run the way the driver runs it (directly, no torchrun: it launches its 8
ranks itself, before any GPU call).  The test box has one GPU, so the 8 ranks share cuda:0 and
talk over gloo (--same-device --backend gloo; RCCL refuses two ranks on one device); on an 8-GPU
node the same code runs one rank per GPU.  The rate is therefore not a scaling number.  Checked:

* the line: n_gpus 8, global_batch 512, the whole-job value over the slowest rank's time;
* 8 disjoint, contiguous seed blocks of 64 (pf_dist.panorama_block);
* every rank's fused batch equals a fresh one-process fusion of the same panoramas
  (bit_exact_all_ranks, each rank's own flag);
* one sampled panorama per rank (a different position in each block) equals the CPU oracle's
  warp + MergeDepthMaps (Depth.cpp:754-1041, Main.cpp:489-685's per-panorama loop) bit for bit,
  from the inputs the rank dumped (--sample-dump), and hashes as the rank reported.
"""
import hashlib
import json
import os
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD, B, STEPS = 8, 64, 2


@pytest.mark.timeout(900)
def test_c4_eight_ranks_every_rank_checked(tmp_path):
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    dump = tmp_path / "samples"
    cmd = [sys.executable, "bench.py", "--gpus", str(WORLD), "--same-device", "--backend", "gloo",
           "--batch", str(B), "--steps", str(STEPS), "--warmup", "1", "--prof-steps", "1",
           "--no-cpu-baseline", "--no-extra-configs", "--sample-dump", str(dump)]
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=840, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == WORLD and d["config"]["global_batch"] == WORLD * B
    assert d["bit_exact_all_ranks"] is True
    pr = sorted(d["per_rank"], key=lambda x: x["rank"])
    assert [p["rank"] for p in pr] == list(range(WORLD))
    assert all(p["bit_exact"] is True for p in pr)
    blocks = [set(range(p["seed0"], p["seedN"] + 1)) for p in pr]
    assert all(len(b) == B for b in blocks)
    assert len(set().union(*blocks)) == WORLD * B  # disjoint
    tmax = max(p["elapsed_s"] for p in pr)
    assert d["value"] == pytest.approx(WORLD * B * STEPS / tmax, rel=1e-6)

    import pf_layouts as PL
    import pyoracle as O
    lay = PL.config_layout("C2")
    tiles, total = O.make_tiles(lay)
    positions = set()
    for p in pr:
        z = np.load(dump / f"rank{p['rank']}.npz")
        s = p["sample"]
        assert int(z["seed"]) == s["seed"] and s["seed"] in blocks[p["rank"]]
        positions.add(s["index"])
        got = z["out"]
        assert hashlib.sha256(got.tobytes()).hexdigest() == s["sha256"]
        data = O.warp_depth(z["gt"], tiles, total, O.responses(z["resp"]))
        ref, _ = O.merge(z["emap"], tiles, data, 2048, PL.ZENITH_RANGE)
        bad = int((got != ref).sum())
        assert bad == 0, f"rank {p['rank']} panorama {s['seed']}: {bad} pixels differ from the oracle"
    assert len(positions) == WORLD  # a different position of the block on every rank
