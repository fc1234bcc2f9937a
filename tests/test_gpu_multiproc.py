"""The multi-process paths of bench.py on the one GPU of the test box: two
ranks launched by torch.distributed.run, both on cuda:0, talking over gloo with host-staged
tensors (RCCL refuses two ranks on one device; on a node every rank has its own GPU and the
same code paths run over RCCL).  Readiness only -- the driver's 8-GPU node measures scaling.

* C5 (--mode c5 --c5-shard rows): tiles and sweep row bands sharded over the 2 ranks, the
  partial target rows each band reads sent by the rank that owns the tiles (a sparse
  reduce-scatter), halo rows exchanged before every pass, the previous level's halo rows before
  each level, the u16 rows gathered to rank 0; rank 0 then fuses the same panorama alone (every
  tile warped and registered on its GPU) and the sharded u16 must equal it bit for bit
  (bench.py's bit_exact_vs_one_gpu).
* Batch (--mode batch, config C4's shape at a small batch): each rank its own contiguous seed
  block, disjoint; the line's value is the whole job over the MAX of the ranks' times; rank 0's
  fused batch equals a fresh one-process fusion of the same panoramas.
The launcher runs as a child process started before this test touches the GPU itself."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _launch(args, timeout=600):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "2",
           "--backend", "gloo", "--same-device", "--no-cpu-baseline", "--no-extra-configs"] + args
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]  # rank 0 prints the one line
    return json.loads(lines[0])


def test_c5_row_sharded_two_processes():
    d = _launch(["--mode", "c5", "--c5-shard", "rows", "--steps", "1", "--warmup", "0"])
    assert d["n_gpus"] == 2 and d["backend"] == "gloo"
    assert d["bit_exact_vs_one_gpu"] is True
    assert d["nonzero_px"] > 0


def test_batch_mode_two_processes():
    B, steps = 4, 2
    d = _launch(["--mode", "batch", "--batch", str(B), "--steps", str(steps), "--warmup", "1",
                 "--prof-steps", "1"])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * B
    assert d["bit_exact_vs_one_process"] is True
    pr = sorted(d["per_rank"], key=lambda x: x["rank"])
    assert [p["rank"] for p in pr] == [0, 1]
    blocks = [set(range(p["seed0"], p["seedN"] + 1)) for p in pr]
    assert all(len(b) == B for b in blocks) and not (blocks[0] & blocks[1])
    # whole-job value over the slowest rank's time
    tmax = max(p["elapsed_s"] for p in pr)
    assert d["value"] == pytest.approx(2 * B * steps / tmax, rel=1e-6)


def _direct(args, timeout=600):
    """bench.py run directly, as the driver runs `python3 bench.py --gpus N` (no torchrun)."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    return subprocess.run([sys.executable, "bench.py"] + args, cwd=ROOT, capture_output=True,
                          text=True, timeout=timeout, env=env)


def test_bench_gpus2_self_launch_same_device():
    """`bench.py --gpus 2` without torchrun launches two ranks itself."""
    B = 4
    r = _direct(["--gpus", "2", "--same-device", "--backend", "gloo", "--batch", str(B),
                 "--steps", "2", "--warmup", "1", "--prof-steps", "1", "--no-cpu-baseline",
                 "--no-extra-configs"])
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["global_batch"] == 2 * B
    assert d["bit_exact_vs_one_process"] is True
    pr = sorted(d["per_rank"], key=lambda x: x["rank"])
    blocks = [set(range(p["seed0"], p["seedN"] + 1)) for p in pr]
    assert all(len(b) == B for b in blocks) and not (blocks[0] & blocks[1])


def test_bench_gpus_more_than_visible_refused():
    import torch
    n = torch.cuda.device_count()  # counting devices does not initialise HIP
    r = _direct(["--gpus", str(n + 1), "--steps", "1", "--warmup", "0", "--batch", "2",
                 "--no-cpu-baseline"], timeout=300)
    assert r.returncode != 0
    assert f"needs {n + 1} GPUs" in r.stderr and not r.stdout.strip()
