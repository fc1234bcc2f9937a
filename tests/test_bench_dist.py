"""bench.py's batch-sharded launcher (configs C3/C4) at world size 2, on the CPU.

The driver runs `python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N` on an
8-GPU node; here the same launcher, seeding and timing code runs with bench.py's --stand-in step
over gloo (a rank-dependent sleep instead of the GPU step).  Checked: every rank owns a disjoint
contiguous seed block (and the block the GPU path generates its panoramas from), the reported
elapsed time is the MAX over ranks of each rank's barrier-bracketed time, and value /
global_batch count the whole job (B x world panoramas per step).
"""
import json
import os
import socket
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_bench_batch_launcher_world2():
    B, steps, world = 4, 3, 2
    env = dict(os.environ)
    env.pop("CUDA_VISIBLE_DEVICES", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={world}", "--master-addr", "127.0.0.1",
           "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"),
           "--gpus", str(world), "--steps", str(steps), "--warmup", "1", "--batch", str(B),
           "--stand-in"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, cwd=ROOT, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 prints one JSON line
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["steps"] == steps
    assert d["config"]["global_batch"] == B * world
    per = sorted(d["per_rank"], key=lambda x: x["rank"])
    assert [p["rank"] for p in per] == list(range(world))
    sys.path.insert(0, ROOT)
    import bench
    seen = set()
    for p in per:
        assert p["seeds"] == bench.rank_seeds(B, p["rank"])
        assert len(p["seeds"]) == B
        assert not (seen & set(p["seeds"]))
        seen |= set(p["seeds"])
    assert d["elapsed"] == max(p["elapsed"] for p in per)
    assert abs(d["value"] - B * world * steps / d["elapsed"]) < 1e-9 * d["value"]
    # rank 1's stand-in step is the slower one: the MAX is at least its own sleeping time
    assert d["elapsed"] >= steps * 0.02


def _run_bench(args, env_extra=None, timeout=240):
    env = dict(os.environ)
    env.pop("CUDA_VISIBLE_DEVICES", None)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env.update(env_extra or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args,
                          capture_output=True, text=True, timeout=timeout, cwd=ROOT, env=env)


def test_bench_self_launches_n_ranks():
    """`bench.py --gpus N` run directly (no torchrun, no WORLD_SIZE) starts the
    N ranks itself and prints one N-rank line."""
    B, world = 3, 3
    r = _run_bench(["--gpus", str(world), "--steps", "2", "--warmup", "0", "--batch", str(B),
                    "--stand-in"])
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == world and d["config"]["global_batch"] == B * world
    per = sorted(d["per_rank"], key=lambda x: x["rank"])
    assert [p["rank"] for p in per] == list(range(world))
    seeds = [s for p in per for s in p["seeds"]]
    assert len(seeds) == len(set(seeds)) == B * world


def test_bench_refuses_more_gpus_than_visible():
    """`bench.py --gpus 2` where fewer than 2 devices are visible (this CPU host: none) exits
    non-zero with a message instead of printing a 1-GPU line."""
    r = _run_bench(["--gpus", "2", "--steps", "1", "--warmup", "0", "--batch", "2"])
    assert r.returncode != 0
    assert "needs 2 GPUs" in r.stderr and not r.stdout.strip()


def test_bench_refuses_gpus_world_mismatch():
    r = _run_bench(["--gpus", "4", "--stand-in", "--steps", "1", "--warmup", "0"],
                   env_extra={"WORLD_SIZE": "2", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def test_bench_refuses_same_device_nccl():
    r = _run_bench(["--gpus", "2", "--same-device", "--steps", "1", "--warmup", "0"])
    assert r.returncode != 0 and "--backend gloo" in r.stderr
