"""The RCCL path of bench.py on the one GPU of the test box.

Every multi-process GPU run so far used gloo with host-staged tensors (several ranks on one
device).  Here bench.py runs under torch.distributed.run at world 1 with the default backend:
init_dist creates the process group with `init_process_group("nccl", device_id=cuda:0)` -- the
call every rank of the driver's 8-GPU runs makes -- and comm_check drives each TorchComm
collective of the sharded C5 flow on device tensors with stage_host=False (the RCCL branch):
all_reduce_sum, agree on the device, the int16 broadcast as bytes.  (The ring exchange needs
two ranks on two GPUs; its device branch is pinned on the CPU in tests/test_comm.py.)"""
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


def _launch(args, timeout=400):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), "bench.py", "--gpus", "1",
           "--no-cpu-baseline", "--no-extra-configs"] + args
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    r = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=timeout, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


def _check(cc):
    assert cc is not None, "no process group: init_dist did not run under the launcher"
    assert cc["backend"] == "nccl" and cc["stage_host"] is False and cc["world"] == 1
    assert cc["all_reduce_sum"] and cc["agree"] and cc["broadcast_i16"] and cc["ok"]


def test_batch_mode_nccl_world1():
    d = _launch(["--batch", "4", "--steps", "2", "--warmup", "1", "--prof-steps", "1"])
    assert d["n_gpus"] == 1 and d["bit_exact_vs_one_process"] is True
    _check(d["comm_check"])


def test_c5_mode_nccl_world1():
    d = _launch(["--mode", "c5", "--steps", "1", "--warmup", "0"])
    assert d["n_gpus"] == 1 and d["bit_exact_vs_one_gpu"] is True
    _check(d["comm_check"])
