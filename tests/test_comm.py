"""pf_dist.TorchComm's two branches, on the CPU.

The multi-GPU runs use TorchComm(stage_host=False): RCCL moves the device tensors themselves.
The gloo rehearsals on one GPU use stage_host=True: every collective runs on host copies.  No
8-GPU node has run the first branch yet, so it is pinned here with a recording stand-in for
torch.distributed and a stand-in for a device tensor:

  * stage_host=False: the exact tensor objects go into all_reduce / reduce / isend / irecv /
    broadcast, un-copied (RCCL takes device memory);
  * stage_host=True: a device tensor travels as its host copy and the result is copied back;
  * agree() allocates its tensors on the given device (RCCL cannot take host tensors), on the
    host when staging;
  * an int16 broadcast (the u16 result) travels as uint8 bytes;
  * auto_rep_levels with a comm: every rank takes rank 0's choice even when a rank's own plans
    differ (gloo world 2, a PF_J*-style override on rank 1 only).

The same collectives run on real device tensors over RCCL in tests/test_gpu_rccl.py."""
import os
import socket

import pytest

torch = pytest.importorskip("torch")
import torch.distributed as tdist  # noqa: E402
import torch.multiprocessing as mp  # noqa: E402

import pf_dist  # noqa: E402


class FakeDevice:
    type = "cuda"
    index = 0

    def __repr__(self):
        return "cuda:0"


class DevTensor:
    """Just enough of a device tensor for TorchComm: .device, .cpu(), .copy_, .dtype, .view."""

    def __init__(self, host):
        self.host = host
        self.device = FakeDevice()
        self.dtype = host.dtype
        self.copied_from = []

    def cpu(self):
        return self.host.clone()

    def copy_(self, h):
        self.copied_from.append(h)
        self.host.copy_(h)
        return self

    def view(self, dtype):
        return DevTensor(self.host.view(dtype))

    def numel(self):
        return self.host.numel()


class Req:
    def wait(self):
        return True


class RecordingDist:
    """torch.distributed stand-in: records (op, tensor object) and does world-1 arithmetic."""

    class ReduceOp:
        SUM = "sum"
        MAX = "max"

    def __init__(self):
        self.calls = []

    def all_reduce(self, t, op=None, group=None):
        self.calls.append(("all_reduce", t))

    def reduce(self, t, dst=0, op=None, group=None):
        self.calls.append(("reduce", t))

    def broadcast(self, t, src=0, group=None):
        self.calls.append(("broadcast", t))

    def isend(self, t, peer, group=None):
        self.calls.append(("isend", t))

    def irecv(self, t, peer, group=None):
        self.calls.append(("irecv", t))

    class P2POp:
        def __init__(self, fn, t, peer, group=None):
            self.fn, self.t, self.peer = fn, t, peer

    def batch_isend_irecv(self, ops):
        for o in ops:
            o.fn(o.t, o.peer)
        return [Req() for _ in ops]


def test_device_tensors_go_unstaged_into_rccl_calls():
    d = RecordingDist()
    comm = pf_dist.TorchComm(d, stage_host=False)
    a, b = DevTensor(torch.ones(8)), DevTensor(torch.ones(8))
    s, r = DevTensor(torch.arange(4.0)), DevTensor(torch.zeros(4))
    comm.all_reduce_sum(a)
    comm.reduce_sum(b, 0)
    comm.exchange([(1, s)], [(1, r)])
    got = {op: t for op, t in d.calls}
    assert got["all_reduce"] is a and got["reduce"] is b
    assert got["isend"] is s and got["irecv"] is r
    # nothing was copied back: the collective wrote the device tensor itself
    assert not a.copied_from and not b.copied_from and not r.copied_from


def test_host_staging_copies_device_tensors_both_ways():
    d = RecordingDist()
    comm = pf_dist.TorchComm(d, stage_host=True)
    a = DevTensor(torch.ones(8))
    r = DevTensor(torch.zeros(4))
    comm.all_reduce_sum(a)
    comm.exchange([], [(1, r)])
    ops = dict(d.calls)
    assert isinstance(ops["all_reduce"], torch.Tensor) and ops["all_reduce"] is not a.host
    assert isinstance(ops["irecv"], torch.Tensor)
    assert len(a.copied_from) == 1 and a.copied_from[0] is ops["all_reduce"]
    assert len(r.copied_from) == 1 and r.copied_from[0] is ops["irecv"]


def test_int16_broadcast_travels_as_bytes():
    for stage in (False, True):
        d = RecordingDist()
        comm = pf_dist.TorchComm(d, stage_host=stage)
        t = torch.arange(-5, 5, dtype=torch.int16)
        comm.broadcast(t, 0)
        (op, sent), = d.calls
        assert op == "broadcast" and sent.dtype == torch.uint8 and sent.numel() == 2 * t.numel()
        assert sent.data_ptr() == t.data_ptr() or stage  # a view of the same bytes (no staging)


def test_agree_allocates_on_the_given_device(monkeypatch):
    seen = []
    real_tensor, real_zeros = torch.tensor, torch.zeros

    def rec_tensor(data, dtype=None, device=None):
        seen.append(("tensor", str(device) if device is not None else None))
        return real_tensor(data, dtype=dtype)

    def rec_zeros(n, dtype=None, device=None):
        seen.append(("zeros", str(device)))
        return real_zeros(n, dtype=dtype)

    d = RecordingDist()
    monkeypatch.setattr(torch, "tensor", rec_tensor)
    monkeypatch.setattr(torch, "zeros", rec_zeros)
    out = pf_dist.TorchComm(d, stage_host=False).agree([10, 7, 10], 0, "cuda:3")
    assert out == [10, 7, 10]
    # the length and the values are broadcast from tensors made on cuda:3
    assert ("tensor", "cuda:3") in seen and ("zeros", "cuda:3") in seen
    assert [op for op, _ in d.calls] == ["broadcast", "broadcast"]
    seen.clear()
    pf_dist.TorchComm(d, stage_host=True).agree([1], 0, "cuda:3")
    assert ("tensor", "cpu") in seen and ("zeros", "cpu") in seen


class PlanBackend:
    """dims/plan stand-in: rank 1's plan is deeper (a per-process override), which alone would
    change its auto_rep_levels answer."""

    def __init__(self, rank):
        self.rank = rank
        self.device = "cpu"

    def dims(self, lv):
        h1 = [60, 120, 240, 480][lv]
        return 64 << lv, 2 * h1, 1, h1

    def plan(self, lv, world):
        return [10] * 5 if self.rank == 0 else [2] * 20


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rep_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    tdist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        be = PlanBackend(rank)
        own = pf_dist.auto_rep_levels(be, 4, world)
        agreed = pf_dist.auto_rep_levels(be, 4, world, comm=pf_dist.TorchComm(tdist))
        q.put((rank, own, agreed))
    finally:
        tdist.destroy_process_group()


def test_auto_rep_levels_agreed_over_ranks_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rep_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
        assert p.exitcode == 0
    res = sorted(q.get() for _ in range(2))
    (_, own0, agreed0), (_, own1, agreed1) = res
    assert own0 != own1  # the ranks' own plans disagree ...
    assert agreed0 == agreed1 == own0  # ... and both take rank 0's choice
