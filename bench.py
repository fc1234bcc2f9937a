#!/usr/bin/env python3
"""Throughput benchmark of the panorama-depth fusion path (BASELINE.json metric).

One step = one batch of synthetic 2048x1024 panoramas through the whole hot path on the GPU:
E->P warp of the ground-truth panorama into 20 tiles of 512^2 (plus the synthetic depth-net
response), per-tile cubic registration against the 512x256 baseline (MergeDepthMaps' SolveDepthToDepth
loop), 3-level Laplacian fusion with 200/100/50 damped Jacobi sweeps, u16 quantisation.  Inputs are
resident in HBM before the timed region.  Per GPU the workload is BASELINE config C3 (batch 64);
launched on 8 GPUs it is C4 (512 panoramas, 64 per GPU, no collective on the data path).

    python bench.py [--gpus N --steps K --warmup W --batch B]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

Run directly with --gpus N > 1 it launches the N ranks itself (torch.distributed.run as a child,
started before any GPU call; launch_ranks), so both forms print the same N-rank line.

Rank 0 prints one JSON line.  `roofline` is for the dominant kernel (the Jacobi sweep) against
its real roof, VALU issue: algorithmic FLOP (14 per pixel-update) per launch over its average
hipEvent-measured launch time; `roofline_hbm` puts the same kernel's measured PMC traffic on the
HBM roof and `effective_hbm` keeps SURVEY.md 8d's 12 B/update as an effective rate.
`cpu_baseline` is the CPU oracle (the C restatement of Depth.cpp, OpenMP) running the same
per-panorama pipeline on every usable host core and on one core, over a bounded sample.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "wacv2023-high-resolution-depth-estimation-for-panoramas-through-"
                         "perspective-map-registrations_amd")
sys.path.insert(0, PKG)

METRIC = "panoramas/sec (whole node), 2048×1024 × 20 tiles, at 1/2/4/8 MI355X"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
VALU_PEAK_TF = 157.3   # MI355X_MICROARCH.md: peak FP32 vector (packed FMA), spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=64, help="panoramas per GPU per step")
    ap.add_argument("--c5-shard", choices=("rows", "tiles"), default="rows",
                    help="c5 mode: rows = tiles AND sweep row bands sharded over the ranks "
                         "(pf_dist.fuse_row_sharded, halo exchange per pass); tiles = tiles "
                         "sharded, every sweep on rank 0 (pf_dist.fuse_tile_sharded)")
    ap.add_argument("--c5-rep", type=int, default=-1,
                    help="c5 rows mode: the coarsest levels replicated on every rank instead of "
                         "row-sharded (pf_dist.fuse_row_sharded rep_levels); -1 = auto "
                         "(pf_dist.auto_rep_levels)")
    ap.add_argument("--c5-side", type=int, default=1,
                    help="c5 rows mode: 1 = each rank's row-sharded levels' tile sums, their "
                         "exchange and adds on a second stream beside the replicated levels' "
                         "sweeps (HipRowShardBackend.enable_side); 0 = one stream")
    ap.add_argument("--mode", choices=("batch", "c5"), default="batch",
                    help="batch: configs C3/C4 (the headline metric); c5: one 8192x4096 "
                         "panorama, tiles sharded over the ranks")
    ap.add_argument("--cpu-seconds", type=float, default=15.0)
    ap.add_argument("--prof-steps", type=int, default=5,
                    help="extra untimed steps with the per-stage hipEvent timers on (roofline)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-extra-configs", action="store_true",
                    help="skip the C2 batch-1 latency and the one-GPU C5 sub-records")
    ap.add_argument("--pipeline", type=int, default=2,
                    help="0: serial steps; 1: the warp of batch k+1 (second stream) "
                         "runs while batch k is registered and fused; every step still warps, "
                         "registers and fuses one whole batch; N >= 2: N fusion lanes (own "
                         "context, stream and buffers), batch k on lane k %% N")
    ap.add_argument("--backend", choices=("nccl", "gloo"), default="nccl",
                    help="torch.distributed backend for N > 1: nccl (= RCCL over xGMI, the "
                         "default) or gloo with host-staged tensors (several ranks sharing one "
                         "GPU: RCCL refuses a duplicate device)")
    ap.add_argument("--same-device", action="store_true",
                    help="every rank on cuda:0 (multi-process rehearsal on a one-GPU box; "
                         "use with --backend gloo)")
    ap.add_argument("--sample-dump", default=None, metavar="DIR",
                    help="every rank writes DIR/rank<r>.npz: the inputs (ground truth, baseline, "
                         "depth-net responses) and the fused u16 of one sampled panorama of its "
                         "batch, for an oracle check outside the bench (tests/test_gpu_c4.py)")
    ap.add_argument("--stand-in", action="store_true",
                    help="test hook (tests/test_bench_dist.py): the launcher, seeding and timing "
                         "path with a CPU stand-in step over gloo; no GPU is touched")
    return ap.parse_args()


def host_cpus():
    """CPUs this process may run on: the affinity mask, capped by a cgroup-v2 CPU quota when
    one is set (the GPU box shares its host, and os.cpu_count() reports the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            n = min(n, max(1, int(-(-int(quota) // int(period)))))
    except (OSError, ValueError):
        pass
    return max(1, n)


def _oracle_rate(O, PL, pf_synth, threads, seconds, max_panos, cfg="C2"):
    """Panoramas/s of the oracle pipeline (warp + register + fuse) at `threads` OpenMP threads,
    over at least one panorama and until `seconds` of work or `max_panos` panoramas."""
    O.set_threads(threads)
    lay = PL.config_layout(cfg)
    out_w, ew = PL.CONFIGS[cfg]
    tiles, total = O.make_tiles(lay)
    done, t_work = 0, 0.0
    while done < 1 or (t_work < seconds and done < max_panos):
        seeds = pf_synth.seeds_for(1, 90000 + done)
        gt = pf_synth.scene_depth(seeds, out_w, out_w // 2)[0].numpy()
        emap = pf_synth.baseline_emap(seeds, ew, ew // 2)[0].numpy()
        resp = O.responses(pf_synth.responses(seeds, lay.ntiles))
        t0 = time.perf_counter()
        data = O.warp_depth(gt, tiles, total, resp)
        O.merge(emap, tiles, data, out_w, PL.ZENITH_RANGE)
        t_work += time.perf_counter() - t0
        done += 1
    return done / t_work, done, t_work


def cpu_baseline(seconds):
    """The oracle (C/OpenMP restatement of Depth.cpp, kind=port) on this host's cores: the same
    per-panorama pipeline as the GPU step (warp + registration + 3-level fusion), timed on every
    CPU this process may use ("all host cores, nproc reported") and on 1 core."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pf_layouts as PL
    import pf_synth
    import pyoracle as O
    threads = host_cpus()
    v, done, t_work = _oracle_rate(O, PL, pf_synth, threads, seconds, 64)
    v1, done1, t1 = _oracle_rate(O, PL, pf_synth, 1, min(seconds, 5.0), 8)
    # BASELINE config C1 (the reference's own CPU case, Main.cpp mode 0: one 512x256 panorama,
    # 6 tiles of 256^2, 128x64 baseline), the same pipeline, a few seconds each
    c1, n1, s1 = _oracle_rate(O, PL, pf_synth, threads, min(seconds, 3.0), 256, "C1")
    c11, n11, s11 = _oracle_rate(O, PL, pf_synth, 1, min(seconds, 3.0), 64, "C1")
    return {"value": v, "unit": "panoramas/s", "cores": threads, "kind": "port",
            "nproc": os.cpu_count(), "cpus_usable": threads,
            "value_1core": v1,
            "c1": {"value": c1, "value_1core": c11, "unit": "panoramas/s",
                   "sample": f"C1 (512x256, 6 tiles of 256^2): {n1} panoramas in {s1:.1f} s on "
                             f"{threads} threads, {n11} in {s11:.1f} s on 1"},
            "sample": f"{done} panoramas of C2 (2048x1024, 20 tiles of 512^2): warp + registration"
                      f" + 3-level fusion, {t_work:.1f} s of work, OpenMP {threads} threads "
                      f"(every CPU usable by this process; nproc={os.cpu_count()}); 1 core: "
                      f"{done1} panoramas in {t1:.1f} s"}


def pmc_traffic(family):
    """HBM bytes per launch of a kernel family from the committed rocprofv3 PMC passes
    (tools/pmc_round.sh -> tools/pmc_traffic.py -> profiles/pmc_traffic.json), or None."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            rec = json.load(f).get(family)
        return float(rec["traffic_B"]) if rec else None
    except (OSError, ValueError, KeyError):
        return None


def _pmc_record(family):
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as f:
            return json.load(f).get(family)
    except (OSError, ValueError):
        return None


def jacobi_traffic_per_step(launches_per_step):
    """PMC HBM bytes of one step's Jacobi stage: the streaming passes (k_jlag) plus, where the
    resident level kernel ran, its one launch per fusion (k_jres).  The PMC run's k_jres dispatch
    count is its fusion count, which scales k_jlag's total to one step."""
    rl, rr = _pmc_record("pf::k_jlag"), _pmc_record("pf::k_jres")
    try:
        if rr and rl:
            return (float(rl["traffic_B"]) * float(rl["dispatches"]) / float(rr["dispatches"])
                    + float(rr["traffic_B"]))
        if rl:
            return float(rl["traffic_B"]) * launches_per_step
    except (KeyError, ValueError, ZeroDivisionError):
        pass
    return None


def _metrics_traffic():
    """PMC HBM bytes of one pf_error_metrics call (align_way 1): 3 k_med_hist + k_err_sums."""
    h, e = pmc_traffic("pf::k_med_hist"), pmc_traffic("pf::k_err_sums")
    return 3 * h + e if h is not None and e is not None else None


def c5_measure(args, rank, world, local, dev, steps, warmup):
    """BASELINE config C5: one 8192x4096 panorama, 80 tiles of 1024^2 sharded over the ranks.
    Each rank warps and registers its own tiles (a sub-layout context writing into its slice of
    the full tile block).  --c5-shard rows (pf_dist.fuse_row_sharded): per level each rank sums
    its tiles' targets on the rows it sweeps and the rows its neighbours read, sends those rows
    (a sparse reduce-scatter by band rows), sweeps its row band with a halo exchange per pass,
    and the u16 rows are gathered to rank 0; --c5-shard tiles (pf_dist.fuse_tile_sharded): the
    (sum L, n) grids are reduced to rank 0, which sweeps the whole level.
    One step = one panorama end to end; value = panoramas/s of the whole job."""
    import torch
    import torch.distributed as dist

    import panofuse
    import pf_dist
    import pf_layouts as PL
    import pf_synth

    out_w, ew = PL.CONFIGS["C5"]
    lay = PL.config_layout("C5")
    zr = PL.ZENITH_RANGE
    t0, t1 = pf_dist.shard_range(lay.ntiles, rank, world)
    sub = PL.Layout(f"C5[{t0}:{t1}]", lay.fovs[t0:t1], lay.ranges[t0:t1], lay.tile_w[t0:t1],
                    lay.tile_h[t0:t1])
    seeds = pf_synth.seeds_for(1, 20261015)  # every rank generates the same panorama
    gt = pf_synth.scene_depth(seeds, out_w, out_w // 2, dev).contiguous()
    emap = pf_synth.baseline_emap(seeds, ew, ew // 2, dev).contiguous()
    resp_all = pf_synth.responses(seeds, lay.ntiles)
    fz = panofuse.Fuser(local)
    fz.set_tiles(lay)
    fs = panofuse.Fuser(local) if t1 > t0 else None
    if fs is not None:
        fs.set_tiles(sub)
        resp = panofuse.make_responses(resp_all[t0:t1], dev)
    tiles = torch.zeros((1, fz.tile_elems), dtype=torch.float32, device=dev)
    off0 = int(sum(int(lay.tile_w[i]) * int(lay.tile_h[i]) for i in range(t0)))
    off1 = off0 + (fs.tile_elems if fs is not None else 0)
    coeffs = torch.zeros((lay.ntiles, 4), dtype=torch.float32, device=dev)
    out = torch.empty((out_w // 2, out_w), dtype=torch.int16, device=dev)
    nlevels = panofuse.level_info(out_w, out_w // 2, zr, 0)[5]

    logs = []
    be0 = pf_dist.HipRowShardBackend(fz, emap, tiles, coeffs, out_w, zr, out.view(-1))
    fside = None
    if args.c5_side:  # the row-sharded levels' tile sums beside the replicated levels' sweeps
        fside = panofuse.Fuser(local, stream=torch.cuda.Stream(dev))
        fside.set_tiles(lay)
        be0.enable_side(fside)
    comm = pf_dist.TorchComm(dist, stage_host=args.backend == "gloo") if world > 1 else None
    # one choice for all ranks (rank 0's): the plans behind it depend on per-process state
    rep = args.c5_rep if args.c5_rep >= 0 else pf_dist.auto_rep_levels(be0, nlevels, world,
                                                                        comm=comm)

    def step():
        if fs is not None:
            mine = tiles[:, off0:off1]
            fs.warp_depth(gt, mine, resp)
            fs.register(emap, mine, zr, degree=3, apply=False, coeffs=coeffs[t0:t1][None])
        if args.c5_shard == "rows":  # be0 keeps the per-level geometry across panoramas
            logs.append(pf_dist.ExchangeLog())
            pf_dist.fuse_row_sharded(be0, nlevels, lay.ntiles, rank, world, comm, logs[-1],
                                     rep_levels=rep)
        else:
            be = pf_dist.HipTileShardBackend(fz, emap, tiles, coeffs, out_w, zr, out)
            pf_dist.fuse_tile_sharded(be, nlevels, lay.ntiles, rank, world, comm)

    for _ in range(warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    for _ in range(steps):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - ts
    fz.synchronize()  # PF_ETIMEOUT if any fusion's resident kernel timed out
    mine_s = elapsed
    if world > 1:
        t = torch.tensor([elapsed], dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    bit_exact = None
    if rank == 0:
        # after the timed steps: the same panorama fused on this GPU alone (every tile warped
        # and registered here, pf_merge) must equal the sharded result bit for bit
        full = torch.zeros_like(tiles)
        fz.warp_depth(gt, full, panofuse.make_responses(resp_all, dev))
        ref = torch.empty_like(out)
        fz.merge(emap, full, ref[None], zr, coeffs=torch.zeros_like(coeffs)[None])
        torch.cuda.synchronize()
        bit_exact = bool(torch.equal(ref, out))
    one_call = None
    if world == 1:
        # the same panorama through the library's one-call path (pf_warp_depth + pf_merge on one
        # context, no per-level host orchestration): hipEvents, median of 5
        rall = panofuse.make_responses(resp_all, dev)
        full = torch.zeros_like(tiles)
        ref = torch.empty_like(out)
        cz = torch.zeros_like(coeffs)[None]
        ts_ = []
        for i in range(7):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fz.warp_depth(gt, full, rall)
            fz.merge(emap, full, ref[None], zr, coeffs=cz)
            e1.record()
            torch.cuda.synchronize()
            if i >= 2:
                ts_.append(e0.elapsed_time(e1))
        one_call = sorted(ts_)[len(ts_) // 2]
    model8 = None
    if world == 1 and args.c5_shard == "rows":
        model8 = c5_rehearsal(fz, lay, gt, emap, resp_all, coeffs, tiles, out, out_w, zr,
                              nlevels, dev, local, side=fside)
    nz = int((out != 0).sum().item())
    sent = logs[-1].sent if logs else None  # this rank's bytes of the last step, by kind
    if world > 1 and sent is not None:
        per = [None] * world
        dist.all_gather_object(per, sent)
        sent = per
    return {"value": steps / elapsed, "elapsed": elapsed, "mine_s": mine_s,
            "bit_exact": bit_exact, "nonzero_px": nz, "one_call_ms": one_call,
            "bytes_sent_per_rank": sent, "model_8_ranks": model8, "rep_levels": rep}


# C5 over 8 GPUs, predicted from one GPU.  The exchanges themselves
# cannot run here (one GPU: RCCL refuses two ranks on a device), so they enter as a stated model:
# an exchange round costs XCHG_LAT_US of latency on the critical path (RCCL point-to-point over
# xGMI, small messages) plus its bytes at XCHG_GBS (one xGMI link, ~153 GB/s peak, taken at a
# third).  Each rank's compute is measured: the sharded flow of rank r of 8 run alone on this GPU
# with a communicator that moves nothing (pf_dist.NullComm), its own tiles warped and registered
# first (hipEvents).  Predicted = max over ranks (compute) + rounds x latency + max bytes / rate.
LANE_SHARE = 1.0  # the chip share the fusion lanes plan for (set by lane_steps)
XCHG_LAT_US = 20.0
XCHG_GBS = 50.0


def c5_rehearsal(fz, lay, gt, emap, resp_all, coeffs, tiles, out, out_w, zr, nlevels, dev,
                 local, world=8, side=None):
    import torch

    import panofuse
    import pf_dist
    import pf_layouts as PL
    be = pf_dist.HipRowShardBackend(fz, emap, tiles, coeffs, out_w, zr, out.view(-1))
    if side is not None:
        be.enable_side(side)
    dims = [be.dims(lv) for lv in range(nlevels)]
    ext = [[be.tile_rows(lv, *pf_dist.shard_range(lay.ntiles, r, world)) for r in range(world)]
           for lv in range(nlevels)]
    mc = [be.multicover_count(lv) for lv in range(nlevels)]
    subs = []
    for r in range(world):  # each rank's tile context, maps built before the timing
        a, b = pf_dist.shard_range(lay.ntiles, r, world)
        f = panofuse.Fuser(local)
        f.set_tiles(PL.Layout(f"C5[{a}:{b}]", lay.fovs[a:b], lay.ranges[a:b], lay.tile_w[a:b],
                              lay.tile_h[a:b]))
        off = int(sum(int(lay.tile_w[i]) * int(lay.tile_h[i]) for i in range(a)))
        subs.append((f, a, b, off, panofuse.make_responses(resp_all[a:b], dev)))
    res = {}
    for rep in range(nlevels):
        plans = [be.plan(lv, 1 if lv < rep else world) for lv in range(nlevels)]
        try:
            per = pf_dist.exchange_model(dims, plans, ext, world, mc, rep_levels=rep)
        except ValueError:
            continue
        times, rounds = [], 0
        for r, (f, a, b, off, resp) in enumerate(subs):
            mine = tiles[:, off:off + f.tile_elems]
            log = pf_dist.ExchangeLog()
            ts = []
            for it in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                f.warp_depth(gt, mine, resp)
                f.register(emap, mine, zr, degree=3, apply=False, coeffs=coeffs[a:b][None])
                log = pf_dist.ExchangeLog()
                try:
                    pf_dist.fuse_row_sharded(be, nlevels, lay.ntiles, r, world,
                                             pf_dist.NullComm(), log, rep_levels=rep)
                except ValueError:
                    ts = None
                    break
                e1.record()
                torch.cuda.synchronize()
                if it:
                    ts.append(e0.elapsed_time(e1))
            if ts is None:
                times = None
                break
            times.append(min(ts))
            rounds = max(rounds, log.rounds)
        if times is None:
            continue
        tot = [sum(d.values()) for d in per]
        pred = max(times) + rounds * XCHG_LAT_US * 1e-3 + max(tot) / (XCHG_GBS * 1e9) * 1e3
        res[f"rep{rep}"] = {"rep_levels": rep, "plans": plans, "compute_ms_per_rank": times,
                            "rounds": rounds, "bytes_per_rank": per, "max_rank_bytes": max(tot),
                            "total_bytes": sum(tot), "predicted_ms": pred}
    for f, *_ in subs:
        f.close()
    best = min(res.values(), key=lambda d: d["predicted_ms"]) if res else None
    return {"world": world, "assumed_round_latency_us": XCHG_LAT_US,
            "assumed_link_GBps": XCHG_GBS, "by_rep_levels": res,
            "best": best and {k: best[k] for k in ("rep_levels", "predicted_ms",
                                                   "max_rank_bytes", "total_bytes", "rounds")}}


def run_c5(args, rank, world, local, dev, dist_on=False, comm_res=None):
    """bench.py --mode c5: the C5 line (c5_measure) on `world` ranks."""
    import torch.distributed as dist
    r = c5_measure(args, rank, world, local, dev, args.steps, args.warmup)
    elapsed, mine_s, bit_exact, nz = r["elapsed"], r["mine_s"], r["bit_exact"], r["nonzero_px"]
    if rank == 0:
        print(json.dumps({
            "metric": "panoramas/sec (whole node), 8192x4096 x 80 tiles (BASELINE config C5)",
            "value": args.steps / elapsed, "unit": "panoramas/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic (box-room scene, synthetic depth-net response)",
            "config": {"workload": "C5: one 8192x4096 panorama, 80 tiles of 1024x1024 (10x8), "
                                   "2048x1024 baseline; tiles sharded over ranks, per level "
                                   + ("the partial target rows each row band reads sent by their "
                                      "tiles' rank (sparse reduce-scatter), row-band Jacobi per "
                                      "rank with a halo exchange per pass, the previous level's "
                                      "halo rows per level, u16 rows gathered to rank 0"
                                      if args.c5_shard == "rows"
                                      else "(sum L, n) reduce to rank 0 (RCCL), Jacobi on rank 0"),
                       "parallelism": f"{'row-band' if args.c5_shard == 'rows' else 'tile'}-sharded x{world}"},
            "nonzero_px": nz, "bit_exact_vs_one_gpu": bit_exact,
            "bytes_sent_per_rank": r["bytes_sent_per_rank"],
            "model_8_ranks": r["model_8_ranks"],
            "one_call_ms": r["one_call_ms"],
            "rep_levels": r["rep_levels"],
            "backend": args.backend if world > 1 else None,
            "comm_check": comm_res,
            "elapsed_rank0_s": mine_s}), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    if rank == 0 and not bit_exact:
        sys.exit("C5: the sharded result differs from the one-GPU fusion")


def c2_latency(local, dev, lay, zr, reps=7, cfg="C2"):
    """BASELINE config C2 -- one 2048x1024 panorama, 20 tiles of 512^2, one GPU -- as a latency:
    warp + registration + fusion of ONE panorama (what MergeDepthMaps times per panorama,
    Depth.cpp:792-808, 907-916), hipEvents on the context's stream around each run, after the
    layout caches exist (the facade keeps them across panoramas); median and min of `reps`."""
    import torch

    import panofuse
    import pf_synth
    import pf_layouts as PL
    ow, ew = PL.CONFIGS[cfg]
    seeds = pf_synth.seeds_for(1, 424242)
    gt = pf_synth.scene_depth(seeds, ow, ow // 2, dev).contiguous()
    emap = pf_synth.baseline_emap(seeds, ew, ew // 2, dev).contiguous()
    resp = panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), dev)
    f = panofuse.Fuser(local)
    f.set_tiles(lay)
    tiles = torch.empty((1, f.tile_elems), dtype=torch.float32, device=dev)
    out = torch.empty((1, ow // 2, ow), dtype=torch.int16, device=dev)
    coeffs = torch.empty((1, lay.ntiles, 4), dtype=torch.float32, device=dev)
    times = []
    for i in range(reps + 2):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f.warp_depth(gt, tiles, resp)
        f.merge(emap, tiles, out, zr, coeffs=coeffs)
        e1.record()
        torch.cuda.synchronize()
        if i >= 2:  # two warm runs first
            times.append(e0.elapsed_time(e1))
    f.synchronize()
    times.sort()
    what = {"C2": "C2: one 2048x1024 panorama, 20 tiles of 512^2",
            "C1": "C1: one 512x256 panorama, 6 tiles of 256^2 (the reference's CPU case)"}[cfg]
    return {"median_ms": times[len(times) // 2], "min_ms": times[0], "reps": reps,
            "workload": what + ": warp + registration + 3-level fusion + u16, hipEvents around "
                               "each run (median)"}


def rgb_warp_measure(local, dev, lay, B, reps=7):
    """The E->P RGB warp (a18: SaveCubeMap's tile render, Main.cpp:242-326) at C3's shape: a
    batch of B u8 RGB 2048x1024 panoramas into the 20 u8 RGB tiles of 512^2 each (pf_warp_rgb,
    k_warp_rgb_box), hipEvents on the context's stream around each launch, median of `reps`
    after a first call that builds the layout's taps and patch boxes.  Algorithmic bytes per
    launch = B x (panorama read 3*pw*ph + tile write 3*sum(tw*th))."""
    import torch

    import panofuse
    pw, ph = 2048, 1024
    g = torch.Generator(device=dev).manual_seed(4242)
    pano = torch.randint(0, 256, (B, ph, pw, 3), dtype=torch.uint8, device=dev, generator=g)
    n = sum(int(lay.tile_w[i]) * int(lay.tile_h[i]) * 3 for i in range(lay.ntiles))
    tiles = torch.empty((B, n), dtype=torch.uint8, device=dev)
    f = panofuse.Fuser(local)
    f.set_tiles(lay)
    f.warp_rgb(pano, tiles)
    torch.cuda.synchronize()
    times = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        f.warp_rgb(pano, tiles)
        e1.record()
        torch.cuda.synchronize()
        times.append(e0.elapsed_time(e1))
    f.close()
    times.sort()
    ms = times[len(times) // 2]
    nbytes = B * (3 * pw * ph + n)
    ach = nbytes / (ms * 1e-3) / 1e9
    del pano, tiles
    return {"bound": "hbm", "achieved": ach, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": ach / HBM_PEAK_GBS, "traffic": pmc_traffic("pf::k_warp_rgb_box"),
            "kernel": "k_warp_rgb_box", "avg_launch_us": ms * 1e3, "min_launch_us": times[0] * 1e3,
            "bytes_per_launch": nbytes,
            "workload": f"C3 shape: {B} u8 RGB panoramas 2048x1024 -> 20 u8 RGB tiles of 512^2 "
                        f"(pf_warp_rgb; outside the step, which warps depth)"}


def rank_seeds(batch, rank):
    """Seeds of the panoramas rank `rank` owns in the batch-sharded run (config C4): contiguous
    blocks of `batch`, disjoint across ranks (pf_dist.panorama_block)."""
    import pf_dist
    return pf_dist.panorama_block(batch, rank)


# pipelined steps: the next batch's warp waits for this level of the current fusion (-1: only for
# the fusion that last read its buffer).  Level 0 (default): the memory-bound warp runs beside
# the finer levels' streaming passes instead of contending with the resident level-0 kernel,
# which fills every CU -- measured on MI355X (recipe: tools/gpu_round.sh ab with PF_WARP_AFTER, three alternating rounds):
# 14.12-14.28k panoramas/s against 13.51-14.02k (-1) and 13.94-14.32k (1).
WARP_AFTER_LEVEL = int(os.environ.get("PF_WARP_AFTER", "0"))


def pipelined_step(fz, lay, local, dev, gt, emap, resp, tiles, out, coeffs, zr):
    """The software-pipelined bench step: step k registers and fuses the tiles warped during step
    k-1 (buffer k % 2) on the main stream while a second stream (its own context) warps batch k+1
    into the other buffer, once the fusion that last read it (step k-1) is done.  Same work per
    step as the serial one: one warp, one merge of the whole batch.  Primes buffer 0."""
    import torch

    import panofuse

    sw = torch.cuda.Stream(dev, priority=int(os.environ.get("PF_WARP_PRIO", "0")))
    fw = panofuse.Fuser(local, stream=sw)
    fw.set_tiles(lay)
    bufs = [tiles, torch.empty_like(tiles)]
    main = fz.stream  # the fusion's stream (the caller's current stream unless fz has its own)
    st = {"k": 0, "warped": None, "fused": None, "fw": fw}
    fw.warp_depth(gt, bufs[0], resp)
    st["warped"] = torch.cuda.Event()
    st["warped"].record(sw)

    def pstep():
        k = st["k"]
        cur, nxt = bufs[k % 2], bufs[(k + 1) % 2]
        main.wait_event(st["warped"])
        fz.merge(emap, cur, out, zr, coeffs=coeffs)
        fused = torch.cuda.Event()
        fused.record(main)
        if st["fused"] is not None:
            sw.wait_event(st["fused"])  # the fusion of step k-1 read nxt
        if WARP_AFTER_LEVEL >= 0:  # start the warp beside the finer levels of this fusion
            fz.stream_wait_level(WARP_AFTER_LEVEL, sw)
        fw.warp_depth(gt, nxt, resp)
        warped = torch.cuda.Event()
        warped.record(sw)
        st.update(k=k + 1, warped=warped, fused=fused)

    return pstep


def lane_steps(fz, lay, local, dev, gt, emap, resp, tiles, out, coeffs, zr, nlanes):
    """`--pipeline N` (N >= 2): N fusion lanes, each its own context on its own stream with its own
    tile / output / coefficient buffers; step k warps, registers and fuses one whole batch on lane
    k % N, so N consecutive batches are in flight at once and their kernels fill each other's
    gaps (the under-occupied level-1 passes, launch tails).  Each lane is pipelined like
    `--pipeline 1` (the warp of its next batch on a second stream).  Same work per step as the
    serial step.  Returns (step, lanes): lanes[i] = (context, tiles, out, coeffs); lane 0 uses the
    caller's context and buffers."""
    import torch

    import panofuse

    lanes = [(fz, tiles, out, coeffs)]
    for _ in range(1, nlanes):
        f = panofuse.Fuser(local, stream=torch.cuda.Stream(dev))
        f.set_tiles(lay)
        lanes.append((f, torch.empty_like(tiles), torch.empty_like(out), torch.empty_like(coeffs)))
    # Jacobi pass plans for concurrent fusions: two lanes offset by about half a step overlap
    # their Jacobi stages about half the time, so a lane's expected share of the chip is ~3/4 and
    # its levels take fewer, longer row chunks (less total work; round 6 A/B, DESIGN.md section 5:
    # levels 1 / 2 in 2 / 3 chunks instead of 3 / 4, +1.5 %).  PF_LANE_SHARE overrides (A/B runs).
    global LANE_SHARE
    share = float(os.environ.get("PF_LANE_SHARE", 1.0 - (nlanes - 1) / (2.0 * nlanes)))
    LANE_SHARE = share
    for f, *_ in lanes:
        f.set_jacobi_share(share)
    st = {"k": 0}
    # every lane is itself pipelined (bench.pipelined_step: its warps on a stream of their own,
    # its fusions on the lane's stream); PF_LANE_WARP=0 (A/B runs): warp and fusion in line
    psteps = None
    if os.environ.get("PF_LANE_WARP", "1") != "0":
        psteps = []
        for f, t, o, c in lanes:  # warps on a stream of their own, fusions on f's stream
            psteps.append(pipelined_step(f, lay, local, dev, gt, emap, resp, t, o, c, zr))

    def lstep():
        i = st["k"] % nlanes
        if psteps is not None:
            psteps[i]()
        else:
            f, t, o, c = lanes[i]
            f.warp_depth(gt, t, resp)
            f.merge(emap, t, o, zr, coeffs=c)
        st["k"] += 1

    return lstep, lanes


def timed_steps(step, sync, args, world, dist, device=None):
    """W untimed warmup steps, then EXACTLY K steps bracketed by a barrier + device sync on both
    sides; returns (elapsed seconds of this rank, elapsed MAX over ranks)."""
    for _ in range(args.warmup):
        step()
    sync()
    if world > 1:
        dist.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    sync()
    if world > 1:
        dist.barrier()
    mine = time.perf_counter() - t0
    elapsed = mine
    if world > 1:
        import torch
        on_dev = device is not None and dist.get_backend() != "gloo"
        t = torch.tensor([mine], dtype=torch.float64, device=device if on_dev else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return mine, elapsed


def init_dist(args, world, local):
    """torch.distributed for this process.  Under a launcher (WORLD_SIZE in the environment) the
    process group is created at EVERY world size -- world 1 included, so the RCCL init path of the
    N-GPU runs (`init_process_group("nccl", device_id=...)`) and TorchComm's device-tensor branch
    are exercised on a one-GPU box too (tests/test_gpu_rccl.py); run without a launcher at N = 1
    nothing is created.  Returns True when a process group exists."""
    import torch
    import torch.distributed as dist
    if "WORLD_SIZE" not in os.environ:
        return False
    if args.backend == "nccl":
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    else:
        dist.init_process_group("gloo")
    return True


def comm_check(dist, dev, rank, world, stage_host):
    """One call of every pf_dist.TorchComm collective the sharded C5 flow uses, on device tensors,
    checked against the values every rank can predict: all_reduce_sum, agree (rank 0's plan, on
    `dev`), the int16 broadcast (travels as bytes), and a ring exchange (isend / irecv pairs; a
    rank exchanges with itself only at world 1, where it is skipped).  The RCCL (device) branch
    runs with stage_host=False; gloo rehearsals stage through the host."""
    import torch
    import pf_dist
    comm = pf_dist.TorchComm(dist, stage_host=stage_host)
    res = {"backend": dist.get_backend(), "world": world, "stage_host": stage_host}
    a = torch.full((257,), float(rank + 1), dtype=torch.float32, device=dev)
    comm.all_reduce_sum(a)
    res["all_reduce_sum"] = bool(torch.all(a == world * (world + 1) / 2).item())
    got = comm.agree([10 + rank, 7, 10], 0, dev)
    res["agree"] = got == [10, 7, 10]
    b = torch.arange(1000, dtype=torch.int16, device=dev) * (1 if rank == 0 else 0) - 500
    comm.broadcast(b, 0)
    res["broadcast_i16"] = bool(torch.equal(b.cpu(), torch.arange(1000, dtype=torch.int16) - 500))
    if world > 1:
        nxt, prv = (rank + 1) % world, (rank - 1) % world
        snd = torch.full((4096,), float(rank), dtype=torch.float32, device=dev)
        rcv = torch.empty_like(snd)
        comm.exchange([(nxt, snd)], [(prv, rcv)])
        res["exchange"] = bool(torch.all(rcv == float(prv)).item())
    torch.cuda.synchronize(dev) if dev.type == "cuda" else None
    res["ok"] = all(v for k, v in res.items() if k in ("all_reduce_sum", "agree", "broadcast_i16",
                                                      "exchange"))
    return res


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(args):
    """`bench.py --gpus N` run directly (no WORLD_SIZE in the environment): start the N ranks
    ourselves -- one process per GPU under torch.distributed.run, rendezvous on 127.0.0.1 -- and
    return their exit status.  Runs BEFORE anything touches the GPU: only the device count is read
    (torch.cuda.device_count() does not initialise HIP), and the parent makes no other GPU call,
    so no process that has initialised the GPU is ever replaced or forked.  Returns None when this
    process is itself the (only) rank.  Refuses, with a message and a non-zero exit:
      * --gpus that disagrees with a launcher's WORLD_SIZE;
      * N ranks on fewer than N visible devices (unless --same-device: the one-GPU rehearsal);
      * --same-device with the nccl backend (RCCL refuses two ranks on one device)."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is not None:
        if int(env_world) != args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE="
                     f"{env_world} ranks; pass --gpus {env_world}")
        return None
    if args.gpus < 1:
        sys.exit(f"bench.py: --gpus {args.gpus}: need at least one")
    if args.gpus == 1:
        return None
    if args.same_device and args.backend == "nccl" and not args.stand_in:
        sys.exit("bench.py: --same-device needs --backend gloo (RCCL refuses two ranks on one "
                 "device)")
    if not args.stand_in and not args.same_device:
        import torch
        n = torch.cuda.device_count()
        if n < args.gpus:
            sys.exit(f"bench.py: --gpus {args.gpus} needs {args.gpus} GPUs, {n} visible (for a "
                     f"one-GPU rehearsal add --same-device --backend gloo)")
    import subprocess
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr", "127.0.0.1",
           f"--master-port={_free_port()}", os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")  # dmabuf IPC (RCCL across processes)
    return subprocess.run(cmd, env=env).returncode


def run_stand_in(args, rank, world):
    """The batch-sharded launcher with a CPU stand-in step (gloo): each rank 'processes' its own
    seed block, sleeping a rank-dependent time per step; rank 0 prints the bench line plus the
    gathered per-rank seeds and times, so the test can check disjoint seeds, the MAX reduction and
    global_batch = B x world."""
    import torch.distributed as dist
    B = args.batch
    seeds = rank_seeds(B, rank)
    step = lambda: time.sleep(0.01 * (rank + 1))  # noqa: E731
    mine, elapsed = timed_steps(step, lambda: None, args, world, dist)
    per_rank = [None] * world
    if world > 1:
        dist.all_gather_object(per_rank, {"rank": rank, "seeds": seeds, "elapsed": mine})
    else:
        per_rank = [{"rank": 0, "seeds": seeds, "elapsed": mine}]
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": B * world * args.steps / elapsed,
                          "unit": "panoramas/s", "n_gpus": world, "steps": args.steps,
                          "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
                          "config": {"global_batch": B * world}, "stand_in": True,
                          "elapsed": elapsed, "per_rank": per_rank}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


def main():
    args = parse()
    rc = launch_ranks(args)
    if rc is not None:
        sys.exit(rc)
    import numpy as np
    import torch
    import torch.distributed as dist

    import panofuse
    import pf_layouts as PL
    import pf_synth

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.stand_in:
        if world > 1:
            dist.init_process_group("gloo")
        return run_stand_in(args, rank, world)
    if args.same_device:
        local = 0
    elif torch.cuda.device_count() <= local:
        sys.exit(f"bench.py: rank {rank} wants cuda:{local}, "
                 f"{torch.cuda.device_count()} device(s) visible")
    dist_on = init_dist(args, world, local)
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    comm_res = comm_check(dist, dev, rank, world, args.backend == "gloo") if dist_on else None
    if comm_res is not None and not comm_res["ok"]:
        sys.exit(f"rank {rank}: TorchComm self-check failed: {comm_res}")
    if args.mode == "c5":
        return run_c5(args, rank, world, local, dev, dist_on, comm_res)

    out_w, ew = 2048, 512
    lay = PL.config_layout("C2")
    zr = PL.ZENITH_RANGE
    B = args.batch
    seeds = rank_seeds(B, rank)
    gt = pf_synth.scene_depth(seeds, out_w, out_w // 2, dev).contiguous()
    emap = pf_synth.baseline_emap(seeds, ew, ew // 2, dev).contiguous()
    resp = panofuse.make_responses(pf_synth.responses(seeds, lay.ntiles), dev)

    fz = panofuse.Fuser(local)
    fz.set_tiles(lay)
    tiles = torch.empty((B, fz.tile_elems), dtype=torch.float32, device=dev)
    out = torch.empty((B, out_w // 2, out_w), dtype=torch.int16, device=dev)
    coeffs = torch.empty((B, lay.ntiles, 4), dtype=torch.float32, device=dev)

    def step():
        fz.warp_depth(gt, tiles, resp)
        fz.merge(emap, tiles, out, zr, coeffs=coeffs)

    ctxs = [fz]
    if args.pipeline >= 2:
        lstep, lanes = lane_steps(fz, lay, local, dev, gt, emap, resp, tiles, out, coeffs, zr,
                                  args.pipeline)
        ctxs = [ln[0] for ln in lanes]
        mine_s, elapsed = timed_steps(lstep, torch.cuda.synchronize, args, world, dist, dev)
    elif args.pipeline:
        pstep = pipelined_step(fz, lay, local, dev, gt, emap, resp, tiles, out, coeffs, zr)
        mine_s, elapsed = timed_steps(pstep, torch.cuda.synchronize, args, world, dist, dev)
    else:
        mine_s, elapsed = timed_steps(step, torch.cuda.synchronize, args, world, dist, dev)
    # every fusion of the run was valid: raises PF_ETIMEOUT (non-zero exit) if a resident-kernel
    # hand-off wait timed out in any of them
    for c in ctxs:
        c.synchronize()
    # Per-kernel roofline: the same steps again with the library's hipEvent stage timers on
    # (recorded on the stream the kernels run on).  With the timers on, the library runs each
    # batch unsplit (no half-batch stream overlap), so every stage's time is its own.
    # Each step is read on its own and a stage's time is its MEDIAN over the steps: single serial
    # steps right after the pipelined loop vary by up to ~10 % (the chip's clock after the loop),
    # the median keeps one slow step out of the roofline.
    fz.profile(True)
    per_step = []
    for _ in range(max(1, args.prof_steps)):
        step()
        per_step.append(fz.profile_read())
    nps = len(per_step)
    prof = {k: (nps * sorted(p[k][0] for p in per_step)[nps // 2],  # median ms x steps
                sum(p[k][1] for p in per_step), sum(p[k][2] for p in per_step))
            for k in per_step[0]}
    # The lanes plan their passes for a share of the chip (lane_steps); the profiled steps above
    # run those plans, as the timed steps do.  For the record, the Jacobi stage with the
    # whole-chip plan (the serial step's; fewer rows per chunk, more waves) on the same batch.
    jserial = None
    if args.pipeline >= 2:
        fz.set_jacobi_share(1.0)
        js = []
        for _ in range(max(1, args.prof_steps)):
            step()
            js.append(fz.profile_read()["jacobi"][0])
        jserial = sorted(js)[len(js) // 2]
        fz.set_jacobi_share(LANE_SHARE)
    # Accuracy metrics (ErrorData of each result against its ground truth, median alignment,
    # Depth.cpp:1980-2213): not part of the step (the reference computes them only when a
    # ground-truth file is given), timed the same way on the same batch.
    # The fp64-tree summation is timed for the roofline; the reference's own (sequential float)
    # order, the library default, is timed beside it.
    mres = torch.zeros((B, 16), dtype=torch.int32, device=dev)
    fz.set_metrics_order("tree")
    for _ in range(max(1, args.prof_steps)):
        fz.error_metrics_async(gt, out, zr, mres, 1, True)
    prof["metrics"] = fz.profile_read()["metrics"]
    fz.set_metrics_order("sequential")
    fz.error_metrics_async(gt, out, zr, mres, 1, True)
    metrics_seq_ms = fz.profile_read()["metrics"][0]
    fz.profile(False)
    nprof = max(1, args.prof_steps)
    # SolveDepthBySmoothing (Depth.cpp:1773-1878, an ablation the reference leaves disabled):
    # not part of the step; its cost at batch 1 and at the step's batch, for the record.
    smooth = {}
    for nb in sorted({1, B}):
        o_s = torch.empty((nb, out_w // 2, out_w), dtype=torch.int16, device=dev)
        fz.solve_smoothing(tiles[:nb], o_s, zr, coeffs=coeffs[:nb])  # first call: layout tables
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fz.solve_smoothing(tiles[:nb], o_s, zr, coeffs=coeffs[:nb])
        e1.record()
        torch.cuda.synchronize()
        smooth[f"batch{nb}_ms"] = e0.elapsed_time(e1)
        del o_s

    # the E->P RGB warp (the reference's own split, a18), outside the step, at C3's shape
    rgbw = rgb_warp_measure(local, dev, lay, B) if not args.no_extra_configs else None
    # the other single-GPU BASELINE configs, for the record (outside the timed steps)
    c2 = c2_latency(local, dev, lay, zr) if not args.no_extra_configs else None
    c1 = (c2_latency(local, dev, PL.config_layout("C1"), zr, cfg="C1")
          if not args.no_extra_configs else None)
    c5 = None
    if world == 1 and not args.no_extra_configs:
        r5 = c5_measure(args, 0, 1, local, dev, steps=3, warmup=1)
        c5 = {"value": r5["value"], "unit": "panoramas/s", "ms_per_panorama": 1e3 / r5["value"],
              "steps": 3, "bit_exact_vs_one_gpu": r5["bit_exact"],
              "one_call_ms": r5["one_call_ms"],
              "model_8_ranks": r5["model_8_ranks"],
              "one_call": "pf_warp_depth + pf_merge of the same panorama on one context "
                          "(hipEvents, median of 5): the library path without the sharded "
                          "path's per-level host orchestration",
              "workload": "C5 on one GPU: one 8192x4096 panorama, 80 tiles of 1024^2 (10x8), "
                          "2048x1024 baseline, 4 levels (bench.py --mode c5 at world 1)"}

    total_panos = B * world * args.steps
    value = total_panos / elapsed
    jms, jbytes, jlaunch = prof["jacobi"]
    achieved = jbytes / (jms * 1e-3) / 1e9 if jms > 0 else 0.0
    jtf = jbytes / 12.0 * 14.0 / (jms * 1e-3) / 1e12 if jms > 0 else 0.0
    jtraffic = jacobi_traffic_per_step(jlaunch / nprof if nprof else 0)  # B per step
    wms, wbytes, wlaunch = prof["warp"]  # read 4 B/pano pixel + write 4 B/tile pixel (8d)
    wach = wbytes / (wms * 1e-3) / 1e9 if wms > 0 else 0.0
    stages = {k: {"ms_per_step": v[0] / nprof,
                  "GBps": (v[1] / (v[0] * 1e-3) / 1e9) if v[0] > 0 else 0.0,
                  "launches_per_step": v[2] / nprof} for k, v in prof.items()}
    # sanity, on EVERY rank: its outputs are populated and equal, bit for bit, to a fresh
    # one-process serial fusion of the same batch on a new context (warp + register + fuse);
    # the flags of all ranks are gathered into bit_exact_all_ranks
    nz = int((out[0].view(torch.int16) != 0).sum().item())
    fref = panofuse.Fuser(local)
    fref.set_tiles(lay)
    t_ref = torch.empty_like(tiles)
    o_ref = torch.empty_like(out)
    fref.warp_depth(gt, t_ref, resp)
    fref.merge(emap, t_ref, o_ref, zr, coeffs=torch.empty_like(coeffs))
    torch.cuda.synchronize()
    fref.synchronize()
    bit_exact = bool(torch.equal(o_ref, out))
    del fref, t_ref, o_ref
    # one sampled panorama per rank (a different position in each rank's block), hashed; with
    # --sample-dump its inputs and result are written for the oracle check in the tests
    import hashlib
    si = (rank * 37 + 5) % B
    sample_u16 = out[si].cpu().numpy().view(np.uint16)
    sample = {"index": si, "seed": seeds[si],
              "sha256": hashlib.sha256(sample_u16.tobytes()).hexdigest()}
    if args.sample_dump:
        os.makedirs(args.sample_dump, exist_ok=True)
        np.savez(os.path.join(args.sample_dump, f"rank{rank}.npz"), seed=np.int64(seeds[si]),
                 gt=gt[si].cpu().numpy(), emap=emap[si].cpu().numpy(),
                 resp=pf_synth.responses([seeds[si]], lay.ntiles), out=sample_u16)
    per_rank = [{"rank": rank, "seed0": seeds[0], "seedN": seeds[-1], "elapsed_s": mine_s,
                 "bit_exact": bit_exact, "sample": sample}]
    if world > 1:  # each rank's seed block, its own time (the line's value uses the MAX), checks
        per_rank = [None] * world
        dist.all_gather_object(per_rank, {"rank": rank, "seed0": seeds[0], "seedN": seeds[-1],
                                          "elapsed_s": mine_s, "bit_exact": bit_exact,
                                          "sample": sample})
    bit_exact_all = all(bool(p["bit_exact"]) for p in per_rank)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "panoramas/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (box-room scenes; tiles from the E->P warp + synthetic depth-net "
                    "response; baseline = biased noisy u16 low-res scene)",
            "config": {"workload": f"C3/C4: {B} panoramas per GPU per step, 2048x1024 output, "
                                   f"20 tiles of 512x512 (5x4 layout), 512x256 baseline",
                       "global_batch": B * world, "out": "2048x1024", "tiles": "20x512x512",
                       "parallelism": f"dp{world} (panorama sharding, no collective)",
                       "pipeline": (f"{args.pipeline} fusion lanes: batch k warped, registered "
                                    f"and fused on lane k % {args.pipeline} (own contexts, streams "
                                    f"and buffers; each lane warps its next batch on a second "
                                    f"stream; Jacobi passes planned for {LANE_SHARE:.2f} of the "
                                    f"chip)" if args.pipeline >= 2 else
                                    "warp of batch k+1 on a second stream beside the fusion "
                                    "of batch k, from the end of its level-0 sweeps"
                                    if args.pipeline else "off"),
                       "layout_caches": "tap maps, warp corner tables and level tables are "
                                        "built once per layout and panorama size, outside the "
                                        "timed steps (every step re-warps, re-registers and "
                                        "re-fuses the whole batch)"},
            # Headline: the dominant stage -- the Jacobi sweeps of one step, i.e. the resident
            # level-0 kernel (k_jres, all 200 sweeps in one launch) and the temporally blocked
            # passes of the finer levels (k_jlag) -- against its real roof, VALU issue:
            # algorithmic FLOP = 14 fp32 operations per pixel-update as the reference writes them
            # (Depth.cpp:1680-1717: 4 mul + 4 add for Lcur; sub, mul, add; 2 mul, add for b'),
            # per step, over the stage's hipEvent time, against the vector FP32 peak
            # (MI355X_MICROARCH.md).  `traffic` is the stage's HBM bytes per step measured by the
            # rocprofv3 PMC passes (profiles/pmc_traffic.json).
            "roofline": {"bound": "valu", "achieved": jtf, "peak": VALU_PEAK_TF,
                         "unit": "TFLOP/s", "frac": jtf / VALU_PEAK_TF,
                         "traffic": jtraffic,
                         "traffic_unit": "B per step (all Jacobi launches of the step)",
                         "kernel": "Jacobi stage: k_jres (level 0, resident) + k_jlag passes "
                                   "(levels 1-2), aggregated per step",
                         "flop_per_update": 14,
                         "launches_per_step": (jlaunch / nprof) if nprof else None,
                         "ms_per_step": jms / nprof if nprof else None,
                         "flop_per_step": jbytes / 12.0 * 14.0 / nprof if nprof else None,
                         "updates_per_step": jbytes / 12.0 / nprof,
                         "traffic_source": "profiles/pmc_traffic.json (FETCH_SIZE + WRITE_SIZE "
                                           "per launch of k_jlag and k_jres, scaled to one step)",
                         "plan": (f"lane plan (pf_set_jacobi_share {LANE_SHARE:.2f}: the levels' "
                                  "row chunks re-cut for concurrent lanes), as in the timed steps")
                         if args.pipeline >= 2 else "whole-chip plan",
                         "whole_chip_plan": ({"ms_per_step": jserial,
                                              "frac": jbytes / nprof / 12.0 * 14.0
                                              / (jserial * 1e-3) / 1e12 / VALU_PEAK_TF}
                                             if jserial else None)},
            # the same stage on the HBM roof with its MEASURED traffic (temporal blocking moves
            # T sweeps per pass through HBM once; the resident kernel reads the level once), and
            # the 12 B/update algorithmic rate of SURVEY.md 8d as an "effective" bandwidth (>
            # peak by construction: not a fraction)
            "roofline_hbm": {"bound": "hbm", "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "achieved": (jtraffic / (jms / nprof * 1e-3) / 1e9)
                             if (jtraffic and nprof and jms > 0) else None,
                             "frac": (jtraffic / (jms / nprof * 1e-3) / 1e9 / HBM_PEAK_GBS)
                             if (jtraffic and nprof and jms > 0) else None,
                             "kernel": "Jacobi stage (k_jres + k_jlag)",
                             "basis": "measured PMC bytes per step"},
            "effective_hbm": {"achieved": achieved, "unit": "GB/s",
                              "basis": "12 B per pixel-update (SURVEY.md 8d) / Jacobi time; "
                                       "temporal blocking keeps T-1 of every T sweeps on chip"},
            # north_star's named target: >= 60% of the HBM roofline on the warp kernel
            "roofline_warp": {"bound": "hbm", "achieved": wach, "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": wach / HBM_PEAK_GBS,
                              "traffic": pmc_traffic("pf::k_warp_depth"),
                              "kernel": "k_warp_depth",
                              "avg_launch_us": (wms / wlaunch * 1e3) if wlaunch else None,
                              "bytes_per_launch": (wbytes / wlaunch) if wlaunch else None},
            # the reference's E->P RGB tile render (a18) on the RGB panorama, outside the step
            "roofline_warp_rgb": rgbw,
            "stages": stages,
            # metrics stage (outside the timed step): algorithmic bytes = one read of the
            # compared band of gt (4 B) and result (2 B) per pixel; the kernels make 4 passes
            "roofline_metrics": {"bound": "hbm", "achieved": stages["metrics"]["GBps"],
                                 # HBM bytes of one call: 3 histogram passes + the sums pass
                                 "traffic": _metrics_traffic(),
                                 "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                 "frac": stages["metrics"]["GBps"] / HBM_PEAK_GBS,
                                 "kernel": "pf_error_metrics (k_med_hist x3, k_med_scan x3, "
                                           "k_err_sums, k_align, k_err_final), fp64 tree order",
                                 "ms_per_batch": stages["metrics"]["ms_per_step"],
                                 "ms_per_batch_sequential": metrics_seq_ms,
                                 "sequential": "the reference's float summation order (the "
                                               "facade's and CLI's default, bit-exact means): "
                                               "terms in parallel, verified fp32 add chains"},
            "nonzero_px_pano0": nz,
            "smoothing_ablation": dict(smooth, note="pf_solve_smoothing (SolveDepthBySmoothing, "
                                       "500 Gauss-Seidel sweeps near tile edges), outside the step"),
            "bit_exact_vs_one_process": bit_exact,
            # every rank's own batch against a fresh one-process fusion (C4: 8 checks)
            "bit_exact_all_ranks": bit_exact_all,
            "c1_batch1": c1,
            "c2_batch1_ms": c2["median_ms"] if c2 else None,
            "c2_batch1": c2,
            "c5_one_gpu": c5,
            "backend": args.backend if world > 1 else None,
            # every TorchComm collective once on device tensors (RCCL under a launcher, even at
            # world 1): init_dist / comm_check
            "comm_check": comm_res,
            "per_rank": per_rank if world > 1 else None,
            "sample_pano": per_rank[0]["sample"],
        }
        if not args.no_cpu_baseline and world == 1:  # the contract: rank 0 at N = 1 only
            line["cpu_baseline"] = cpu_baseline(args.cpu_seconds)
        print(json.dumps(line), flush=True)
    if dist_on:
        dist.barrier()
        dist.destroy_process_group()
    if not bit_exact_all:
        sys.exit(f"rank {rank}: a rank's fused batch differs from a fresh one-process fusion "
                 f"({[p['rank'] for p in per_rank if not p['bit_exact']]})")


if __name__ == "__main__":
    main()
