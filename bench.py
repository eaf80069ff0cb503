#!/usr/bin/env python3
"""Benchmark: batched racing-MPC solves/s on MI355X (BASELINE.json metric).

Workload (default ``--config C4``): BASELINE config 4, the blended-bicycle
contouring MPC at N = 40 in fp32 on the Shanghai centerline, 8 192 synthetic
instances per GPU (weak scaling: 8 GPUs = the 65 536-instance C4 batch).  One
"step" = one batched solve of the rank's shard, inputs resident in HBM, outputs
written to HBM (libmpcracing.so, one kernel launch).  Multi-GPU: one process per
GPU, contiguous shards, no data-path collective; RCCL only gathers the counters.

Prints ONE JSON line (rank 0).  Also reports the roofline of the solve kernel
against HBM (algorithmic bytes per SURVEY.md §8(d): 2*257*W*N bytes per
instance-iteration plus (13N+31)*W bytes of per-solve I/O) and a CPU baseline
(the oracle's dense IPM on a bounded sample, rank 0 / N=1 only).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def algorithmic_bytes(N, W, iters):
    """sum_i [2*257*W*N*I_i + (13N+31)*W]."""
    iters = np.asarray(iters, dtype=np.float64)
    return float((2 * 257 * W * N * iters).sum() + iters.size * (13 * N + 31) * W)


def cpu_baseline(name, budget_s):
    """Oracle (dense IPM, numpy/torch autograd, fp64) on the first instances of the same shard."""
    import torch
    torch.set_num_threads(1)
    from mpcracing import workload as wl
    from oracle.nlp import MPCProblem, solve_ipm
    cfg = wl.CONFIGS[name]
    b = wl.make_batch(name, limit=64)
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    n = 0
    t0 = time.time()
    for inst in wl.instance_dicts(b):
        p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=cfg["N"],
                       Ts=cfg["Ts"], model=cfg["model"], lane_bounds=cfg["lane"], tyres=tyres,
                       elastic=1e5 if cfg["lane"] else None)
        solve_ipm(p, tol=1e-8, max_iter=500)
        n += 1
        if time.time() - t0 > budget_s and n >= 2:
            break
    dt = time.time() - t0
    return {"value": n / dt, "unit": "solves/s", "cores": 1, "kind": "port",
            "sample": f"first {n} instances of the {name} shard, oracle dense primal-dual IPM "
                      f"(fp64, tol 1e-8, single thread, {dt:.1f} s)"}


def reduce_counters(counts, elapsed, world):
    """Whole-job totals over the ranks (the only collective of the run): SUM of the per-rank
    counters [solves, sum of iterations, algorithmic bytes, status histogram...] and MAX of the
    timed wall clock.  RCCL on the GPU box (backend "nccl"), gloo in the CPU tests."""
    import torch
    import torch.distributed as dist
    tot = counts.to(torch.float64)
    tmax = torch.tensor([float(elapsed)], dtype=torch.float64, device=tot.device)
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    return tot.cpu().numpy(), float(tmax.item())


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C4")
    ap.add_argument("--per-gpu", type=int, default=None)
    ap.add_argument("--cpu-budget", type=float, default=15.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true", help="skip the B = 1 latency probe (profiling runs)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    from mpcracing import workload as wl
    from mpcracing.batch import solver_for_config

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", local)
    cfg = wl.CONFIGS[args.config]
    per = args.per_gpu or cfg["per_gpu"]
    batch = wl.make_batch(args.config, rank=rank, world=world, per_gpu=per)
    B = int(batch["s0"].shape[0])
    solver = solver_for_config(args.config, B, device=local)
    dev_in = solver.to_device(batch)
    out = solver.alloc_outputs(B)
    stream = torch.cuda.current_stream(dev)

    for _ in range(args.warmup):
        solver.launch(dev_in, out, stream)
    torch.cuda.synchronize(dev)

    starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
    iters_sum = 0.0
    alg_bytes = 0.0
    statuses = np.zeros(5, dtype=np.int64)
    W = 4 if cfg["precision"] == "fp32" else 8
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for s in range(args.steps):
        starts[s].record(stream)
        solver.launch(dev_in, out, stream)
        ends[s].record(stream)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # per-launch kernel durations (HIP events on the launch stream)
    kms = [starts[s].elapsed_time(ends[s]) for s in range(args.steps)]
    it = out["iters"].cpu().numpy()
    stc = np.bincount(out["status"].cpu().numpy(), minlength=5)[:5]
    iters_sum = float(it.sum())
    alg_bytes = algorithmic_bytes(cfg["N"], W, it)
    statuses += stc

    # B = 1 latency (same configuration, first instance), p50 of 5 runs
    lat_b1_ms = None
    if not args.no_latency:
        b1 = {k: (v[..., :1].copy() if v is not None else None) for k, v in batch.items()}
        s1 = solver_for_config(args.config, 1, device=local)
        d1 = s1.to_device(b1)
        o1 = s1.alloc_outputs(1)
        lat = []
        for _ in range(6):
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            s1.launch(d1, o1, stream)
            torch.cuda.synchronize(dev)
            lat.append(time.perf_counter() - t)
        lat_b1_ms = float(np.median(lat[1:]) * 1e3)

    tot, elapsed_max = reduce_counters(
        torch.tensor([B * args.steps, iters_sum, alg_bytes] + statuses.tolist(), dtype=torch.float64, device=dev),
        elapsed, world)

    if rank == 0:
        solves = tot[0]
        kavg = float(np.mean(kms)) / 1e3
        achieved = alg_bytes / kavg / 1e9  # this rank's algorithmic bytes per launch / avg launch time
        traffic = None
        pmc_path = os.path.join(REPO, "profiles", f"pmc_{args.config}.json")
        if os.path.exists(pmc_path):
            with open(pmc_path) as f:
                pm = json.load(f)
            if pm.get("B") == B:
                traffic = pm.get("hbm_bytes_per_launch")
        line = {
            "metric": "MPC solves/sec (batch, N=40) + p50 per-solve latency, 1/2/4/8 MI355X",
            "value": solves / elapsed_max,
            "unit": "solves/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": elapsed_max / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32" if cfg["precision"] == "fp32" else "fp64",
            "data": "synthetic (SURVEY §8(d) seeded instance distribution on the reference's track assets)",
            "config": {"workload": f"{args.config}: {cfg['model']} bicycle MPC, N={cfg['N']}, "
                                   f"{cfg['precision']}, {per} instances per GPU, track {cfg['track']}"
                                   + (", lane-bound rows" if cfg["lane"] else ""),
                       "config_id": args.config, "N": cfg["N"], "instances_per_gpu": per,
                       "global_batch": int(per * world), "parallelism": f"dp{world} (instance shards)"},
            "p50_batch_latency_ms": float(np.median(kms)),
            "p50_latency_b1_ms": lat_b1_ms,
            "iters_mean": tot[1] / solves * args.steps / args.steps if solves else None,
            "status_hist": {"solved": int(tot[3]), "acceptable": int(tot[4]), "max_iter": int(tot[5]),
                            "failed": int(tot[6]), "lane_infeasible": int(tot[7])},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel": "mr_wave_kernel", "avg_launch_ms": kavg * 1e3,
                         "alg_bytes_per_launch": alg_bytes},
        }
        line["iters_mean"] = float(iters_sum / B)
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, REPO)
            line["cpu_baseline"] = cpu_baseline(args.config, args.cpu_budget)
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
