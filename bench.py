#!/usr/bin/env python3
"""Benchmark: batched racing-MPC solves/s on MI355X (BASELINE.json metric).

Workload (default ``--config C4``): BASELINE config 4, the blended-bicycle
contouring MPC at N = 40 in fp32 on the Shanghai centerline, 8 192 synthetic
instances per GPU (weak scaling; the 8 shards of 8 192 union to the 65 536-instance
C4 batch, mpcracing/workload.py).  One "step" = one batched solve of the rank's
shard, inputs resident in HBM, outputs written to HBM (libmpcracing.so, one
kernel launch).  Multi-GPU: one process per GPU, disjoint shards, no data-path
collective; RCCL only reduces the counters.  ``--gpus N`` without a launcher
(WORLD_SIZE unset) spawns the N rank processes itself before touching the GPU.

Prints ONE JSON line (rank 0), with the roofline of the solve kernel against HBM
(algorithmic bytes per SURVEY.md §8(d): 2*257*W*N bytes per instance-iteration
plus (13N+31)*W bytes of per-solve I/O) and the CPU baseline (rank 0, N = 1 only):
the scalar C++ fp64 build of the same interior-point solver (mr_solver.h
``Solver``, OpenMP over instances) on a time-bounded sample of the same shard.
"""
import argparse
import hashlib
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
METRIC = "MPC solves/sec (batch, N=40) + p50 per-solve latency, 1/2/4/8 MI355X"


def algorithmic_bytes(N, W, iters):
    """sum_i [2*257*W*N*I_i + (13N+31)*W]."""
    iters = np.asarray(iters, dtype=np.float64)
    return float((2 * 257 * W * N * iters).sum() + iters.size * (13 * N + 31) * W)


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def _cpu_threads():
    avail = len(os.sched_getaffinity(0))
    want = int(os.environ.get("OMP_NUM_THREADS", avail))
    return max(1, min(avail, want))


def cpu_baseline(name, batch, gpu_iters, budget_s):
    """The scalar C++ fp64 IPM (libmpcracing_host.so ``mrh_solve_batch_scalar``: mr_solver.h Solver, the
    same algorithm as the kernel, one instance per thread) on the host cores, on chunks of the rank's
    shard until ``budget_s``; plus the single-instance latency of BASELINE.md §2 (C1 + 100 C2 instances,
    one thread).  Termination: the fp64 defaults of the library (scaled KKT tol 1e-8, acceptable 1e-6
    over 15 iterations)."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import host_twin as ht
    from mpcracing import workload as wl
    cfg = wl.CONFIGS[name]
    cores = _cpu_threads()
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    c = ht.config(cfg["N"], cfg["model"], "fp64", cfg["lane"], cfg["Ts"], tol=1e-8, acceptable_iter=15,
                  acceptable_tol=1e-6)
    B = batch["s0"].shape[0]
    chunk = 128 * cores
    n = 0
    iters = []
    t0 = time.perf_counter()
    while n < B and time.perf_counter() - t0 < budget_s:
        m = min(chunk, B - n)
        sub = {k: (v[..., n:n + m].copy() if v is not None else None) for k, v in batch.items()}
        o = ht.solve(c, sub, tyres=tyres, nthreads=cores, scalar=True)
        iters.append(o["iters"])
        n += m
    dt = time.perf_counter() - t0
    it = np.concatenate(iters)
    # single-instance latency, one thread: C1 and 100 C2 instances
    lat = []
    c1 = wl.make_batch("C1")
    k1 = ht.config(20, "kin", "fp64", False, 0.1, tol=1e-8, acceptable_iter=15, acceptable_tol=1e-6)
    b2 = wl.make_batch("C2", limit=100)
    k2 = ht.config(20, "kin", "fp64", False, 0.05, tol=1e-8, acceptable_iter=15, acceptable_tol=1e-6)
    for kk, bb in [(k1, c1)] + [(k2, {k: (v[..., i:i + 1].copy() if v is not None else None)
                                      for k, v in b2.items()}) for i in range(100)]:
        t = time.perf_counter()
        ht.solve(kk, bb, nthreads=1, scalar=True)
        lat.append(time.perf_counter() - t)
    lat = np.array(lat) * 1e3
    return {"value": n / dt, "unit": "solves/s", "cores": cores, "kind": "port",
            "sample": f"first {n} instances of this rank's {name} shard ({cfg['model']}, N={cfg['N']}), "
                      f"scalar C++ fp64 build of the same IPM (mr_solver.h Solver, g++ -O2, OpenMP, "
                      f"{cores} threads), tol 1e-8, {dt:.1f} s",
            "cpu_model": _cpu_model(),
            "iters_mean_cpu_fp64": float(it.mean()), "iters_mean_gpu_same_instances": float(gpu_iters[:n].mean()),
            "latency_1core_ms": {"p50": float(np.median(lat)), "p90": float(np.quantile(lat, 0.9)),
                                 "sample": "C1 + 100 C2 instances, one at a time, 1 thread"},
            "fp32_ref_options": cpu_fp32_leg(name, batch, budget_s / 2),
            "agent_call_1thread_ms": agent_call_cpu(),
            "other_configs": cpu_other_configs(budget_s)}


AGENT_N, AGENT_TS = 15, 0.05  # /root/reference/agent.py:154 (N = 15), :181 (Ts = 0.05); dynamic model


def _agent_instances(n=100):
    """The agent's call (agent.py:171-183 -> control/MPC.py): B = 1, N = 15, the reference's dynamic model,
    fp64, the reference's IPOPT options; inputs = the first n C2 instances (state, progress, centerline
    polynomials and lane width drawn on the reference's track; no warm start)."""
    from mpcracing import workload as wl
    b = wl.make_batch("C2", limit=n)
    return [{k: (v[..., i:i + 1].copy() if v is not None else None) for k, v in b.items()} for i in range(n)]


def agent_call_gpu(local, n=100):
    """GPU side of the agent's call on the same instances: per call p50/p90 of (a) the kernel alone with
    the inputs resident (HIP-synchronised launch) and (b) the whole call from host arrays to host results
    (H2D copies, launch, D2H of States / U / S_hat, what control.MPC does)."""
    import torch
    from mpcracing.batch import BatchSolver
    s = BatchSolver(AGENT_N, "dyn", "fp64", False, AGENT_TS, max_batch=1, device=local, tol=1e-4, acceptable_tol=1e-2,
                    acceptable_iter=15)
    dev = torch.device("cuda", local)
    kern, call, st = [], [], []
    for sub in _agent_instances(n):
        d = s.to_device(sub)
        o = s.alloc_outputs(1)
        s.launch(d, o)  # warm (first touch of this instance's buffers)
        torch.cuda.synchronize(dev)
        t = time.perf_counter()
        s.launch(d, o)
        torch.cuda.synchronize(dev)
        kern.append(time.perf_counter() - t)
        t = time.perf_counter()
        r = s.solve(sub)
        _ = (r["X"].cpu(), r["U"].cpu(), r["S"].cpu(), r["status"].cpu())
        call.append(time.perf_counter() - t)
        st.append(int(o["status"][0]))
    kern, call = np.array(kern) * 1e3, np.array(call) * 1e3
    return {"kernel_ms": {"p50": float(np.median(kern)), "p90": float(np.quantile(kern, 0.9))},
            "call_ms": {"p50": float(np.median(call)), "p90": float(np.quantile(call, 0.9))},
            "status_hist": np.bincount(st, minlength=5).tolist()}


def agent_call_cpu(n=100):
    """CPU side: the scalar C++ solver (mr_solver.h Solver, the same IPM, fp64, same options), one thread,
    one instance at a time, on the same instances."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import host_twin as ht
    c = ht.config(AGENT_N, "dyn", "fp64", False, AGENT_TS, tol=1e-4, acceptable_iter=15, acceptable_tol=1e-2)
    lat, st = [], []
    for sub in _agent_instances(n):
        t = time.perf_counter()
        o = ht.solve(c, sub, nthreads=1, scalar=True)
        lat.append(time.perf_counter() - t)
        st.append(int(o["status"][0]))
    lat = np.array(lat) * 1e3
    return {"p50": float(np.median(lat)), "p90": float(np.quantile(lat, 0.9)),
            "status_hist": np.bincount(st, minlength=5).tolist(), "threads": 1}


def cpu_fp32_leg(name, batch, budget_s):
    """The scalar solver in fp32 at the reference's options (tol 1e-4, acceptable 1e-2 / 15: the GPU line's
    own precision and termination) on a bounded sample of the bench shard, all host threads."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import host_twin as ht
    from mpcracing import workload as wl
    cfg = wl.CONFIGS[name]
    cores = _cpu_threads()
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    c = ht.config(cfg["N"], cfg["model"], "fp32", cfg["lane"], cfg["Ts"], tol=1e-4, acceptable_iter=15,
                  acceptable_tol=1e-2)
    B = batch["s0"].shape[0]
    chunk = 128 * cores
    n, st = 0, []
    t0 = time.perf_counter()
    while n < B and time.perf_counter() - t0 < budget_s:
        m = min(chunk, B - n)
        sub = {k: (v[..., n:n + m].copy() if v is not None else None) for k, v in batch.items()}
        o = ht.solve(c, sub, tyres=tyres, nthreads=cores, scalar=True)
        st.append(o["status"])
        n += m
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "solves/s", "cores": cores, "instances": n, "seconds": dt,
            "status_hist": np.bincount(np.concatenate(st), minlength=5).tolist(),
            "sample": f"first {n} instances of the {name} shard, scalar C++ fp32 build, tol 1e-4 / acceptable 1e-2 x 15"}


def copy_bandwidth(dev, gib=1.0, reps=10):
    """Measured device copy bandwidth (frac against a measured copy as well as
    the 8 TB/s spec): torch's vectorised elementwise copy of a gib-GiB fp32 buffer into another, timed
    with HIP events over reps launches; bytes moved = read + write."""
    import torch
    n = int(gib * (1 << 30)) // 4
    a = torch.ones(n, dtype=torch.float32, device=dev)
    b = torch.empty_like(a)
    b.copy_(a)
    torch.cuda.synchronize(dev)
    st = torch.cuda.current_stream(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(st)
    for _ in range(reps):
        b.copy_(a)
    e1.record(st)
    torch.cuda.synchronize(dev)
    ms = e0.elapsed_time(e1) / reps
    del a, b
    return 2.0 * n * 4 / (ms * 1e-3) / 1e9


def cpu_other_configs(budget_s):
    """Scalar C++ fp64 twin throughput on bounded samples of C2 and C3 (BASELINE.md §2 asks for the
    C2 and C3 instance sets too): solves/s on this host's cores."""
    sys.path.insert(0, os.path.join(REPO, "tests"))
    import host_twin as ht
    from mpcracing import workload as wl
    cores = _cpu_threads()
    res = {}
    for name, n in (("C2", 1024), ("C3", 32 * cores)):
        cfg = wl.CONFIGS[name]
        b = wl.make_batch(name, limit=n)
        c = ht.config(cfg["N"], cfg["model"], "fp64", cfg["lane"], cfg["Ts"], tol=1e-8, acceptable_iter=15,
                      acceptable_tol=1e-6)
        t0 = time.perf_counter()
        o = ht.solve(c, b, nthreads=cores, scalar=True)
        dt = time.perf_counter() - t0
        res[name] = {"value": n / dt, "unit": "solves/s", "instances": n, "seconds": dt,
                     "solved_frac": float((o["status"] <= 1).mean()), "iters_mean": float(o["iters"].mean())}
        if time.perf_counter() - t0 > budget_s:
            break
    return res


def reduce_counters(counts, elapsed, world, pg=False):
    """Whole-job totals over the ranks (the only collective of the run): SUM of the per-rank
    counters [solves, sum of iterations, algorithmic bytes, status histogram...] and MAX of the
    timed wall clock.  RCCL on the GPU box (backend "nccl"), gloo in the CPU tests."""
    import torch
    import torch.distributed as dist
    tot = counts.to(torch.float64)
    tmax = torch.tensor([float(elapsed)], dtype=torch.float64, device=tot.device)
    if world > 1 or pg:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    return tot.cpu().numpy(), float(tmax.item())


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def spawn(nproc, argv):
    """One child process per rank (the launcher the driver would otherwise provide).  Runs before this
    process touches the GPU; returns the worst exit code."""
    port = str(_free_port())
    procs = []
    for r in range(nproc):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nproc), LOCAL_WORLD_SIZE=str(nproc),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env))
    codes = [p.wait() for p in procs]
    return max(abs(c) for c in codes)


def _lib_sha():
    from mpcracing import abi
    h = hashlib.sha256()
    with open(os.environ.get("MR_PRODUCT_LIB") or abi.PRODUCT_LIB, "rb") as f:
        h.update(f.read())
    return h.hexdigest()[:16]


def pipelined(args, solver, dev_in, out, batch, B, dev, local, nstreams):
    """Serving-mode figure, reported beside the line's value (which times one batch at a time): the same
    batch on ``nstreams`` independent handles (own workspaces) and HIP streams, 2 x steps launches
    round-robin, so one batch's bulk runs on the CUs the previous batch's few long solves leave idle.
    Each launch solves the whole batch (results checked identical to the timed leg's)."""
    import torch
    from mpcracing.batch import solver_for_config
    hs = [solver] + [solver_for_config(args.config, B, device=local, dispatch_order=args.dispatch_order)
                     for _ in range(nstreams - 1)]
    ins = [dev_in] + [h.to_device(batch) for h in hs[1:]]
    outs = [h.alloc_outputs(B) for h in hs]
    streams = [torch.cuda.Stream(dev) for _ in range(nstreams)]
    for h, i, o, st in zip(hs, ins, outs, streams):
        h.launch(i, o, st)
    torch.cuda.synchronize(dev)
    n = 2 * args.steps
    t0 = time.perf_counter()
    for q in range(n):
        j = q % nstreams
        hs[j].launch(ins[j], outs[j], streams[j])
    torch.cuda.synchronize(dev)
    el = time.perf_counter() - t0
    same = all(bool(torch.equal(o[k], out[k])) for o in outs for k in ("status", "iters", "obj"))
    return {"streams": nstreams, "launches": n, "value": B * n / el, "unit": "solves/s",
            "ms_per_batch": el / n * 1e3, "results_identical": same,
            "note": "independent batches in flight on separate streams (not the line's value)"}


def shard_spread(args, solver, out, dev, stream, ms0):
    """The other shards of the multi-GPU split solved one at a time on this GPU (N = 1 only; not the line's
    value): the batch time is the slowest solve's latency, and which instances run to max_iter is decided by
    rounding, so shard 0's time is one draw -- the 8-GPU job's time is the slowest shard's.  One warm launch per
    shard, HIP events on the launch stream."""
    import torch
    from mpcracing import workload as wl
    cfg = wl.CONFIGS[args.config]
    per = args.per_gpu or cfg["per_gpu"]
    n = max(1, cfg["B"] // per)
    if n < 2:
        return None
    ms = [ms0]
    for r in range(1, n):
        b = wl.make_batch(args.config, rank=r, world=n, per_gpu=per)
        d = solver.to_device(b)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        solver.launch(d, out, stream)
        e1.record(stream)
        torch.cuda.synchronize(dev)
        ms.append(e0.elapsed_time(e1))
    return {"shards": n, "ms_per_shard": [round(x, 2) for x in ms], "ms_max": round(max(ms), 2),
            "ms_mean": round(float(np.mean(ms)), 2),
            "note": "shard r of the 8-GPU split (workload.make_batch(config, r, 8)) on this GPU, one launch each "
                    "(shard 0: the timed steps' p50); the 8-GPU job's batch time is the slowest shard's"}


def cpu_check(args, rank, world):
    """--cpu-check: the multi-rank plumbing without a GPU (gloo): each rank builds its shard and the
    counters go through reduce_counters; rank 0 prints the shard layout.  Used by tests/test_multirank.py."""
    import torch
    import torch.distributed as dist
    from mpcracing import workload as wl
    if world > 1:
        dist.init_process_group("gloo", rank=rank, world_size=world)
    per = args.per_gpu or wl.CONFIGS[args.config]["per_gpu"]
    segs, K, n_shards = wl.shard_segments(args.config, rank, world, per)
    b = wl.make_batch(args.config, rank=rank, world=world, per_gpu=per)
    B = int(b["s0"].shape[0])
    counts = torch.tensor([B, float(b["state0"][3].sum()), float(len(segs))], dtype=torch.float64)
    tot, tmax = reduce_counters(counts, 1.0 + rank, world)
    gathered = [None] * world
    if world > 1:
        dist.all_gather_object(gathered, segs)
    else:
        gathered = [segs]
    if rank == 0:
        print(json.dumps({"n_gpus": world, "instances": int(tot[0]), "vx_sum": float(tot[1]), "K": K,
                          "n_shards": n_shards, "segments": gathered, "elapsed_max": tmax}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="C4")
    ap.add_argument("--per-gpu", type=int, default=None)
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-latency", action="store_true", help="skip the B = 1 latency probe and the pipelined figure (profiling runs: "
                                                           "only the timed launches)")
    ap.add_argument("--cpu-check", action="store_true", help="multi-rank plumbing on CPU (gloo), no solve")
    ap.add_argument("--dispatch-order", type=int, default=1, help="mr_config.dispatch_order (A/B runs)")
    ap.add_argument("--pipeline", type=int, default=4,
                    help="streams of the serving-mode figure 'pipelined' (< 2: skip it)")
    ap.add_argument("--dry-run", action="store_true",
                    help="CPU test of the rank plumbing of the real path (MR_BENCH_BACKEND=gloo): process group, "
                         "shards, counter reduction and the JSON line, with the solves skipped (no GPU)")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        sys.exit(spawn(args.gpus, sys.argv[1:]))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE {world}")
    if args.cpu_check:
        return cpu_check(args, rank, world)

    import torch
    import torch.distributed as dist
    from mpcracing import workload as wl
    from mpcracing.batch import solver_for_config

    # backend: RCCL ("nccl") on the GPU box; MR_BENCH_BACKEND=gloo with --dry-run drives this same path
    # on CPU in tests/test_multirank.py
    backend = os.environ.get("MR_BENCH_BACKEND", "nccl")
    dry = args.dry_run
    if dry and backend != "gloo":
        raise SystemExit("--dry-run needs MR_BENCH_BACKEND=gloo (it is the CPU test of the rank plumbing)")
    # MR_BENCH_PG=1: the process group and its collectives also at world size 1 -- the multi-GPU path's RCCL
    # initialisation (device_id), barriers and counter all-reduce exercised on a one-GPU box
    pg = world > 1 or os.environ.get("MR_BENCH_PG") == "1"
    if pg:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        if dry:
            dist.init_process_group(backend, rank=rank, world_size=world)
        else:
            torch.cuda.set_device(local)
            dist.init_process_group(backend, rank=rank, world_size=world, device_id=torch.device("cuda", local))
    elif not dry:
        torch.cuda.set_device(0)
    dev = torch.device("cpu") if dry else torch.device("cuda", local)
    cfg = wl.CONFIGS[args.config]
    per = args.per_gpu or cfg["per_gpu"]
    batch = wl.make_batch(args.config, rank=rank, world=world, per_gpu=per)
    B = int(batch["s0"].shape[0])
    W = 4 if cfg["precision"] == "fp32" else 8
    if dry:  # no solve: zero iterations, every instance "solved", unit timings
        if pg:
            dist.barrier()
        t0 = time.perf_counter()
        if pg:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        kms = [1.0] * args.steps
        it = np.zeros(B, dtype=np.int32)
        stc = np.array([B, 0, 0, 0, 0])
    else:
        solver = solver_for_config(args.config, B, device=local, dispatch_order=args.dispatch_order)
        dev_in = solver.to_device(batch)
        out = solver.alloc_outputs(B)
        stream = torch.cuda.current_stream(dev)

        for _ in range(args.warmup):
            solver.launch(dev_in, out, stream)
        torch.cuda.synchronize(dev)

        starts = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
        ends = [torch.cuda.Event(enable_timing=True) for _ in range(args.steps)]
        if pg:
            dist.barrier()
        torch.cuda.synchronize(dev)
        t0 = time.perf_counter()
        for s in range(args.steps):
            starts[s].record(stream)
            solver.launch(dev_in, out, stream)
            ends[s].record(stream)
        torch.cuda.synchronize(dev)
        if pg:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        # per-launch kernel durations (HIP events on the launch stream)
        kms = [starts[s].elapsed_time(ends[s]) for s in range(args.steps)]
        it = out["iters"].cpu().numpy()
        stc = np.bincount(out["status"].cpu().numpy(), minlength=5)[:5]
    iters_launch = float(it.sum())            # one launch (every launch solves the same shard)
    alg_bytes = algorithmic_bytes(cfg["N"], W, it)

    # B = 1 latency (same configuration, first instance), p50 of 5 runs
    lat_b1_ms = None
    if not args.no_latency and not dry:
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

    agent = None
    if not args.no_latency and not dry and rank == 0:
        agent = agent_call_gpu(local)

    pipe = None
    if args.pipeline >= 2 and world == 1 and not dry and not args.no_latency:
        pipe = pipelined(args, solver, dev_in, out, batch, B, dev, local, args.pipeline)

    spread = None
    if world == 1 and not dry and not args.no_latency:
        spread = shard_spread(args, solver, out, dev, stream, float(np.median(kms)))

    tot, elapsed_max = reduce_counters(
        torch.tensor([B * args.steps, iters_launch, alg_bytes, B] + stc.tolist(), dtype=torch.float64, device=dev),
        elapsed, world, pg)

    copy_gbs = None
    if rank == 0 and not dry:
        copy_gbs = copy_bandwidth(dev)

    if rank == 0:
        solves = tot[0]
        kavg = float(np.mean(kms)) / 1e3
        achieved = alg_bytes / kavg / 1e9  # this rank's algorithmic bytes per launch / avg launch time
        traffic, traffic_src, compute = None, None, None
        pmc_path = os.path.join(REPO, "profiles", f"pmc_{args.config}.json")
        if os.path.exists(pmc_path):
            with open(pmc_path) as f:
                pm = json.load(f)
            if pm.get("B") == B and pm.get("lib_sha") == _lib_sha():
                traffic = pm.get("hbm_bytes_per_launch")
                compute = pm.get("compute")
                traffic_src = (f"{os.path.relpath(pmc_path, REPO)}: rocprofv3 --pmc passes of this command on "
                               f"the same libmpcracing.so build (sha {pm['lib_sha']})")
        line = {
            "metric": METRIC,
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
                       "global_batch": int(tot[3]), "parallelism": f"dp{world} (instance shards)"},
            # what the reference's opti.solve() accepts: IPOPT's "solved" and "solved to acceptable level"
            # (status <= 1); the status-3 stops at the mu floor are the except branch
            "solved_per_s": float(tot[4] + tot[5]) * args.steps / elapsed_max,
            "solved_frac": float(tot[4] + tot[5]) / float(tot[3]),
            "p50_batch_latency_ms": float(np.median(kms)),
            "p50_latency_b1_ms": lat_b1_ms,
            "iters_mean": float(tot[1] / tot[3]),
            "status_hist": {"solved": int(tot[4]), "acceptable": int(tot[5]), "max_iter": int(tot[6]),
                            "failed": int(tot[7]), "infeasible": int(tot[8])},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                         "kernel": "mr_wave_kernel", "avg_launch_ms": kavg * 1e3,
                         "alg_bytes_per_launch": alg_bytes,
                         "scope": ("per rank: rank 0's algorithmic bytes per launch over rank 0's average launch "
                                   "time (weak scaling: every rank solves an equal shard; the whole job's "
                                   "throughput is `value`)") if world > 1 else "the single GPU's launch",
                         "copy_gbs": copy_gbs,
                         "frac_vs_copy": (achieved / copy_gbs) if copy_gbs else None,
                         "copy_source": "measured in this run: 1 GiB fp32 device-to-device copy (torch copy_, "
                                        "read + write bytes), HIP events",
                         "compute": compute},
        }
        if pipe is not None:
            line["pipelined"] = pipe
        if spread is not None:
            line["shard_spread"] = spread
        if agent is not None:
            line["agent_call"] = dict(agent, config=f"agent.py:154,171-183: B = 1, N = {AGENT_N}, dyn, fp64, "
                                                    f"Ts {AGENT_TS}, tol 1e-4 / acceptable 1e-2 x 15; the first 100 "
                                                    "C2 instances (cpu side: cpu_baseline.agent_call_1thread_ms)")
        if dry:
            line["dry_run"] = True
        if pg:
            line["process_group"] = {"backend": dist.get_backend(), "world_size": world,
                                     "collectives": "barrier around the timed steps; all_reduce SUM of the counters, "
                                                    "MAX of the wall clock"}
        if world == 1 and not args.no_cpu_baseline and not dry:
            line["cpu_baseline"] = cpu_baseline(args.config, batch, it, args.cpu_budget)
        print(json.dumps(line), flush=True)
    if pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
