"""Developer tool: batched closed-loop throughput and a GA population evaluation on the GPU.

  python mpc-racing_amd/tools/closed_loop_bench.py [B] [ticks]

B vehicles spread along Shanghai (fp64 dynamic-model MPC, N = 15, blended plant, control from
tick 1), then a 16-individual x 5-segment GA fitness evaluation (mpcracing.ga).  Writes
gpurun_out/closed_loop_bench.json.
"""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
from mpcracing import ga  # noqa: E402
from mpcracing.closed_loop import ClosedLoop  # noqa: E402
from mpcracing.geometry import DeviceTrack  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    T = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    res = {}
    tr = DeviceTrack("shanghai_intl_circuit")
    # fp64 in index order and in hint order (dispatch_order 2: the previous tick's iterations, the
    # ClosedLoop default), fp32 in hint order
    for prec, order in (("fp64", 0), ("fp64", 2), ("fp32", 2)):
        loop = ClosedLoop(tr, B=B, N=15, plant="blend", precision=prec, start_control_at=1, dispatch_order=order)
        s0 = (np.arange(B) + 0.5) * tr.length / B
        loop.reset(ClosedLoop.start_states(tr, s0, v0=15.0))
        loop.run(2)  # global projections of the first tick, warm-up
        torch.cuda.synchronize()
        t = time.time()
        recs = loop.run(T)
        torch.cuda.synchronize()
        dt = time.time() - t
        st = np.stack([r["status"].cpu().numpy() for r in recs])
        it = np.stack([r["iters"].cpu().numpy() for r in recs])
        err = np.abs(recs[-1]["error"].cpu().numpy())
        res[f"{prec}_order{order}"] = {"B": B, "dispatch_order": order, "ticks": T, "s": dt, "ticks_per_s": T / dt, "vehicle_ticks_per_s": B * T / dt,
                     "status_hist": np.bincount(st.ravel(), minlength=5).tolist(), "iters_mean": float(it.mean()),
                     "iters_max": int(it.max()), "abs_error_p50": float(np.median(err)),
                     "abs_error_max": float(err.max())}
        print(prec, order, json.dumps(res[f"{prec}_order{order}"]), flush=True)
    host_track = __import__("mpcracing.track", fromlist=["Track"]).Track("shanghai_intl_circuit")
    seg = ga.TrackSegments(host_track, 5, 30, 1500, 1500, 250)   # GA/mpcGA.py:31
    rng = np.random.default_rng(0)
    pop = np.stack([rng.uniform(500, 2000, 16), np.full(16, 0.85), rng.uniform(20, 80, 16), np.full(16, 2.0),
                    rng.uniform(2000, 8000, 16)], 1)
    t = time.time()
    times, _ = ga.evaluate_population(tr, pop, seg.bounds, ticks=500, v0=15.0)
    dt = time.time() - t
    r, avg = ga.rewards(np.where(np.isfinite(times), times, 1e3), np.full(5, seg.lap_time / 5))
    res["ga"] = {"population": 16, "segments": 5, "ticks": 500, "s": dt, "bounds": seg.bounds,
                 "lap_time_model": seg.lap_time, "reached": int(np.isfinite(times).sum()),
                 "times_mean": float(np.nanmean(np.where(np.isfinite(times), times, np.nan))),
                 "best": int(np.argmax(r))}
    print("ga", json.dumps(res["ga"]), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "closed_loop_bench.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
