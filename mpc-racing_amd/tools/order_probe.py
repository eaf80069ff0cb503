"""Dispatch-order probe: how much of a C4 batch's time is the slowest instances starting late?

Solves the C4 shard in its natural order, then the same instances permuted (slowest first by the
measured iteration counts = the ideal longest-first order; and reversed), timing each launch with
HIP events.  Writes per-instance iterations and the initial states to gpurun_out/order_probe.json
for offline analysis of iteration-count predictors.  Developer tool (not the product path)."""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
from mpcracing import workload as wl  # noqa: E402
from mpcracing.batch import solver_for_config  # noqa: E402


def permute(batch, p):
    return {k: (v[..., p].copy() if v is not None else None) for k, v in batch.items()}


def timed(solver, batch, reps=3):
    d = solver.to_device(batch)
    out = solver.alloc_outputs(int(batch["s0"].shape[0]))
    st = torch.cuda.current_stream()
    solver.launch(d, out, st)
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record(st)
        solver.launch(d, out, st)
        b.record(st)
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    return float(np.median(ts)), out["iters"].cpu().numpy(), out["status"].cpu().numpy()


def main(cfg="C4"):
    batch = wl.make_batch(cfg)
    B = int(batch["s0"].shape[0])
    solver = solver_for_config(cfg, B)
    res = {}
    t, it, stt = timed(solver, batch)
    res["natural_ms"] = t
    print("natural", t, flush=True)
    p = np.argsort(-it, kind="stable")
    t2, it2, _ = timed(solver, permute(batch, p))
    assert np.array_equal(it2, it[p]), "iterations depend on the position in the batch"
    res["longest_first_ms"] = t2
    print("longest-first", t2, flush=True)
    t3, _, _ = timed(solver, permute(batch, np.arange(B)[::-1].copy()))
    res["reversed_ms"] = t3
    print("reversed", t3, flush=True)
    res["iters"] = it.tolist()
    res["status"] = stt.tolist()
    res["state0"] = batch["state0"].tolist()
    res["s0"] = batch["s0"].tolist()
    os.makedirs("gpurun_out", exist_ok=True)
    with open(f"gpurun_out/order_probe_{cfg}.json", "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main(*(sys.argv[1:2] or ["C4"]))
