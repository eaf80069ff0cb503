"""Developer probe: one config's batch on every shard of the multi-GPU split (workload.make_batch(name, rank, W)),
solved one shard at a time on this GPU -- per shard the launch time (HIP events, best of 2 after a warm-up), the
status histogram, max_iter count and total iterations.  The batch time is the slowest solve's latency, and which
instances run long is decided by rounding, so a change of the arithmetic is judged over the 8 shards (the
8-GPU job's time is the slowest shard's), not on shard 0 alone.  MR_PRODUCT_LIB selects the build.

Usage: python mpc-racing_amd/tools/shard_sweep.py C4 [--world 8] [--out gpurun_out/shards.json]
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch
    from mpcracing import workload as wl
    from mpcracing.batch import solver_for_config
    cfg = wl.CONFIGS[a.config]
    B = cfg["per_gpu"]
    s = solver_for_config(a.config, B)
    outs = s.alloc_outputs(B)
    recs = []
    for r in range(a.world):
        ins = s.to_device(wl.make_batch(a.config, r, a.world))
        s.launch(ins, outs)
        torch.cuda.synchronize()
        ms = []
        for _ in range(2):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            s.launch(ins, outs)
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
        st = outs["status"].cpu().numpy()
        it = outs["iters"].cpu().numpy()
        rec = {"config": a.config, "rank": r, "world": a.world, "ms": round(min(ms), 2),
               "status": np.bincount(st, minlength=5).tolist(), "max_iter": int((st == 2).sum()),
               "iters_total": int(it.sum()), "lib": os.environ.get("MR_PRODUCT_LIB", "product")}
        print(json.dumps(rec), flush=True)
        recs.append(rec)
    summ = {"config": a.config, "ms_per_shard": [x["ms"] for x in recs], "ms_max": max(x["ms"] for x in recs),
            "ms_mean": round(float(np.mean([x["ms"] for x in recs])), 2), "iters_total": sum(x["iters_total"] for x in recs),
            "lib": os.environ.get("MR_PRODUCT_LIB", "product")}
    print(json.dumps(summ), flush=True)
    if a.out:
        with open(a.out, "w") as f:
            json.dump({"shards": recs, "summary": summ}, f, indent=1)


if __name__ == "__main__":
    main()
