"""Developer probe: iteration-count distribution and batch time of a config under
several termination settings (writes gpurun_out/iter_probe.json)."""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
from mpcracing import workload as wl  # noqa: E402
from mpcracing.batch import solver_for_config  # noqa: E402

SETTINGS = {
    "default": {},
    "reference_ipopt": dict(tol=1e-4, acceptable_tol=1e-2, acceptable_iter=15),
}


def main():
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["C4"]
    res = {}
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    for name in names:
        b = wl.make_batch(name)
        B = b["s0"].shape[0]
        for sname, kw in SETTINGS.items():
            solver = solver_for_config(name, B, **kw)
            dev = solver.to_device(b)
            out = solver.alloc_outputs(B)
            torch.cuda.synchronize()
            t = time.time()
            solver.launch(dev, out)
            torch.cuda.synchronize()
            dt = time.time() - t
            o = {k: v.cpu().numpy() for k, v in out.items()}
            it = o["iters"]
            r = {"B": B, "time_s": dt, "solves_per_s": B / dt, "status": np.bincount(o["status"], minlength=5).tolist(),
                 "iters_mean": float(it.mean()), "iters_max": int(it.max()),
                 "iters_q": [float(np.quantile(it, q)) for q in (0.5, 0.9, 0.99, 0.999)],
                 "hist": np.histogram(it, bins=[0, 10, 20, 30, 40, 50, 75, 100, 150, 200, 300, 400, 501])[0].tolist(),
                 "slow_idx": np.argsort(-it)[:8].tolist(), "slow_kkt": o["kkt"][np.argsort(-it)[:8]].tolist()}
            res[f"{name}/{sname}"] = r
            print(name, sname, json.dumps(r), flush=True)
    with open(os.path.join(REPO, "gpurun_out", "iter_probe.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
