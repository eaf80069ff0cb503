"""Developer probe: per-iteration traces of selected instances, GPU vs host build."""
import os
import sys

import numpy as np

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
import host_twin as ht  # noqa: E402
from mpcracing import workload as wl  # noqa: E402
from mpcracing.batch import BatchSolver  # noqa: E402

name, model, prec = sys.argv[1], sys.argv[2], sys.argv[3]
idx = [int(v) for v in sys.argv[4].split(",")]
cfg = wl.CONFIGS[name]
b = wl.make_batch(name, limit=max(idx) + 1)
res = {}
for i in idx:
    s = BatchSolver(cfg["N"], model, prec, cfg["lane"], cfg["Ts"], max_batch=b["s0"].shape[0], acceptable_iter=0)
    o = s.solve(b, trace_instance=i, trace_cap=200)
    res[f"gpu_{i}"] = o["trace"].cpu().numpy()
    res[f"gpu_status_{i}"] = int(o["status"][i])
    h = ht.solve(ht.config(cfg["N"], model, prec, cfg["lane"], cfg["Ts"], tol=s.cfg.tol, acceptable_iter=0,
                           acceptable_tol=s.cfg.acceptable_tol), b, trace_instance=i, trace_cap=200)
    res[f"host_{i}"] = h["trace"]
    res[f"host_status_{i}"] = int(h["status"][i])
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.savez(os.path.join(REPO, "gpurun_out", "trace.npz"), **res)
print("ok")
