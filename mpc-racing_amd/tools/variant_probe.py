"""Developer probe: solve 64 C4 fp64 instances with a given build of libmpcracing and compare
statuses/iterations with the host build."""
import os
import sys

import numpy as np
import torch  # noqa: F401  (torch first: one HIP runtime in the process)

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from mpcracing import abi  # noqa: E402

abi.load_product(sys.argv[1])
import host_twin as ht  # noqa: E402
from mpcracing import workload as wl  # noqa: E402
from mpcracing.batch import BatchSolver  # noqa: E402

name = sys.argv[2] if len(sys.argv) > 2 else "C4"
prec = sys.argv[3] if len(sys.argv) > 3 else "fp64"
cfg = wl.CONFIGS[name]
b = wl.make_batch(name, limit=64)
tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
s = BatchSolver(cfg["N"], cfg["model"], prec, cfg["lane"], cfg["Ts"], max_batch=64, acceptable_iter=0, tyres=tyres)
o = {k: v.cpu().numpy() for k, v in s.solve(b).items()}
h = ht.solve(ht.config(cfg["N"], cfg["model"], prec, cfg["lane"], cfg["Ts"], tol=s.cfg.tol, acceptable_iter=0,
                       acceptable_tol=s.cfg.acceptable_tol), b, tyres=tyres, nthreads=16)
print(os.path.basename(sys.argv[1]), name, prec, "gpu", np.bincount(o["status"], minlength=5).tolist(),
      "host", np.bincount(h["status"], minlength=5).tolist(), "same_iters",
      float((o["iters"] == h["iters"]).mean()), flush=True)
