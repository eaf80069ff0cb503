"""Developer probe (GPU): the per-iteration trace of one instance of a config's batch, solved alone with
the config's product settings.  usage: python mpc-racing_amd/tools/gpu_trace1.py C4 844 [cap]
Writes gpurun_out/trace_<cfg>_<i>.npy and prints status / iterations / restoration markers."""
import os
import sys

import numpy as np

REPO = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
from mpcracing import workload as wl  # noqa: E402
from mpcracing.batch import solver_for_config  # noqa: E402

name, i = sys.argv[1], int(sys.argv[2])
cap = int(sys.argv[3]) if len(sys.argv) > 3 else 600
b = wl.make_batch(name, limit=i + 1)
sub = {k: (v[..., i:i + 1].copy() if v is not None else None) for k, v in b.items()}
s = solver_for_config(name, 1)
o = s.solve(sub, trace_instance=0, trace_cap=cap)
tr = o["trace"].cpu().numpy().reshape(-1, 8)
it = int(o["iters"][0])
os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
np.save(os.path.join(REPO, "gpurun_out", f"trace_{name}_{i}.npy"), tr)
m = tr[:it, 7]
print(name, i, "status", int(o["status"][0]), "iters", it, "resto its", int((m <= -200).sum()),
      "resto entries", int((m == -300).sum()), "watchdog", int(((m <= -100) & (m > -200)).sum()))
