"""Developer probe: iteration traces of the slowest fp32 instances of a config, in fp32 and fp64."""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
from mpcracing import workload as wl  # noqa: E402
from mpcracing.batch import BatchSolver, solver_for_config  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "C4"
    cfg = wl.CONFIGS[name]
    b = wl.make_batch(name)
    B = b["s0"].shape[0]
    s = solver_for_config(name, B)
    o = {k: v.cpu().numpy() for k, v in s.solve(b).items()}
    order = np.argsort(-o["iters"])[:4]
    res = {}
    for i in order.tolist():
        sub = {k: (v[..., i:i + 1].copy() if v is not None else None) for k, v in b.items()}
        rows = {}
        for prec in ("fp32", "fp64"):
            sv = BatchSolver(cfg["N"], cfg["model"], prec, cfg["lane"], cfg["Ts"], max_batch=1)
            out = sv.solve(sub, trace_instance=0, trace_cap=520)
            tr = out["trace"].cpu().numpy()
            it = int(out["iters"][0])
            rows[prec] = {"iters": it, "status": int(out["status"][0]), "kkt": float(out["kkt"][0]),
                          "trace": [[round(float(x), 6) for x in tr[j]] for j in list(range(0, min(it, 40))) +
                                    list(range(40, it, 25))]}
        res[i] = rows
        print(i, "fp32", rows["fp32"]["iters"], rows["fp32"]["status"], rows["fp32"]["kkt"], "| fp64",
              rows["fp64"]["iters"], rows["fp64"]["status"], rows["fp64"]["kkt"], flush=True)
    with open(os.path.join(REPO, "gpurun_out", f"tail_{name}.json"), "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
