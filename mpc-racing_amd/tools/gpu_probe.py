"""Developer probe: run each BASELINE config once on the GPU, compare with the
host build of the same solver on a subset, and time it (writes gpurun_out/probe.json)."""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))
from mpcracing import workload as wl  # noqa: E402
from mpcracing.batch import solver_for_config  # noqa: E402


def main():
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["C1", "C2", "C4", "C3"]
    sub = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    res = {}
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    for name in names:
        cfg = wl.CONFIGS[name]
        t0 = time.time()
        b = wl.make_batch(name)
        B = b["s0"].shape[0]
        gen = time.time() - t0
        solver = solver_for_config(name, B)
        dev = solver.to_device(b)
        out = solver.alloc_outputs(B)
        solver.launch(dev, out)
        torch.cuda.synchronize()
        times = []
        for _ in range(3):
            torch.cuda.synchronize()
            t = time.time()
            solver.launch(dev, out)
            torch.cuda.synchronize()
            times.append(time.time() - t)
        o = {k: v.cpu().numpy() for k, v in out.items()}
        st = np.bincount(o["status"], minlength=5).tolist()
        r = {"B": B, "gen_s": gen, "times": times, "solves_per_s": B / min(times), "status": st,
             "iters_mean": float(o["iters"].mean()), "iters_max": int(o["iters"].max()),
             "iters_p50": float(np.median(o["iters"]))}
        # compare with the host build on a subset
        try:
            import host_twin as ht
            n = min(sub, B)
            bs = {k: (v[..., :n].copy() if v is not None else None) for k, v in b.items()}
            c = ht.config(cfg["N"], cfg["model"], cfg["precision"], cfg["lane"], cfg["Ts"],
                          tol=solver.cfg.tol, acceptable_iter=solver.cfg.acceptable_iter,
                          acceptable_tol=solver.cfg.acceptable_tol)
            tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
            t = time.time()
            oh = ht.solve(c, bs, tyres=tyres, nthreads=16)
            r["host_s"] = time.time() - t
            ok = (o["status"][:n] == 0) & (oh["status"] == 0)
            r["host_status_match"] = float((o["status"][:n] == oh["status"]).mean())
            r["host_iters_match"] = float((o["iters"][:n] == oh["iters"]).mean())
            r["host_max_dU"] = float(np.abs(o["U"][:, :, :n] - oh["U"])[:, :, ok].max()) if ok.any() else None
        except Exception as e:  # noqa: BLE001
            r["host_err"] = repr(e)
        res[name] = r
        print(name, json.dumps(r), flush=True)
    with open(os.path.join(REPO, "gpurun_out", "probe.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
