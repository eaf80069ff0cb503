"""Audit (CPU): the dense IPOPT restatement (oracle/ipopt.py) on chosen instances of a config.

For every instance: the oracle under IPOPT's rules (``IPOPT``) and under the round-3 restatement's rules
(``R3``), at the reference's options (control/MPC.py:152-161: tol 1e-4, acceptable_tol 1e-2,
acceptable_iter 15, max_iter 500) or a tight tolerance, fp64; optionally scipy SLSQP from the reference's
initial guess (an independent method: is there a feasible KKT point?).  One JSON line per instance.

Usage: python mpc-racing_amd/tools/ipopt_audit.py C4 447,4765,... [--tol 1e-4] [--rules IPOPT,R3]
       [--slsqp] [--procs 8] > out.jsonl
       (an index list "first:N" takes instances 0..N-1)
"""
import argparse
import json
import os
import sys
import time
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
sys.path.insert(0, REPO)

ARGS = None


def run(i):
    import torch
    torch.set_num_threads(1)
    from mpcracing import workload as wl
    from oracle import ipopt
    from oracle.nlp import MPCProblem, solve_slsqp
    a = ARGS
    cfg = wl.CONFIGS[a.config]
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    b = wl.make_batch(a.config, limit=i + 1)
    inst = wl.instance_dicts(b)[i]
    p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=cfg["N"], Ts=cfg["Ts"],
                   model=cfg["model"], lane_bounds=cfg["lane"], tyres=tyres)
    acc_tol = 1e-2 if a.tol >= 1e-4 else 1e-6
    rec = {"config": a.config, "i": int(i), "tol": a.tol, "acceptable_tol": acc_tol}
    for rn in a.rules.split(","):
        t0 = time.time()
        r = ipopt.solve_ipopt(p, tol=a.tol, max_iter=500, acceptable_tol=acc_tol, acceptable_iter=15, log=True,
                              rules=getattr(ipopt, rn))
        rec[rn] = {"status": int(r.status), "iters": int(r.iters), "kkt": float(r.kkt), "obj": float(r.obj),
                   "resto_iters": int(sum(1 for row in r.log if row[7])), "cpu_s": round(time.time() - t0, 1),
                   "obj_scale": float(r.obj_scale), "max_row_gradient": float(r.max_row_gradient),
                   "U0": [float(v) for v in p.split(r.w)[0][:, 0]], "why": r.why, "stats": r.stats}
    if a.slsqp:
        import torch as T
        s = solve_slsqp(p)
        w = T.tensor(s.x, dtype=T.float64)
        rec["slsqp"] = {"status": int(s.status), "eq": float(np.abs(p.g(w).numpy()).max()),
                        "ineq": float(p.d(w).numpy().min()), "obj": float(s.fun)}
    print(json.dumps(rec), flush=True)
    return rec


def main():
    global ARGS
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("indices")
    ap.add_argument("--tol", type=float, default=1e-4)
    ap.add_argument("--rules", default="IPOPT,R3")
    ap.add_argument("--slsqp", action="store_true")
    ap.add_argument("--procs", type=int, default=8)
    ARGS = ap.parse_args()
    if ARGS.indices.startswith("first:"):
        idx = list(range(int(ARGS.indices.split(":")[1])))
    else:
        idx = [int(v) for v in ARGS.indices.split(",")]
    with Pool(ARGS.procs) as pool:
        for _ in pool.imap_unordered(run, idx):
            pass


if __name__ == "__main__":
    main()
