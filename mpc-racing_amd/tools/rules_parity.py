"""Product (scalar fp64 build, csrc/mr_solver.h) vs the dense IPOPT restatement (oracle/ipopt.py, rules
PRODUCT) on the first n instances of a config: status, iterations, objective, and the first iteration whose
(alpha, delta, theta, mu) differ.  One JSON line per instance.

Usage: python mpc-racing_amd/tools/rules_parity.py C3 16 [--tol 1e-4] [--procs 8] > out.jsonl
"""
import argparse
import json
import os
import sys
from multiprocessing import Pool

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))
ARGS = None


def run(i):
    import numpy as np
    import torch
    torch.set_num_threads(1)
    import host_twin as ht
    from mpcracing import workload as wl
    from oracle import ipopt
    from oracle.nlp import MPCProblem
    a = ARGS
    cfg = wl.CONFIGS[a.config]
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    acc = 1e-2 if a.tol >= 1e-4 else 1e-6
    b = wl.make_batch(a.config, limit=i + 1)
    sub = {k: (v[..., i:i + 1].copy() if v is not None else None) for k, v in b.items()}
    c = ht.config(cfg["N"], cfg["model"], "fp64", cfg["lane"], cfg["Ts"], tol=a.tol, acceptable_iter=15,
                  acceptable_tol=acc)
    o = ht.solve(c, sub, tyres=tyres, nthreads=1, scalar=True, trace_instance=0, trace_cap=520)
    inst = wl.instance_dicts(b)[i]
    p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=cfg["N"], Ts=cfg["Ts"],
                   model=cfg["model"], lane_bounds=cfg["lane"], tyres=tyres)
    r = ipopt.solve_ipopt(p, tol=a.tol, max_iter=500, acceptable_tol=acc, acceptable_iter=15, log=True,
                          rules=ipopt.PRODUCT)
    tr = o["trace"]
    first = None
    for j, row in enumerate(r.log):
        if row[7] or j >= int(o["iters"][0]) or tr[j, 7] <= -200:
            break
        pa = (tr[j, 2], tr[j, 4], tr[j, 5], tr[j, 1])
        oa = (row[3], row[4], row[5], row[2])
        if any(abs(x - y) > 1e-6 * abs(y) + 1e-9 for x, y in zip(pa, oa)):
            first = j
            break
    rec = {"config": a.config, "i": int(i), "tol": a.tol,
           "product": [int(o["status"][0]), int(o["iters"][0]), float(o["obj"][0])],
           "oracle": [int(r.status), int(r.iters), float(r.obj), r.why],
           "first_diff_iter": first, "compared": min(len(r.log), int(o["iters"][0]))}
    print(json.dumps(rec), flush=True)
    return rec


def main():
    global ARGS
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("n", type=int)
    ap.add_argument("--tol", type=float, default=1e-4)
    ap.add_argument("--procs", type=int, default=8)
    ap.add_argument("--start", type=int, default=0)
    ARGS = ap.parse_args()
    with Pool(ARGS.procs) as pool:
        for _ in pool.imap_unordered(run, range(ARGS.start, ARGS.start + ARGS.n)):
            pass


if __name__ == "__main__":
    main()
