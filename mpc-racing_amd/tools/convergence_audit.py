"""Convergence audit (CPU): instances the solver does not solve, re-run by independent methods.

For the first ``n`` instances of a config, the scalar C++ build of the solver (same algorithm as the
kernel) finds the instances that end in max_iter / failed / lane-infeasible; each of those is then
given to (a) the oracle's dense fp64 IPM (oracle/nlp.py, same IPOPT-style rules, torch autograd
derivatives) and (b) scipy SLSQP from the reference's initial guess (an independent algorithm).  An
instance that (a) or (b) solves to a KKT point but the product does not is a solver weakness.

Usage: python mpc-racing_amd/tools/convergence_audit.py C3 256 [max_checked] > profiles/r02_audit_C3.json
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def main():
    import torch
    import host_twin as ht
    from mpcracing import workload as wl
    from oracle.nlp import MPCProblem, solve_ipm, solve_slsqp, kkt_residuals
    name, n = sys.argv[1], int(sys.argv[2])
    max_checked = int(sys.argv[3]) if len(sys.argv) > 3 else 20
    cfg = wl.CONFIGS[name]
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    b = wl.make_batch(name, limit=n)
    c = ht.config(cfg["N"], cfg["model"], "fp64", cfg["lane"], cfg["Ts"], tol=1e-8, acceptable_iter=15,
                  acceptable_tol=1e-6)
    t0 = time.time()
    o = ht.solve(c, b, tyres=tyres, nthreads=len(os.sched_getaffinity(0)), scalar=True)
    rec = {"config": name, "n": n, "status_hist": np.bincount(o["status"], minlength=5).tolist(),
           "iters_mean": float(o["iters"].mean()), "cpu_s": time.time() - t0, "unsolved": []}
    bad = np.nonzero(o["status"] >= 2)[0][:max_checked]
    insts = wl.instance_dicts(b)
    T = lambda a: torch.tensor(a, dtype=torch.float64)  # noqa: E731
    for i in bad:
        inst = insts[i]
        p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=cfg["N"],
                       Ts=cfg["Ts"], model=cfg["model"], lane_bounds=cfg["lane"], tyres=tyres,
                       elastic=1e5 if cfg["lane"] else None)
        r = solve_ipm(p, tol=1e-8, max_iter=500)
        e = {"i": int(i), "status": int(o["status"][i]), "iters": int(o["iters"][i]), "kkt": float(o["kkt"][i]),
             "oracle_status": r.status, "oracle_iters": r.iters, "oracle_kkt": r.kkt}
        s = solve_slsqp(p)
        g = np.abs(p.g(T(s.x)).numpy()).max()
        dmin = p.d(T(s.x)).numpy().min()
        e.update(slsqp_status=int(s.status), slsqp_eq=float(g), slsqp_ineq=float(dmin), slsqp_obj=float(s.fun),
                 oracle_obj=float(r.obj))
        if cfg["lane"]:
            t = s.x[9 * cfg["N"] + 7:]
            e["slsqp_lane_slack_max"] = float(np.max(t))
        rec["unsolved"].append(e)
        print(json.dumps(e), file=sys.stderr, flush=True)
    print(json.dumps(rec, indent=1))


if __name__ == "__main__":
    main()
