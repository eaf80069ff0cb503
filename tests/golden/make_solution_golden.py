"""Generate tests/golden/solutions_<config>.npz: oracle solutions of the benchmark configs' instances.

TEST FIXTURE GENERATOR (build container only; the GPU box never runs the oracle's solves).

For config 1 (C1dyn: the reference's dynamic model, C1kin: the kinematic variant; one instance) and
each of C2, C3 (hard lane rows), C4 and C5 the first 32 instances of the config's batch
(mpcracing.workload.make_batch, deterministic) are solved in fp64 by oracle.ipopt.solve_ipopt -- the
dense restatement of IPOPT's algorithm with the watchdog and the restoration phase, under the rules the
product restates (``ipopt.PRODUCT``; among them IPOPT's bound_relax_factor 1e-8, so active bounds sit
1e-8 max(1, |b|) outside their nominal value, as in IPOPT's own solutions) -- to a KKT tolerance of 1e-10,
and the ret tuple of control/MPC.py:166-171 (States, U, S_hat, e_C, e_L), the objective, the
status and the iteration count are stored with the instance inputs.  tests/test_gpu_golden.py compares
the GPU's fp64 solves of the same inputs with them.

Usage: python tests/golden/make_solution_golden.py [C1dyn C1kin C2 C3 C4 C5]   (8 worker processes)
"""
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

N_INST = 32
TOL = 1e-10


def _config(name):
    """(config, batch); C1dyn / C1kin: config 1 (script/test_mpc.py's inputs, N = 20, Ts = 0.1) with the
    reference's dynamic model and the kinematic variant."""
    from mpcracing import workload as wl
    if name.startswith("C1"):
        cfg = dict(wl.CONFIGS["C1"], model=name[2:])
        return cfg, wl.make_batch("C1")
    return wl.CONFIGS[name], wl.make_batch(name, limit=N_INST)


def _n(name):
    return 1 if name.startswith("C1") else N_INST


def _solve(args):
    import torch
    torch.set_num_threads(1)
    from mpcracing import workload as wl
    from oracle.nlp import MPCProblem
    from oracle.ipopt import PRODUCT, solve_ipopt
    name, i = args
    cfg, b = _config(name)
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    inst = wl.instance_dicts(b)[i]
    p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=cfg["N"], Ts=cfg["Ts"],
                   model=cfg["model"], lane_bounds=cfg["lane"], tyres=tyres)
    t0 = time.time()
    r = solve_ipopt(p, tol=TOL, max_iter=1000, acceptable_iter=0, log=True, rules=PRODUCT)
    X, U, S, eC, eL = p.unpack(r.w)
    n_resto = sum(1 for e in r.log if e[7])
    return dict(i=i, status=r.status, iters=r.iters, resto_iters=n_resto, obj=r.obj, kkt=r.kkt, X=X, U=U, S=S,
                eC=eC, eL=eL, t=time.time() - t0)


def main():
    from mpcracing import workload as wl
    names = sys.argv[1:] or ["C1dyn", "C1kin", "C2", "C3", "C4", "C5"]
    jobs = [(n, i) for n in names for i in range(_n(n))]
    with Pool(8) as pool:
        res = pool.map(_solve, jobs, chunksize=1)
    for name in names:
        rs = sorted([r for (n, _), r in zip(jobs, res) if n == name], key=lambda r: r["i"])
        _cfg, b = _config(name)
        out = {k: np.stack([r[k] for r in rs], axis=-1) for k in ("X", "U", "S", "eC", "eL")}
        for k in ("status", "iters", "resto_iters"):
            out[k] = np.array([r[k] for r in rs], dtype=np.int32)
        for k in ("obj", "kkt"):
            out[k] = np.array([r[k] for r in rs])
        for k, v in b.items():
            if v is not None:
                out["in_" + k] = v
        np.savez_compressed(os.path.join(HERE, f"solutions_{name}.npz"), **out)
        summ = {"config": name, "n": _n(name), "tol": TOL, "rules": "PRODUCT", "status": out["status"].tolist(),
                "iters": out["iters"].tolist(), "resto_iters": out["resto_iters"].tolist(),
                "seconds": [round(r["t"], 1) for r in rs]}
        print(json.dumps(summ), flush=True)


if __name__ == "__main__":
    main()
