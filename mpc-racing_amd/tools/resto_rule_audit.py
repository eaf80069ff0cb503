"""Which of the restoration phase's rules changes outcomes?  The dense IPOPT restatement (oracle/ipopt.py) on the
C3 sample's restoration-phase instances (tests/golden/c3_sample_ipopt.npz, IPOPT_resto_iters > 0) under rule sets
between ``PRODUCT`` and ``IPOPT`` that differ in one restoration rule each, plus IPOPT without the initial-state
relaxation only.  Status / iterations / restoration iterations per instance and rule set, and agreement with the
fixture's IPOPT column.  CPU only (build container); output JSON lines.

Usage: python mpc-racing_amd/tools/resto_rule_audit.py OUT.jsonl [--procs=8] [--limit=23]
"""
import json
import os
import sys
import time
from dataclasses import replace
from multiprocessing import Pool

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
sys.path.insert(0, REPO)

OPTIONS = dict(tol=1e-8, acceptable_tol=1e-6, acceptable_iter=15, max_iter=500)


def rule_sets():
    from oracle import ipopt
    P = ipopt.PRODUCT
    return {
        "PRODUCT": P,
        "+watchdog": replace(P, resto_watchdog=True),
        "+ls_mult": replace(P, resto_ls_mult=True),
        "+soc": replace(P, resto_soc=True),
        "+relax_x0": replace(P, resto_relax_x0=True),
        "IPOPT-relax_x0": replace(ipopt.IPOPT, tiny_step=False, resto_relax_x0=False),
        "IPOPT-tiny": replace(ipopt.IPOPT, tiny_step=False),
    }


def _solve(args):
    import torch
    torch.set_num_threads(1)
    from mpcracing import workload as wl
    from oracle import ipopt
    from oracle.nlp import MPCProblem
    j, rn = args
    cfg = wl.CONFIGS["C3"]
    b = wl.make_batch("C3", limit=j + 1)
    inst = wl.instance_dicts(b)[j]
    p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=cfg["N"], Ts=cfg["Ts"],
                   model=cfg["model"], lane_bounds=cfg["lane"])
    t0 = time.time()
    r = ipopt.solve_ipopt(p, rules=rule_sets()[rn], log=True, **OPTIONS)
    _X, U, _S, _eC, _eL = p.unpack(r.w)
    return dict(j=j, rules=rn, status=int(r.status), iters=int(r.iters), resto_iters=sum(1 for e in r.log if e[7]),
                why=r.why, U=U.tolist(), t=round(time.time() - t0, 1))


def main():
    out = sys.argv[1]
    procs = int(next((a.split("=")[1] for a in sys.argv[2:] if a.startswith("--procs=")), 8))
    limit = int(next((a.split("=")[1] for a in sys.argv[2:] if a.startswith("--limit=")), 1000))
    g = dict(np.load(os.path.join(REPO, "tests", "golden", "c3_sample_ipopt.npz")))
    sel = np.nonzero(g["IPOPT_resto_iters"] > 0)[0][:limit]
    idx = [int(g["idx"][s]) for s in sel]
    ref = {int(g["idx"][s]): int(g["IPOPT_status"][s]) for s in sel}
    jobs = [(j, rn) for rn in rule_sets() for j in idx]
    with Pool(procs) as pool, open(out, "w") as f:
        res = []
        for r in pool.imap_unordered(_solve, jobs, chunksize=1):
            r["ipopt_status"] = ref[r["j"]]
            f.write(json.dumps(r) + "\n")
            f.flush()
            res.append(r)
        for rn in rule_sets():
            rs = [r for r in res if r["rules"] == rn]
            agree = sum(r["status"] == r["ipopt_status"] for r in rs)
            summ = {"summary": rn, "n": len(rs), "status_equal_to_IPOPT_fixture": agree,
                    "status_counts": np.bincount([r["status"] for r in rs], minlength=5).tolist()}
            f.write(json.dumps(summ) + "\n")
            print(json.dumps(summ), flush=True)


if __name__ == "__main__":
    main()
