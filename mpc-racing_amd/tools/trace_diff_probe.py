"""Developer probe: the per-iteration trace (kkt, mu, alpha, alpha_du, delta, theta, phi, ls code) of given
instances over repeated solves of the same batch; prints the first iteration at which a repeat's trace differs
from the first solve's, with the rows around it (localises a run-to-run difference).

Usage: python mpc-racing_amd/tools/trace_diff_probe.py C5 --limit 512 --precision fp64 --inst 243 287 367
"""
import argparse
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("config")
    ap.add_argument("--limit", type=int, default=512)
    ap.add_argument("--precision", default=None)
    ap.add_argument("--inst", type=int, nargs="+", required=True)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--cap", type=int, default=3100)
    ap.add_argument("--solo", action="store_true", help="each instance solved alone (a batch of one)")
    a = ap.parse_args()
    from mpcracing import workload as wl
    from mpcracing.batch import solver_for_config
    b = wl.make_batch(a.config, limit=a.limit)
    kw = {"precision": a.precision} if a.precision else {}
    s = solver_for_config(a.config, a.limit, **kw)
    np.set_printoptions(precision=17, linewidth=250)
    for i in a.inst:
        trs = []
        bi, ti = b, i
        if a.solo:
            bi = {k: (np.ascontiguousarray(v[..., i:i + 1]) if isinstance(v, np.ndarray) and v.shape[-1] == a.limit
                      else v) for k, v in b.items()}
            ti = 0
        for r in range(a.reps):
            o = s.solve(bi, trace_instance=ti, trace_cap=a.cap)
            trs.append((o["trace"].cpu().numpy(), int(o["iters"][ti]), int(o["status"][ti])))
        t0 = trs[0][0]
        for r in range(1, a.reps):
            t = trs[r][0]
            d = np.nonzero(np.any(t[:-4] != t0[:-4], axis=1))[0]
            rec = {"inst": i, "rep": r, "iters": [trs[0][1], trs[r][1]], "status": [trs[0][2], trs[r][2]],
                   "first_diff_iter": int(d[0]) if d.size else None}
            print(json.dumps(rec), flush=True)
            if d.size:
                k = int(d[0])
                for q in range(max(0, k - 2), k + 2):
                    print(" it", q, "ref", t0[q].tolist(), flush=True)
                    print(" it", q, "rep", t[q].tolist(), flush=True)


if __name__ == "__main__":
    main()
