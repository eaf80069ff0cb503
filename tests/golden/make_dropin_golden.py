"""Generate tests/golden/dropin_C1.npz: the oracle's IPOPT solve of config 1 at the reference's options.

TEST FIXTURE GENERATOR (build container only).

Config 1 (script/test_mpc.py's inputs, N = 20, Ts = 0.1) with the reference's dynamic model and the
kinematic variant, solved in fp64 by oracle.ipopt.solve_ipopt under the product's rules at the reference's
IPOPT options (control/MPC.py:152-161: tol 1e-4, acceptable_tol 1e-2; IPOPT's acceptable_iter 15,
max_iter 500).  Stored: IPOPT's status (0 solved, 1 acceptable, 3 restoration failed ...), the iteration
count, the reason, the objective scaling df and the final iterate (States, U, S_hat) -- what the
reference's ``solution()`` returns, from ``opti.debug`` when the solve fails (MPC.py:172-181).
tests/test_gpu.py::test_dropin_mpc_class checks the drop-in class against it.

Usage: python tests/golden/make_dropin_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
sys.path.insert(0, REPO)


def main():
    import torch
    torch.set_num_threads(1)
    from mpcracing import workload as wl
    from oracle import ipopt
    from oracle.nlp import MPCProblem
    b = wl.make_batch("C1")
    inst = wl.instance_dicts(b)[0]
    out = {}
    for m in ("dyn", "kin"):
        p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=20, Ts=0.1, model=m)
        r = ipopt.solve_ipopt(p, tol=1e-4, max_iter=500, acceptable_tol=1e-2, acceptable_iter=15,
                              rules=ipopt.PRODUCT)
        X, U, S, _eC, _eL = p.unpack(r.w)
        out.update({f"{m}_status": np.int32(r.status), f"{m}_iters": np.int32(r.iters), f"{m}_X": X, f"{m}_U": U,
                    f"{m}_S": S, f"{m}_obj": np.float64(r.obj), f"{m}_obj_scale": np.float64(r.obj_scale)})
        print(json.dumps({"model": m, "status": int(r.status), "iters": int(r.iters), "why": r.why,
                          "obj_scale": float(r.obj_scale), "obj": float(r.obj)}), flush=True)
    np.savez_compressed(os.path.join(HERE, "dropin_C1.npz"), **out)


if __name__ == "__main__":
    main()
