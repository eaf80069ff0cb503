"""Iteration-level parity of the solver's IPOPT rules with the dense IPOPT restatement (oracle/ipopt.py).

The product solves the stage-wise restatement of the reference's NLP with a Riccati recursion
(csrc/mr_solver.h, the host build of the same source as the kernel); the oracle solves the NLP in the
reference's own variables (control/MPC.py:62-64) with a full-space KKT matrix and LDL inertia.  IPOPT's
iterates are determined by the step, the inertia correction delta_w (applied to the reference's variables,
mr_solver.h delta_var), the fraction-to-boundary rule and the filter line search, so the two must produce
the same per-iteration primal step size alpha, shift delta, constraint violation theta and barrier
parameter mu -- checked here over the first iterations of
  * a C2 instance (kinematic, no inertia correction), and
  * C3 instance 374 (dynamic model + hard lane rows; delta > 0 from the second iteration on, growing past
    1e2 within these iterations -- the instance the round-2 product left at max_iter).
The oracle runs under ``ipopt.PRODUCT``: IPOPT 3.14's rules (oracle/ipopt.py ``IPOPT``) less the few the
product does not restate (soft restoration, tiny-step termination, the restoration phase's own
watchdog / SOC / least-squares multipliers) -- none of which is reached in these iterations.
Tolerances: alpha, theta 1e-6 relative (different linear algebra, same arithmetic; theta also 1e-10
absolute: near feasibility it is roundoff of the defects), delta and mu exact to 1e-12 (they are products
of IPOPT's constants).
"""
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))

import host_twin as ht  # noqa: E402
from mpcracing import workload as wl  # noqa: E402


@pytest.mark.parametrize("name,i,K", [("C2", 5, 9), ("C3", 374, 14)])
def test_iterates_match_dense_ipopt(name, i, K):
    from oracle.ipopt import PRODUCT, solve_ipopt
    from oracle.nlp import MPCProblem
    cfg = wl.CONFIGS[name]
    b = wl.make_batch(name, limit=i + 1)
    sub = {k: (v[..., i:i + 1].copy() if v is not None else None) for k, v in b.items()}
    c = ht.config(cfg["N"], cfg["model"], "fp64", cfg["lane"], cfg["Ts"], tol=1e-8, acceptable_iter=15,
                  acceptable_tol=1e-6)
    tr = ht.solve(c, sub, nthreads=1, scalar=True, trace_instance=0, trace_cap=520)["trace"]
    inst = wl.instance_dicts(b)[i]
    p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=cfg["N"],
                   Ts=cfg["Ts"], model=cfg["model"], lane_bounds=cfg["lane"])
    r = solve_ipopt(p, tol=1e-8, max_iter=K, acceptable_tol=1e-6, acceptable_iter=15, log=True, rules=PRODUCT)
    rows = r.log[:K]
    assert len(rows) >= min(K, 8)
    for j, (_it, _kkt, mu, alpha, delta, th, _ph, in_resto) in enumerate(rows):
        assert not in_resto
        np.testing.assert_allclose(tr[j, 2], alpha, rtol=1e-6, err_msg=f"{name} {i} iteration {j}: alpha")
        np.testing.assert_allclose(tr[j, 4], delta, rtol=1e-12, err_msg=f"{name} {i} iteration {j}: delta")
        np.testing.assert_allclose(tr[j, 5], th, rtol=1e-6, atol=1e-10, err_msg=f"{name} {i} iteration {j}: theta")
        np.testing.assert_allclose(tr[j, 1], mu, rtol=1e-12, err_msg=f"{name} {i} iteration {j}: mu")
    if name == "C3":
        assert max(row[4] for row in rows) > 1e2  # the inertia correction is exercised


@pytest.mark.parametrize("i", [1, 10])
def test_whole_solve_matches_dense_ipopt(i):
    """Over a whole C2 solve (kinematic, tol 1e-8): the same optimality error at every iteration (IPOPT's
    scaled stationarity / primal / complementarity measure on the reference's NLP, mr_solver.h
    MR_KKT_RESTATED), hence the same barrier-parameter updates, the same termination iteration and the
    same objective.  (Instance 1 ended one iteration later than IPOPT while the error was measured on the
    restatement.)"""
    from oracle.ipopt import PRODUCT, solve_ipopt
    from oracle.nlp import MPCProblem
    cfg = wl.CONFIGS["C2"]
    b = wl.make_batch("C2", limit=i + 1)
    sub = {k: (v[..., i:i + 1].copy() if v is not None else None) for k, v in b.items()}
    c = ht.config(cfg["N"], cfg["model"], "fp64", cfg["lane"], cfg["Ts"], tol=1e-8, acceptable_iter=15,
                  acceptable_tol=1e-6)
    o = ht.solve(c, sub, nthreads=1, scalar=True, trace_instance=0, trace_cap=520)
    inst = wl.instance_dicts(b)[i]
    p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=cfg["N"],
                   Ts=cfg["Ts"], model=cfg["model"], lane_bounds=cfg["lane"])
    r = solve_ipopt(p, tol=1e-8, max_iter=500, acceptable_tol=1e-6, acceptable_iter=15, log=True, rules=PRODUCT)
    assert r.status == 0 and int(o["status"][0]) == 0
    assert int(o["iters"][0]) == r.iters
    for j, row in enumerate(r.log):
        np.testing.assert_allclose(o["trace"][j, 0], row[1], rtol=1e-6, err_msg=f"iteration {j}: kkt")
        np.testing.assert_allclose(o["trace"][j, 1], row[2], rtol=1e-12, err_msg=f"iteration {j}: mu")
    np.testing.assert_allclose(o["obj"][0], r.obj, rtol=1e-10)
