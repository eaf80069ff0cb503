"""The reference's dual output, ``opti.lam_g`` (control/MPC.py:171), from the solver's stage-wise multipliers.

Bar: at fp64 tol 1e-10 the exported lam_g [13N+9] equals the oracle's multipliers mapped to the
reference's Opti rows (oracle.ipopt.solve_ipopt under the product's rules, oracle.nlp.MPCProblem.lam_g_ipopt; row
order pinned against the reference's own constraint recording in tests/test_nlp_golden.py) to 1e-7 relative
to max |lam_g|.  CasADi's sign
convention: Lagrangian f + lam_g . g with the canonical Opti rows (stated, not pinned: no casadi here).
CPU test: the host build of the kernel source (emulated wavefront); GPU test: libmpcracing.so."""
import numpy as np
import pytest

import host_twin as ht
from mpcracing import workload as wl
from oracle.ipopt import PRODUCT, solve_ipopt
from oracle.nlp import MPCProblem


def _oracle_lam(cfg, inst, model, N, Ts):
    p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=N, Ts=Ts, model=model)
    r = solve_ipopt(p, tol=1e-10, max_iter=1000, acceptable_iter=0, rules=PRODUCT)
    assert r.status == 0
    return p.lam_g_ipopt(r.nu, r.lam)


def _check(lg, mine):
    ok = ~np.isnan(mine)
    assert ok.sum() == len(lg)
    assert np.abs(lg - mine[ok]).max() <= 1e-7 * np.abs(lg).max(), np.abs(lg - mine[ok]).max()


@pytest.mark.parametrize("model", ["kin", "dyn"])
def test_lam_g_host_build_vs_oracle(model):
    b = wl.make_batch("C1")
    o = ht.solve(ht.config(20, model, "fp64", False, 0.1, tol=1e-10), b, nthreads=1, duals=True)
    assert o["status"][0] == 0
    _check(_oracle_lam(None, wl.instance_dicts(b)[0], model, 20, 0.1), o["lam_g"][:, 0])


def test_lam_g_state0_controls_none():
    """state0.throttle / steer None: the two state0 rows are absent (NaN in the fixed layout), 13N+7 rows."""
    b = wl.make_batch("C1")
    b["state0"][6:, 0] = np.nan
    rng = np.random.default_rng(3)
    u = np.stack([rng.uniform(-0.5, 0.8, 20), rng.uniform(-0.3, 0.3, 20)])
    u[:, -1] = u[:, -2]  # a shifted last_controls repeats its last column (MPC.py:120-121)
    b["u_init"] = u[:, :, None].copy()
    o = ht.solve(ht.config(20, "dyn", "fp64", False, 0.1, tol=1e-10), b, nthreads=1, duals=True)
    assert o["status"][0] == 0 and np.isnan(o["lam_g"][-2:, 0]).all()
    inst = wl.instance_dicts(b)[0]
    cols = [(float(a), float(s)) for a, s in zip(*u)]
    lc = [(0.0, 0.0)] + cols[:-1]  # MPCProblem shifts last_controls itself: lc[1:] + [lc[-1]] == cols
    p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=20, Ts=0.1, model="dyn",
                   last_controls=lc)
    r = solve_ipopt(p, tol=1e-10, max_iter=1000, acceptable_iter=0, rules=PRODUCT)
    _check(p.lam_g_ipopt(r.nu, r.lam), o["lam_g"][:, 0])


@pytest.mark.gpu
def test_lam_g_gpu_vs_oracle():
    from mpcracing.batch import BatchSolver
    cfg = wl.CONFIGS["C2"]
    b = wl.make_batch("C2", limit=3)
    s = BatchSolver(cfg["N"], cfg["model"], "fp64", False, cfg["Ts"], max_batch=3, tol=1e-10, acceptable_iter=0)
    o = {k: v.cpu().numpy() for k, v in s.solve(b, duals=True).items()}
    for i, inst in enumerate(wl.instance_dicts(b)):
        assert o["status"][i] == 0
        _check(_oracle_lam(cfg, inst, cfg["model"], cfg["N"], cfg["Ts"]), o["lam_g"][:, i])
