"""The CPU baseline solver (scalar C++ build of mr_solver.h ``Solver``: the same IPM, one instance per
thread, OpenMP over instances -- what bench.py's cpu_baseline times) against the oracle.

Same parity bar as the GPU tests (tests/test_gpu.py): fp64 at KKT tol 1e-10, controls / states /
progress / errors within 1e-6 of the oracle's IPOPT solution (oracle.ipopt.solve_ipopt, the product's rules:
bounds relaxed by IPOPT's bound_relax_factor) (U[0, N-1] and vx_N excluded: only the
barrier fixes them), objective within 1e-8 relative."""
import numpy as np
import pytest

import host_twin as ht
from mpcracing import workload as wl
from oracle.ipopt import PRODUCT, solve_ipopt
from oracle.nlp import MPCProblem


@pytest.mark.parametrize("name,n,model", [("C1", 1, "kin"), ("C1", 1, "dyn"), ("C2", 2, None), ("C4", 1, None)])
def test_scalar_solver_vs_oracle(name, n, model):
    cfg = dict(wl.CONFIGS[name])
    if model:
        cfg["model"] = model
    b = wl.make_batch(name, limit=n)
    c = ht.config(cfg["N"], cfg["model"], "fp64", cfg["lane"], cfg["Ts"], tol=1e-10)
    o = ht.solve(c, b, nthreads=2, scalar=True)
    for i, inst in enumerate(wl.instance_dicts(b)):
        assert o["status"][i] == 0
        p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=cfg["N"],
                       Ts=cfg["Ts"], model=cfg["model"])
        r = solve_ipopt(p, tol=1e-10, max_iter=1000, acceptable_iter=0, rules=PRODUCT)
        X, U, S, eC, eL = p.unpack(r.w)
        dU = np.abs(U - o["U"][:, :, i])
        dU[0, -1] = 0.0
        dX = np.abs(X - o["X"][:, :, i])
        dX[3, -1] = 0.0
        assert dU.max() < 1e-6 and dX.max() < 1e-6, (dU.max(), dX.max())
        assert np.abs(S - o["S"][:, i]).max() < 1e-6
        assert np.abs(eC - o["eC"][:, i]).max() < 1e-6 and np.abs(eL - o["eL"][:, i]).max() < 1e-6
        assert abs(r.obj - o["obj"][i]) <= 1e-8 * max(1.0, abs(r.obj))


def test_scalar_matches_wave_twin_statuses():
    """Same algorithm as the wave solver (host emulation of the gfx950 kernel): same statuses and
    solutions on a C2 sample (iteration counts may differ by rounding of the Riccati order)."""
    cfg = wl.CONFIGS["C2"]
    b = wl.make_batch("C2", limit=16)
    c = ht.config(cfg["N"], cfg["model"], "fp64", cfg["lane"], cfg["Ts"], tol=1e-10)
    a = ht.solve(c, b, nthreads=8, scalar=True)
    w = ht.solve(c, b, nthreads=8)
    assert np.array_equal(a["status"], w["status"])
    dU = np.abs(a["U"] - w["U"])
    dU[0, -1] = 0.0
    assert dU.max() < 1e-6
