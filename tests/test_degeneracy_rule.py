"""IPOPT's structural-degeneracy bookkeeping is not restated (oracle/ipopt.py header) -- pinned as inert here.

IPOPT (PDPerturbationHandler) declares the Hessian "degenerate", and from then on starts every
iteration's inertia correction with a perturbation instead of delta = 0, only when delta = 0 fails in
each of the first degen_iters_max = 3 iterations; one success declares it non-degenerate for the rest of
the solve.  The product and the oracle try delta = 0 first every iteration.  On the long C2 solve that
sets the C2 batch time (instance 628: 1.44 factorisations per iteration on the GPU, DESIGN.md §3.1 /
§11), the oracle's delta = 0 succeeds in iterations 0-3, so IPOPT would declare the Hessian
non-degenerate at once and its delta sequence is the one restated.
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))


def test_c2_long_solve_hessian_not_degenerate_at_start():
    import torch
    torch.set_num_threads(4)
    import oracle.ipopt as ip
    from oracle.nlp import MPCProblem
    from mpcracing import workload as wl
    cfg = wl.CONFIGS["C2"]
    b = wl.make_batch("C2")
    i = 628
    inst = wl.instance_dicts({k: (v[..., i:i + 1] if v is not None else None) for k, v in b.items()})[0]
    p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=cfg["N"], Ts=cfg["Ts"],
                   model=cfg["model"], lane_bounds=cfg["lane"])
    cls = [c for c in vars(ip).values() if isinstance(c, type) and hasattr(c, "factorize")][0]
    orig = cls.factorize
    deltas = []

    def rec(self, it, E, mu, delta_c=0.0):
        r = orig(self, it, E, mu, delta_c)
        deltas.append(None if r is None else r["delta"])
        return r

    cls.factorize = rec
    try:
        ip.solve_ipopt(p, rules=ip.IPOPT, tol=1e-4, acceptable_tol=1e-2, acceptable_iter=15, max_iter=500)
    finally:
        cls.factorize = orig
    assert all(d == 0.0 for d in deltas[:4]), deltas[:6]
    assert sum(1 for d in deltas if d) >= 10  # ... although delta = 0 fails often later in the solve
