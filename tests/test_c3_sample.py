"""C3 (hard lane rows, IPOPT's restoration phase) against the full IPOPT restatement on a random sample.

Fixture: tests/golden/c3_sample_ipopt.npz (generator tests/golden/make_c3_sample_golden.py) -- 128 instances
drawn uniformly from the 8 192-instance C3 batch, solved by oracle.ipopt.solve_ipopt at the C3 tests'
tolerance (tol 1e-8, acceptable_tol 1e-6 over 15, max_iter 500) under the FULL IPOPT rules (``IPOPT``) and
under the product's (``PRODUCT``: no least-square multipliers, second-order corrections or watchdog inside
the restoration phase, the initial-state rows kept hard there -- DESIGN.md §2).  23 of the 128 enter the
restoration phase.  What it shows:
  * the restatement of IPOPT itself solves 123 of 128 (96.1 %): the failures of the C3 batch are largely
    IPOPT's (max_iter, restoration failure, local infeasibility), not the port's;
  * the product's remaining restoration-phase deviations change few outcomes: the emulated kernel (host
    build) ends with IPOPT's status on 127 of 128 (22 of the 23 that enter restoration), and at the same
    point (1e-6 in U) on 115 of the 123 both solve (measured).
Bars: status equal to IPOPT's on >= 95 % of the sample; on its restoration instances the status class
(converged / not) equal on >= 85 % and the exact status on >= 75 % (GPU, round 5: 22 / 23 and 19 / 23 -- the
four differing codes are failures both ways but one: max_iter vs failed, failed vs infeasible); where both
solve, the same point (max |dU| < 1e-6) on >= 85 %; the product solves at least IPOPT's count - 2.
"""
import os

import numpy as np
import pytest

import host_twin as ht
from mpcracing import workload as wl

HERE = os.path.dirname(os.path.abspath(__file__))


def _fix():
    return dict(np.load(os.path.join(HERE, "golden", "c3_sample_ipopt.npz")))


def _batch(idx):
    full = wl.make_batch("C3")
    return {k: (v[..., idx].copy() if v is not None else None) for k, v in full.items()}


def _check(o, g, sel, bar_all=0.95, bar_resto=0.85):
    st = o["status"]
    gs = g["IPOPT_status"][sel]
    resto = g["IPOPT_resto_iters"][sel] > 0
    assert (st == gs).mean() >= bar_all, (np.bincount(st, minlength=5), np.bincount(gs, minlength=5))
    if resto.any():
        # on the restoration instances: the status class (converged <= 1 / not converged) at
        # bar_resto; which failure IPOPT reports (max_iter 2 / failed 3 / infeasible 4) is a property of a
        # long, rounding-sensitive trajectory, so the exact code only at bar_resto - 0.1
        cls = (st <= 1) == (gs <= 1)
        assert cls[resto].mean() >= bar_resto, (st[resto], gs[resto])
        assert (st == gs)[resto].mean() >= bar_resto - 0.1, (st[resto], gs[resto])
    both = (st == 0) & (gs == 0)
    dU = np.abs(g["IPOPT_U"][..., sel] - o["U"])[:, :-1, both].max(axis=(0, 1))
    assert (dU < 1e-6).mean() >= 0.85, np.sort(dU)[-10:]
    assert (st == 0).sum() >= (gs == 0).sum() - 2
    return (st == gs).mean(), (st == gs)[resto].mean() if resto.any() else 1.0


def test_host_build_restoration_instances_vs_ipopt():
    """The emulated kernel on 8 of the sample's restoration-phase instances (CPU suite budget)."""
    g = _fix()
    sel = np.nonzero(g["IPOPT_resto_iters"] > 0)[0][:8]
    cfg = wl.CONFIGS["C3"]
    b = _batch(g["idx"][sel])
    o = ht.solve(ht.config(cfg["N"], cfg["model"], "fp64", cfg["lane"], cfg["Ts"], tol=1e-8, acceptable_tol=1e-6,
                           acceptable_iter=15), b, nthreads=8)
    _check(o, g, sel, bar_all=7 / 8, bar_resto=7 / 8)


@pytest.mark.gpu
def test_gpu_c3_sample_vs_ipopt():
    from mpcracing.batch import solver_for_config
    g = _fix()
    idx = g["idx"]
    b = _batch(idx)
    s = solver_for_config("C3", idx.size)
    o = {k: v.cpu().numpy() for k, v in s.solve(b).items()}
    a, ar = _check(o, g, np.arange(idx.size))
    print(f"C3 sample: status agreement with IPOPT {a:.3f} (restoration instances {ar:.3f}); "
          f"product {np.bincount(o['status'], minlength=5)}, IPOPT {np.bincount(g['IPOPT_status'], minlength=5)}")
