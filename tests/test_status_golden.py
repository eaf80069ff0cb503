"""The IPOPT status class at the reference's own options (the solver status class must match).

Fixture: tests/golden/status_ref_options.npz (generator tests/golden/make_status_golden.py) -- config 1 (the
reference's script/test_mpc.py instance, dynamic and kinematic model) and 64 instances each of C2, C4 and C5
drawn uniformly from the per-GPU batch, solved in fp64 by the dense IPOPT restatement under the FULL IPOPT
rules (``oracle.ipopt.IPOPT``) with control/MPC.py:152-161's options: tol 1e-4, acceptable_tol 1e-2
(acceptable_iter 15), max_iter 500.  At these options most cold starts end at IPOPT's mu floor: "acceptable"
(status 1) or a failed line search at an almost-feasible point (status 3, the reference's except branch) --
DESIGN.md §2.  Parity UNPINNED against IPOPT itself (no IPOPT / CasADi here); pinned against the restatement.

Two columns: ``IPOPT`` (the full rules) and ``PRODUCT_`` (oracle.ipopt.PRODUCT, the rule set the kernel compiles:
IPOPT's less the tiny-step termination; tests/test_rules_label.py ties it to the kernel's switches).
IPOPT's tiny-step rule (every step component below 10 eps of double relative to the variable) tests the step's
ROUNDING FLOOR at the mu floor: the oracle's dense LU leaves steps of ~1e-14 relative there (just above the
2.2e-15 threshold: C2's instance 0 logs 1.2e-14 .. 3.4e-14 for eight iterations), the product's block-tridiagonal
Riccati sweep leaves smaller ones, so with the rule compiled in the product stops where the oracle does not (host
build, fp64: C2 56 of 64 status 3 against the oracle's 1) -- which instances it ends is a property of the linear
solver's rounding, not of the algorithm, so the product keeps it off.

Bars (the product runs the same options):
  * status equal to the PRODUCT column's on >= 95 % of EVERY config's instances, fp64 and fp32 (the benchmarked
    precision; its mu-floor rules MR_F32_STALL) -- one bar, no instance excluded;
  * status equal to the full-rules IPOPT column's on >= 90 % of every config; on the instances IPOPT ends by its
    tiny-step rule (C2 1, C4 1, C5 13 of 64) the product returns IPOPT's point all the same: fp64 median |dU|
    <= 1e-6 (measured ~1e-14), fp32 <= 1e-3 -- the label differs, the controls handed to the vehicle do not;
  * where both stop at the mu floor with the same status, the returned controls are the oracle's: fp64 median
    |dU| <= 1e-6, fp32 median <= 1e-3 (fp32 rounding at the floor);
  * the full per-GPU batch's status-3 fraction lies within 4 binomial standard deviations of the fixture's
    (64 spread samples) -- the bound that replaces test_gpu.py's former unbounded status-3 allowance.
CPU tests: the host build of the kernel source (emulated wavefront) on config 1 and 16 instances of C2 / C4;
GPU tests: libmpcracing.so on every fixture instance and on the full batches.
"""
import os

import numpy as np
import pytest

import host_twin as ht
from mpcracing import workload as wl

HERE = os.path.dirname(os.path.abspath(__file__))
OPTS = dict(tol=1e-4, acceptable_tol=1e-2, acceptable_iter=15)


def _fix():
    return dict(np.load(os.path.join(HERE, "golden", "status_ref_options.npz")))


def _case(g, name, n=None):
    """(config, batch of the fixture's instances, IPOPT column, PRODUCT column) for fixture entry ``name``."""
    if name.startswith("C1"):
        cfg = dict(wl.CONFIGS["C1"], model=name[2:])
        b = wl.make_batch("C1")
        idx = np.arange(1)
    else:
        cfg = wl.CONFIGS[name]
        idx = g[f"{name}_idx"]
        full = wl.make_batch(name)
        b = {k: (v[..., idx].copy() if v is not None else None) for k, v in full.items()}
    sel = slice(0, n)
    b = {k: (v[..., sel].copy() if v is not None else None) for k, v in b.items()}
    cols = ("status", "iters", "U", "viol", "why")
    ref = {k: g[f"{name}_{k}"][..., sel] for k in cols}
    prod = {k: g[f"PRODUCT_{name}_{k}"][..., sel] for k in cols}
    return cfg, b, ref, prod


def _dU(a, b, sel):
    return np.abs(a["U"] - b["U"])[:, :-1, sel].max(axis=(0, 1))


def _check(name, prec, o, ref, prod, bar=0.95, bar_ipopt=0.90):
    st = o["status"]
    tol = 1e-6 if prec == "fp64" else 1e-3
    # the product's rule set: one bar over every instance
    agree = (st == prod["status"]).mean()
    assert agree >= bar, (name, prec, agree, np.bincount(st, minlength=5), np.bincount(prod["status"], minlength=5),
                          np.nonzero(st != prod["status"])[0])
    # the full IPOPT rules: the status on bar_ipopt, and where IPOPT stops by its tiny-step rule, the same point
    agree_i = (st == ref["status"]).mean()
    assert agree_i >= bar_ipopt, (name, prec, agree_i, np.bincount(st, minlength=5),
                                  np.bincount(ref["status"], minlength=5))
    tiny = ref["why"] == "tiny_step"
    if tiny.any():
        dU = _dU(ref, o, tiny)
        assert np.median(dU) <= tol, (name, prec, "tiny-step stops", dU)
    floor = (st == prod["status"]) & ((prod["status"] <= 1) | ((prod["status"] == 3) & (prod["viol"] <= 1e-4)))
    if floor.any():
        dU = _dU(prod, o, floor)
        assert np.median(dU) <= tol, (name, prec, np.median(dU), dU.max())
    return agree, agree_i


@pytest.mark.parametrize("name", ["C1dyn", "C1kin", "C2", "C4"])
@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_host_build_status_class(name, prec):
    cfg, b, ref, prod = _case(_fix(), name, n=16)
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    o = ht.solve(ht.config(cfg["N"], cfg["model"], prec, cfg["lane"], cfg["Ts"], **OPTS), b, tyres=tyres, nthreads=8)
    _check(name, prec, o, ref, prod, bar=15 / 16, bar_ipopt=15 / 16)


def test_fp32_stall_rule_agrees_with_fp64_on_512():
    """DESIGN.md §2's fp32-only mu-floor rules (MR_F32_STALL) give the fp64 outcome: the scalar build in fp32
    and in fp64 at the reference's options on the first 512 instances of C4 and of C5 (round-4 VERDICT weak 4:
    the former evidence was 32 + 16 instances)."""
    for name, bar in (("C4", 0.95), ("C5", 0.95)):
        cfg = wl.CONFIGS[name]
        tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
        b = wl.make_batch(name, limit=512)
        st = {}
        for prec in ("fp64", "fp32"):
            c = ht.config(cfg["N"], cfg["model"], prec, cfg["lane"], cfg["Ts"], **OPTS)
            st[prec] = ht.solve(c, b, tyres=tyres, nthreads=8, scalar=True)["status"]
        agree = (st["fp32"] == st["fp64"]).mean()
        print(f"{name}: fp32 {np.bincount(st['fp32'], minlength=5)} fp64 {np.bincount(st['fp64'], minlength=5)} "
              f"agree {agree:.3f}")
        assert agree >= bar, (name, agree)


@pytest.mark.gpu
@pytest.mark.parametrize("name", ["C1dyn", "C1kin", "C2", "C4", "C5"])
@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_gpu_status_class_vs_oracle(name, prec):
    from mpcracing.batch import BatchSolver
    cfg, b, ref, prod = _case(_fix(), name)
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    s = BatchSolver(cfg["N"], cfg["model"], prec, cfg["lane"], cfg["Ts"], max_batch=b["s0"].shape[0], tyres=tyres,
                    **OPTS)
    o = {k: v.cpu().numpy() for k, v in s.solve(b).items()}
    agree, agree_i = _check(name, prec, o, ref, prod)
    print(f"{name} {prec}: status agreement with the product's rules {agree:.3f}, with IPOPT's {agree_i:.3f}; "
          f"{np.bincount(o['status'], minlength=5)}")


def status3_band(g, name, B):
    """[lo, hi] of a per-GPU batch's status-3 count: the fixture's spread-sample fraction p +- 4 binomial
    standard deviations of a 64-instance sample (sqrt(p (1 - p) / 64)), scaled to B instances."""
    gs = g[f"{name}_status"]
    p = float((gs == 3).mean())
    sd = max(np.sqrt(p * (1 - p) / gs.size), 1.0 / gs.size)
    return max(0.0, p - 4 * sd) * B, min(1.0, p + 4 * sd) * B
