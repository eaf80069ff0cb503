"""The IPOPT status class at the reference's own options (the solver status class must match).

Fixture: tests/golden/status_ref_options.npz (generator tests/golden/make_status_golden.py) -- config 1 (the
reference's script/test_mpc.py instance, dynamic and kinematic model) and 64 instances each of C2, C4 and C5
drawn uniformly from the per-GPU batch, solved in fp64 by the dense IPOPT restatement under the FULL IPOPT
rules (``oracle.ipopt.IPOPT``) with control/MPC.py:152-161's options: tol 1e-4, acceptable_tol 1e-2
(acceptable_iter 15), max_iter 500.  At these options most cold starts end at IPOPT's mu floor: "acceptable"
(status 1) or a failed line search at an almost-feasible point (status 3, the reference's except branch) --
DESIGN.md §2.  Parity UNPINNED against IPOPT itself (no IPOPT / CasADi here); pinned against the restatement.

Bars (the product runs the same options):
  * status equal to the oracle's on >= 90 % of the instances of every config, in fp64 AND in fp32 (the
    benchmarked precision; its mu-floor rules MR_F32_STALL), and on >= 95 % of those the oracle
    does not end by IPOPT's tiny-step rule.  That rule (every step component below 10 eps of double relative
    to the variable) tests the step's ROUNDING FLOOR at the mu floor: the oracle's dense LU leaves steps of
    ~1e-14 relative there (just above the 2.2e-15 threshold: C2's instance 0 logs 1.2e-14 .. 3.4e-14 for
    eight iterations), the product's block-tridiagonal Riccati sweep leaves smaller ones, so with the rule on
    the product stops where the oracle does not (host build, fp64: C2 56 of 64 status 3 against the
    oracle's 1) -- the product keeps the rule off (mr_solver.h MR_TINY_STEP).  The oracle's
    tiny-step stops (C2 1, C4 1, C5 13 of 64) the product then ends either by its own failed line search at
    the floor (status 3, C5: 8 of 13) or as acceptable (C5: 5 of 13, C2: instance 146) -- measured host build
    and GPU alike: 100 % agreement on every other instance;
  * where both stop at the mu floor with the same status, the returned controls are the oracle's: fp64 median
    |dU| <= 1e-6 (measured ~1e-14: the same point), fp32 median <= 1e-3 (fp32 rounding at the floor);
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
    """(config, batch of the fixture's instances, fixture slice) for fixture entry ``name``."""
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
    ref = {k: g[f"{name}_{k}"][..., sel] for k in ("status", "iters", "U", "viol", "why")}
    return cfg, b, ref


def _check(name, prec, o, ref, bar=0.95, bar_all=0.90):
    st, gs = o["status"], ref["status"]
    agree = (st == gs).mean()
    assert agree >= bar_all, (name, prec, agree, np.bincount(st, minlength=5), np.bincount(gs, minlength=5))
    # the oracle's tiny-step stops are a coin flip at the step's rounding floor (module docstring): the
    # strict bar applies to the instances the oracle ends by any other rule
    nt = ref["why"] != "tiny_step"
    agree_nt = (st == gs)[nt].mean()
    assert agree_nt >= bar, (name, prec, agree_nt, np.nonzero((st != gs) & nt)[0], st[(st != gs) & nt])
    floor = (st == gs) & ((gs == 1) | ((gs == 3) & (ref["viol"] <= 1e-4)) | (gs == 0))
    if floor.any():
        dU = np.abs(ref["U"] - o["U"])[:, :-1, floor].max(axis=(0, 1))
        assert np.median(dU) <= (1e-6 if prec == "fp64" else 1e-3), (name, prec, np.median(dU), dU.max())
    return agree


@pytest.mark.parametrize("name", ["C1dyn", "C1kin", "C2", "C4"])
@pytest.mark.parametrize("prec", ["fp64", "fp32"])
def test_host_build_status_class(name, prec):
    cfg, b, ref = _case(_fix(), name, n=16)
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    o = ht.solve(ht.config(cfg["N"], cfg["model"], prec, cfg["lane"], cfg["Ts"], **OPTS), b, tyres=tyres, nthreads=8)
    _check(name, prec, o, ref, bar=15 / 16, bar_all=15 / 16)


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
    cfg, b, ref = _case(_fix(), name)
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    s = BatchSolver(cfg["N"], cfg["model"], prec, cfg["lane"], cfg["Ts"], max_batch=b["s0"].shape[0], tyres=tyres,
                    **OPTS)
    o = {k: v.cpu().numpy() for k, v in s.solve(b).items()}
    agree = _check(name, prec, o, ref)
    print(f"{name} {prec}: status agreement {agree:.3f}, {np.bincount(o['status'], minlength=5)}")


def status3_band(g, name, B):
    """[lo, hi] of a per-GPU batch's status-3 count: the fixture's spread-sample fraction p +- 4 binomial
    standard deviations of a 64-instance sample (sqrt(p (1 - p) / 64)), scaled to B instances."""
    gs = g[f"{name}_status"]
    p = float((gs == 3).mean())
    sd = max(np.sqrt(p * (1 - p) / gs.size), 1.0 / gs.size)
    return max(0.0, p - 4 * sd) * B, min(1.0, p + 4 * sd) * B
