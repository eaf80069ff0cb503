"""GPU parity tests of libmpcracing.so (gfx950) through its C ABI.

Parity tolerances: fp64 solves at KKT tol 1e-10 match the oracle's
NLP solution (itself pinned to the reference's MPC.__init__, tests/test_nlp_golden.py)
to 1e-6 in controls, states (terminal column included), progress and errors, except
the last throttle U[0, N-1] (it only reaches the cost through
exp(q_v_max (vx_N - v_max)) ~ e^-60, so only the barrier fixes it) and the one
state it drives, vx_N.  fp32 solves are checked against fp64 and the oracle with
the bounds derived in DESIGN.md §4 and by full-batch feasibility properties.
"""
import math

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from mpcracing import workload as wl  # noqa: E402
from mpcracing.batch import BatchSolver, solver_for_config  # noqa: E402
from oracle import dynamics as dyn  # noqa: E402


def _np(out):
    return {k: v.cpu().numpy() for k, v in out.items()}


def test_c2_full_batch_matches_host_build():
    """Same solver source on gfx950 and on the host: identical statuses, same solutions."""
    import host_twin as ht
    cfg = wl.CONFIGS["C2"]
    b = wl.make_batch("C2")
    s = solver_for_config("C2", 1024, tol=1e-10, acceptable_iter=0)
    o = _np(s.solve(b))
    h = ht.solve(ht.config(cfg["N"], cfg["model"], "fp64", cfg["lane"], cfg["Ts"], tol=1e-10), b, nthreads=16)
    assert (o["status"] == 0).all() and (h["status"] == 0).all()
    dU = np.abs(o["U"] - h["U"])
    dU[0, -1, :] = 0.0
    assert dU.max() < 1e-6


def _defects(cfg, o, ok, tyres=None):
    """Dynamics residual F(X_k, U_k) - X_{k+1} of the returned trajectories (oracle dynamics, fp64)."""
    f = dyn.model_fn(cfg["model"])
    fns = None
    if tyres is not None:
        from oracle.nlp import pacejka_torch
        import torch as _t
        pf, pr = (pacejka_torch(a, Fz) for a, Fz in tyres)
        fns = (lambda al: float(pf(_t.tensor(float(al), dtype=_t.float64))) if al != 0 else 0.0,
               lambda al: float(pr(_t.tensor(float(al), dtype=_t.float64))) if al != 0 else 0.0)
    N = cfg["N"]
    X = o["X"][:, :, ok]
    U = o["U"][:, :, ok]
    worst = 0.0
    for k in range(N):
        x = [X[j, k] for j in range(6)]
        u = [U[0, k], U[1, k]]
        if cfg["model"] in ("kin", "dyn"):
            fk = f(x, u, cfg["Ts"])
        else:  # blended law per instance
            fk = np.stack([dyn.f_blend([X[j, k, i] for j in range(6)], [U[0, k, i], U[1, k, i]], cfg["Ts"],
                                       tyres=fns) for i in range(X.shape[2])], axis=1)
        worst = max(worst, float(np.abs(fk - X[:, k + 1]).max()))
    return worst


def _check_feasible(cfg, o, ok, tol):
    N, Ts = cfg["N"], cfg["Ts"]
    U, S = o["U"][:, :, ok], o["S"][:, ok]
    assert (U[0] >= -1 - tol).all() and (U[0] <= 0.85 + tol).all()
    assert (np.abs(U[1]) <= 0.9 + tol).all()
    dS = np.diff(S, axis=0)
    assert (dS >= 0.1 - tol).all() and (dS <= Ts * 50 + tol).all()
    dthr = U[0] - np.roll(U[0], 1, axis=0)  # i = 0 wraps to U[:, N-1] (MPC.py:142-143)
    dst = U[1] - np.roll(U[1], 1, axis=0)
    assert (dthr >= -0.4 - tol).all() and (dthr <= 2.0 + tol).all()
    assert (np.abs(dst) <= 0.2 + tol).all()


def _ipopt_outcomes(o, B, max_iter_frac, name):
    """IPOPT's outcomes at the reference's options: solved / acceptable, or -- where the
    objective scaling df is below ~1e-3, so the unscaled complementarity at IPOPT's mu floor cannot meet
    compl_inf_tol nor the acceptable level -- restoration failure at an almost-feasible point (status 3,
    the reference's except branch with opti.debug values).  The status-3 count is bounded by the oracle's
    fraction on 64 spread instances of the same batch (tests/golden/status_ref_options.npz, full IPOPT rules,
    +- 4 binomial standard deviations: test_status_golden.status3_band).  max_iter only for a small minority,
    never local infeasibility."""
    from test_status_golden import _fix, status3_band
    st = np.bincount(o["status"], minlength=5)
    assert st[2] <= max_iter_frac * B and st[4] == 0, st
    lo, hi = status3_band(_fix(), name, B)
    assert lo <= st[3] <= hi, (st, lo, hi)
    # a status-3 stop at an almost-feasible point (IPOPT's constr_viol_tol 1e-4 on the returned point's
    # unscaled violation, mr_outputs.constr_viol) vs a failed restoration: the latter only rarely
    feas3 = (o["status"] == 3) & (o["constr_viol"] <= 1e-4)
    assert ((o["status"] == 3) & ~feas3).sum() <= 0.01 * B, np.sort(o["constr_viol"][o["status"] == 3])[-10:]
    return (o["status"] <= 1) | feas3


def _host_statuses_agree(name, o, n, min_agree):
    """The GPU's fp32 statuses vs the host build of the same kernel source (emulated wavefront) on the
    first n instances: the same IPOPT decisions up to fp32 rounding (FMA contraction, hardware
    transcendentals on the GPU)."""
    import host_twin as ht
    cfg = wl.CONFIGS[name]
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    b = wl.make_batch(name, limit=n)
    h = ht.solve(ht.config(cfg["N"], cfg["model"], "fp32", cfg["lane"], cfg["Ts"], tol=1e-4, acceptable_tol=1e-2,
                           acceptable_iter=15), b, tyres=tyres, nthreads=16)
    agree = (h["status"] == o["status"][:n]).mean()
    assert agree >= min_agree, (agree, np.bincount(h["status"], minlength=5), np.bincount(o["status"][:n], minlength=5))


def test_c4_full_batch_fp32_properties():
    cfg = wl.CONFIGS["C4"]
    b = wl.make_batch("C4")
    B = b["s0"].shape[0]
    s = solver_for_config("C4", 8192)
    o = _np(s.solve(b))
    o2 = _np(s.solve(b))
    for k in o:  # deterministic: no atomics, no inter-thread communication
        assert np.array_equal(o[k], o2[k]), k
    ok = _ipopt_outcomes(o, B, 0.005, "C4")
    # solved points (tol 1e-4) may violate rows by 1e-3; acceptable points (acceptable_tol 1e-2) and the
    # almost-feasible stops by that tolerance
    _check_feasible(cfg, o, o["status"] == 0, 1e-3)
    _check_feasible(cfg, o, ok, 1e-2)
    assert _defects(cfg, {k: v[..., :512] for k, v in o.items()}, ok[:512]) < 5e-3
    _host_statuses_agree("C4", o, 128, 0.9)


def test_c3_full_batch_lane_rows():
    cfg = wl.CONFIGS["C3"]
    b = wl.make_batch("C3")
    s = solver_for_config("C3", 8192)
    o = _np(s.solve(b))
    ok = o["status"] == 0
    # hard lane rows from the reference's initial guess (S_i at top speed: far outside the lane for slow
    # cars) need IPOPT's restoration phase; >= 96.5 % solve to tol 1e-8.  The audit of the failures
    # (profiles/r04_audit_C3.json: the dense oracle under the same rules, and SLSQP) finds the oracle
    # failing too on 34 of 47 sampled (max_iter / restoration failure / the same 7 local-infeasibility
    # verdicts); the other 13 the oracle solves only after 134-477 iterations (long solves whose
    # trajectories the two linear algebras round apart)
    assert ok.mean() >= 0.965, np.bincount(o["status"], minlength=5)
    _check_feasible(cfg, o, ok, 1e-6)
    m = b["max_error"][ok]
    assert (np.abs(o["eC"][1:, ok]) <= m + 1e-6).all()  # |e_C(S_i, X_i)| <= max_error, i >= 1
    assert _defects(cfg, {k: v[..., :256] for k, v in o.items()}, ok[:256]) < 1e-7


@pytest.mark.parametrize("name", ["C4", "C5"])
def test_fp32_accuracy_vs_reference_tolerance(name):
    """fp32 (the benchmarked precision) against the exact fp64 optimum (tol 1e-10), measured against what
    the reference's own termination leaves: an fp64 solve with IPOPT's options of control/MPC.py:152-161
    (tol 1e-4, acceptable_tol 1e-2 over 15 iterations), which the fp32 solve also uses.  Bar (DESIGN.md
    §4): fp32 rounding adds essentially nothing beyond that tolerance -- the distribution of the
    per-instance control error of fp32 matches that of fp64-at-reference-tolerance (median ratio
    <= 1.2, 90th percentile <= 3: both stop somewhere inside the same tolerance region, so single
    instances scatter), and the median relative objective gap is within 1.5x (+1e-6) of it, the 90th
    percentile within 2.5x (C5's learned-tyre model: 2.0x measured), the largest within 3x -- on the instances both solves converge (status <= 1; DESIGN.md §2 for the status-3 stops)."""
    cfg = wl.CONFIGS[name]
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    n = 512
    b = wl.make_batch(name, limit=n)
    mk = lambda prec, **kw: BatchSolver(cfg["N"], cfg["model"], prec, max_batch=n, tyres=tyres, **kw)  # noqa: E731
    o64 = _np(mk("fp64", tol=1e-10, acceptable_iter=0).solve(b))
    o32 = _np(mk("fp32").solve(b))
    oref = _np(mk("fp64", tol=1e-4, acceptable_tol=1e-2, acceptable_iter=15).solve(b))
    # fp32 and fp64 under the reference's options end with the same IPOPT outcome (solved / acceptable /
    # stopped at an almost-feasible point, _ipopt_outcomes) on nearly every instance
    assert (o32["status"] == oref["status"]).mean() >= 0.9, (np.bincount(o32["status"]), np.bincount(oref["status"]))
    # accuracy where both converged (solved / acceptable): a status-3 stop is wherever the line search
    # failed at the mu floor, in fp32 as in fp64, and says nothing about fp32's accuracy
    ok = (o64["status"] == 0) & (o32["status"] <= 1) & (oref["status"] <= 1)
    assert ok.sum() >= 32, (np.bincount(o64["status"]), np.bincount(o32["status"]), np.bincount(oref["status"]))
    d32 = np.abs(o64["U"] - o32["U"])[:, :-1, ok].max(axis=(0, 1))
    dref = np.abs(o64["U"] - oref["U"])[:, :-1, ok].max(axis=(0, 1))
    ratio = d32 / np.maximum(dref, 1e-4)
    assert np.median(ratio) <= 1.2 and np.quantile(ratio, 0.9) <= 3.0, np.quantile(ratio, [0.5, 0.9, 0.99])
    for q in (0.5, 0.9):
        assert np.quantile(d32, q) <= 1.5 * np.quantile(dref, q) + 1e-4, (q, np.quantile(d32, q), np.quantile(dref, q))
    loc = lambda o: (o["obj"] + 300.0 * b["s0"])[ok]  # noqa: E731  (local objective, -lambda_s s0 removed)
    g32 = (loc(o32) - loc(o64)) / np.abs(loc(o64))
    gref = (loc(oref) - loc(o64)) / np.abs(loc(o64))
    for q, f in ((0.5, 1.5), (0.9, 2.5)):
        assert np.quantile(g32, q) <= f * np.quantile(gref, q) + 1e-6, (q, np.quantile(g32, q), np.quantile(gref, q))
    assert g32.max() <= 3.0 * gref.max() + 1e-6, (g32.max(), gref.max())
    assert np.median(g32) < 1e-4  # the objective itself: median within 1e-4 of the optimum


def test_c5_full_batch_fp32_properties():
    """C5 (blended + learned Pacejka, N = 60, fp32, the 16 384-instance shard): statuses, feasibility of every
    row, dynamics defects of the returned trajectories against the oracle's fp64 model (pacejka-2 tyres)."""
    cfg = wl.CONFIGS["C5"]
    tyres = wl.tyre_coeffs(cfg["tyres"])
    b = wl.make_batch("C5")
    assert b["s0"].shape[0] == 16384
    s = solver_for_config("C5", 16384)
    o = _np(s.solve(b))
    ok = _ipopt_outcomes(o, 16384, 0.03, "C5")
    _check_feasible(cfg, o, o["status"] == 0, 1e-3)
    _check_feasible(cfg, o, ok, 1e-2)
    assert _defects(cfg, {k: v[..., :256] for k, v in o.items()}, ok[:256], tyres=tyres) < 5e-3
    _host_statuses_agree("C5", o, 64, 0.85)


def test_dropin_mpc_class():
    """The drop-in class on config 1 (script/test_mpc.py's inputs) with the reference's IPOPT options
    (MPC.py:152-161, the class's defaults): the same IPOPT outcome as the oracle's restatement
    (tests/golden/dropin_C1.npz: restoration failure at an almost-feasible point -- the cold start's
    objective scaling df ~ 1.6e-4 leaves the unscaled complementarity at the mu floor above IPOPT's
    acceptable level) -> ``sol`` None and ``dual`` None as the reference's except branch, ``ret`` the
    oracle's final iterate (fp64, 1e-6); at tol 1e-8 the solve converges: ``sol`` set, lam_g returned.
    The failure verdict at the reference's options is pinned against the IPOPT RESTATEMENT only (parity
    unpinned against IPOPT itself: no running IPOPT / CasADi here, none of its output in the reference)."""
    import os
    from control.MPC import MPC
    from control.ControllerParameters import RuntimeControllerParameters
    from models.State import State
    g = dict(np.load(os.path.join(os.path.dirname(__file__), "golden", "dropin_C1.npz")))
    c = wl.config1_instance()
    st = State(x=171, y=91.8, yaw=-0.219, v_x=20, v_y=0.48, yaw_dot=-0.059, throttle=0.19, steer=0.63)
    args = (st, 69.6, c["cx"][:, 0].tolist(), c["cy"][:, 0].tolist(), float(c["max_error"][0]),
            RuntimeControllerParameters())
    m = MPC(*args, Ts=0.1, N=20)
    sol, ret, dual = m.solution()
    assert (sol is None) == (int(g["dyn_status"]) not in (0, 1))
    assert m.info.status == {0: "solved", 1: "acceptable", 3: "failed"}[int(g["dyn_status"])]
    States, U, S_hat, eC, eL = ret
    assert States.shape == (6, 21) and U.shape == (2, 20) and S_hat.shape == (21,)
    assert len(eC) == 20 and len(eL) == 20 and math.isclose(S_hat[0], 69.6)
    dU = np.abs(U - g["dyn_U"])
    dU[0, -1] = 0.0
    assert dU.max() < 1e-6 and np.abs(S_hat - g["dyn_S"]).max() < 1e-6
    m1 = MPC(*args, Ts=0.1, N=20, tol=1e-8, acceptable_iter=0)
    sol, ret, dual = m1.solution()
    assert sol and dual.shape == (13 * 20 + 9,)
    # warm start from the previous controls (agent.py:205 -> MPC.py:120-121)
    U = ret[1]
    lc = [(float(a), float(b_)) for a, b_ in zip(U[0], U[1])]
    m2 = MPC(*args, last_controls=lc, Ts=0.1, N=20, tol=1e-8, acceptable_iter=0)
    assert m2.solution()[0]


def test_abi_errors():
    s = BatchSolver(20, "kin", max_batch=2)
    with pytest.raises(RuntimeError):
        s.solve(wl.make_batch("C2", limit=4))  # B > max_batch
    with pytest.raises(RuntimeError):
        BatchSolver(20, "blend_pacejka", max_batch=1).solve(wl.make_batch("C2", limit=1))  # no tyres set
    # a device index the machine does not have is an error of mr_create / mr_track_create, not a silent
    # handle on whichever device is current
    ndev = torch.cuda.device_count()
    with pytest.raises(RuntimeError, match="out of range"):
        BatchSolver(20, "kin", max_batch=1, device=ndev)
    # max_iter beyond the line-search filter's capacity (mr_solver.h FCAP) is rejected, not silently truncated
    with pytest.raises(RuntimeError, match="max_iter out of range"):
        BatchSolver(20, "kin", max_batch=1, max_iter=10000)
    import ctypes
    from mpcracing import abi
    lib = abi.load_product()
    tr = ctypes.c_void_p()
    t = np.zeros(12)
    t[4:] = np.arange(1, 9)
    cx = np.ascontiguousarray(np.arange(8, dtype=np.float64))
    P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))  # noqa: E731
    assert lib.mr_track_create(ctypes.byref(tr), ndev, P(t), 12, P(cx), P(cx), 8, 8.0, None, None, 0) == -1
    assert b"out of range" in lib.mr_last_error()
    # mr_plant_step runs on the device that owns its arrays; a host pointer is rejected
    st = np.zeros((6, 4))
    assert lib.mr_plant_step(0, 4, st.ctypes.data_as(ctypes.c_void_p), st.ctypes.data_as(ctypes.c_void_p), 0.05,
                             st.ctypes.data_as(ctypes.c_void_p), None) == -1


@pytest.mark.parametrize("model", ["kin", "dyn", "blend", "blend_pacejka", "dyn_pacejka"])
def test_device_dynamics_match_host(model):
    """The generated dynamics compiled for gfx950 vs the same source on the host (fp64)."""
    import ctypes
    import host_twin as ht
    tyres = wl.tyre_coeffs("pacejka-2") if "pacejka" in model else None
    s = BatchSolver(20, model, "fp64", max_batch=1, tyres=tyres)
    rng = np.random.default_rng(3)
    n = 512
    x = np.stack([rng.normal(0, 50, n), rng.normal(0, 50, n), rng.uniform(-3, 3, n), rng.uniform(0.5, 45, n),
                  rng.normal(0, 1, n), rng.normal(0, 0.5, n)], 1)
    u = np.stack([rng.uniform(-1, 0.85, n), rng.uniform(-0.9, 0.9, n)], 1)
    nu = rng.normal(0, 10, (n, 6))
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).cuda()  # noqa: E731
    X, Uu, NU = d(x), d(u), d(nu)
    f, J, H = (torch.zeros((n, m), dtype=torch.float64, device="cuda") for m in (6, 48, 36))
    rc = s.lib.mr_eval_dynamics(s.h, n, *[ctypes.c_void_p(t.data_ptr()) for t in (X, Uu, NU, f, J, H)],
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    f2 = torch.zeros((n, 6), dtype=torch.float64, device="cuda")
    rc = s.lib.mr_eval_dynamics(s.h, n, ctypes.c_void_p(X.data_ptr()), ctypes.c_void_p(Uu.data_ptr()), None,
                                ctypes.c_void_p(f2.data_ptr()), None, None,
                                ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
    assert rc == 0
    torch.cuda.synchronize()
    np.testing.assert_allclose(f2.cpu().numpy(), f.cpu().numpy(), rtol=1e-13, atol=1e-12)  # value-only == fjh
    c = ht.config(20, model)
    P = lambda a: np.ascontiguousarray(a).ctypes.data_as(ctypes.POINTER(ctypes.c_double))  # noqa: E731
    for i in range(n):
        fo, Jo, Ho = np.zeros(6), np.zeros(48), np.zeros(36)
        ht.lib().mrh_eval_dynamics(ctypes.byref(c), P(tyres[0][0]) if tyres else None, tyres[0][1] if tyres else 0.0,
                                   P(tyres[1][0]) if tyres else None, tyres[1][1] if tyres else 0.0,
                                   P(x[i]), P(u[i]), P(nu[i]), P(fo), P(Jo), P(Ho))
        np.testing.assert_allclose(f[i].cpu().numpy(), fo, rtol=1e-13, atol=1e-12)
        np.testing.assert_allclose(J[i].cpu().numpy(), Jo, rtol=1e-11, atol=1e-11)
        np.testing.assert_allclose(H[i].cpu().numpy(), Ho, rtol=1e-9, atol=1e-9 * max(1, np.abs(Ho).max()))


def test_c4_fp64_gpu_vs_host_statuses():
    import host_twin as ht
    b = wl.make_batch("C4", limit=64)
    s = BatchSolver(40, "blend", "fp64", max_batch=64, acceptable_iter=0)
    o = _np(s.solve(b))
    h = ht.solve(ht.config(40, "blend", "fp64", tol=1e-8), b, nthreads=16)
    print("gpu status", o["status"].tolist(), "iters", o["iters"].tolist())
    print("host status", h["status"].tolist(), "iters", h["iters"].tolist())
    print("gpu kkt", o["kkt"].tolist())
    assert (o["status"] == h["status"]).all()


def test_dispatch_order_does_not_change_results():
    """mr_config.dispatch_order = 1 (the three-tier long-solves-first permutation of the workgroups,
    mr_order_kernel) must give bit-identical outputs to index order: every instance solved exactly once,
    by the same code, on the same inputs."""
    b = wl.make_batch("C4", limit=3000)  # not a multiple of the order kernel's 1024 threads
    o0 = _np(solver_for_config("C4", 3000, dispatch_order=0).solve(b))
    o1 = _np(solver_for_config("C4", 3000, dispatch_order=1).solve(b))
    for k in o0:
        assert np.array_equal(o0[k], o1[k]), k


def test_dispatch_order_hint_does_not_change_results():
    """mr_config.dispatch_order = 2 (longest-expected-first by mr_inputs.order_hint, mr_order_hint_kernel):
    bit-identical outputs to index order, with a real hint (the iterations of a first solve, as the
    closed loop passes the previous tick's), with out-of-range hints (clamped buckets), with a uniform
    (all-zero) hint (instance order), and without a hint -- on a fresh handle (no previous solve: instance
    order) and on a handle that solved this batch size before (its stored iterations are the hint)."""
    import torch
    b = wl.make_batch("C4", limit=3000)
    o0 = _np(solver_for_config("C4", 3000, dispatch_order=0).solve(b))
    s2 = solver_for_config("C4", 3000, dispatch_order=2)
    rng = np.random.default_rng(7)
    for hint in (o0["iters"].astype(np.int32), rng.integers(-50, 5000, 3000).astype(np.int32),
                 np.zeros(3000, np.int32)):
        o2 = _np(s2.solve(dict(b, order_hint=hint)))
        for k in o0:
            assert np.array_equal(o0[k], o2[k]), k
    s3 = solver_for_config("C4", 3000, dispatch_order=2)
    for _ in range(2):  # first call: no stored iterations (instance order); second: the first call's iterations
        o3 = _np(s3.solve(b))
        for k in o0:
            assert np.array_equal(o0[k], o3[k]), k
    with pytest.raises(ValueError):
        s2.solve(dict(b, order_hint=torch.zeros(5, dtype=torch.int32)))


def test_concurrent_handles_on_streams_match_serial():
    """bench.py's serving-mode figure: independent handles (own workspaces) launched on separate HIP
    streams while each other's solves are in flight give bit-identical results to one handle solving the
    batch alone (no shared state between handles, mpcracing.hip mr_create)."""
    b = wl.make_batch("C4", limit=2048)
    ref = _np(solver_for_config("C4", 2048).solve(b))
    hs = [solver_for_config("C4", 2048) for _ in range(3)]
    ins = [h.to_device(b) for h in hs]
    outs = [h.alloc_outputs(2048) for h in hs]
    streams = [torch.cuda.Stream() for _ in hs]
    for _ in range(2):
        for h, i, o, st in zip(hs, ins, outs, streams):
            h.launch(i, o, st)
    torch.cuda.synchronize()
    for o in outs:
        o = _np(o)
        for k in ref:
            assert np.array_equal(ref[k], o[k]), k


@pytest.mark.parametrize("name,precision,n", [("C5", "fp64", 512), ("C5", "fp32", 2048), ("C4", "fp32", 2048),
                                              ("C3", "fp64", 1024)])
def test_repeated_solves_are_bitwise_identical(name, precision, n):
    """The same batch solved three times on one handle (each solve starting on the previous one's workspace
    and LDS leftovers) and once on a fresh handle returns bitwise-identical outputs.  Guards the run-to-run
    nondeterminism of fp64 C5 found in round 6 (second-order-correction steps differing in their last bits
    from solve to solve, tools/determinism_probe.py)."""
    b = wl.make_batch(name, limit=n)
    s = solver_for_config(name, n, precision=precision)
    ref = _np(s.solve(b))
    outs = [_np(s.solve(b)) for _ in range(2)] + [_np(solver_for_config(name, n, precision=precision).solve(b))]
    for o in outs:
        for k in ref:
            assert np.array_equal(ref[k], o[k], equal_nan=True), (k, np.nonzero(np.any(
                (ref[k] != o[k]).reshape(-1, n), axis=0))[0][:16])
