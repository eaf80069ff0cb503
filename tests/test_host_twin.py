"""CPU checks of the product's solver source through its host (g++) build:
generated analytic derivatives vs torch autograd of the oracle dynamics, the
Pacejka jets, and full solves vs the oracle NLP solver (small cases)."""
import ctypes
import json
import os

import numpy as np
import pytest
import torch

import host_twin as ht
from mpcracing import workload as wl
from oracle import dynamics as dyn
from oracle.ipopt import PRODUCT, solve_ipopt
from oracle.nlp import MPCProblem, pacejka_torch

HERE = os.path.dirname(os.path.abspath(__file__))
GJ = json.load(open(os.path.join(HERE, "golden", "golden.json")))
TY = GJ["tyres"]["pacejka-2"]
TYRES = ((TY["front_tire.a"], TY["front_tire.Fz"][0]), (TY["back_tire.a"], TY["back_tire.Fz"][0]))
P = lambda a: np.ascontiguousarray(a, np.float64).ctypes.data_as(ctypes.POINTER(ctypes.c_double))  # noqa: E731


def _torch_model(model):
    M = dyn._torch_ns()
    tyres = None
    if "pacejka" in model:
        tyres = (pacejka_torch(*TYRES[0]), pacejka_torch(*TYRES[1]))

    def f(v, Ts=0.05):
        x, u = [v[i] for i in range(6)], [v[6], v[7]]
        if model == "kin":
            return dyn.f_vehicle_kinematic(x, u, Ts, M)
        fd = dyn.f_vehicle(x, u, Ts, M, tyres)
        if model in ("dyn", "dyn_pacejka"):
            return fd
        fk = dyn.f_vehicle_kinematic(x, u, Ts, M)
        vel = torch.sqrt(v[3] ** 2 + v[4] ** 2)
        lo, hi = dyn.VP.Vblendmin, dyn.VP.Vblendmax
        lam = torch.where(vel <= lo, torch.zeros_like(vel),
                          torch.where(vel >= hi, torch.ones_like(vel), (vel - lo) / (hi - lo)))
        return lam * fd + (1 - lam) * fk
    return f


@pytest.mark.parametrize("model", ["kin", "dyn", "blend", "blend_pacejka", "dyn_pacejka"])
def test_generated_derivatives_match_autograd(model):
    rng = np.random.default_rng(7)
    c = ht.config(20, model)
    f = _torch_model(model)
    for trial in range(12):
        vx = [1.5, 8.0, 25.0][trial % 3]  # kinematic / blend / dynamic regions of the blended law
        x = np.array([rng.normal(100, 50), rng.normal(-20, 50), rng.uniform(-3, 3), vx,
                      rng.normal(0, 1), rng.normal(0, 0.5)])
        u = np.array([rng.uniform(-1, 0.85), rng.uniform(-0.9, 0.9)])
        nu = rng.normal(0, 10, 6)
        fo, J, H = np.zeros(6), np.zeros(48), np.zeros(36)
        tyr = TYRES if "pacejka" in model else None
        rc = ht.lib().mrh_eval_dynamics(ctypes.byref(c), P(tyr[0][0]) if tyr else None, tyr[0][1] if tyr else 0.0,
                                        P(tyr[1][0]) if tyr else None, tyr[1][1] if tyr else 0.0,
                                        P(x), P(u), P(nu), fo.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                        J.ctypes.data_as(ctypes.POINTER(ctypes.c_double)),
                                        H.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        assert rc == 0
        v = torch.tensor(np.concatenate([x, u]))
        fr = f(v).numpy()
        Jr = torch.func.jacrev(f)(v).numpy()
        Hr = torch.func.hessian(lambda w: torch.dot(torch.tensor(nu), f(w)))(v).numpy()
        Hp = np.zeros((8, 8))
        q = 0
        for a in range(8):
            for b in range(a, 8):
                Hp[a, b] = Hp[b, a] = H[q]
                q += 1
        np.testing.assert_allclose(fo, fr, rtol=1e-13, atol=1e-11)
        np.testing.assert_allclose(J.reshape(6, 8), Jr, rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(Hp, Hr, rtol=1e-8, atol=1e-8 * max(1.0, np.abs(Hr).max()))


@pytest.mark.parametrize("coef", ["pacejka-1", "pacejka-2", "vehicle_default_Fz1"])
def test_pacejka_jet(coef):
    if coef == "vehicle_default_Fz1":
        # the initial coefficients of learning/vehicle.py:75 at a small load: |B*alpha| ~ 1 exercises
        # the non-series branch
        a, Fz = [1.3, -22.1, 1011, 1078, 1.82, 0.208, 0.0, -0.354, 0.707], 1.0
    else:
        t = GJ["tyres"][coef]
        a, Fz = t["front_tire.a"], t["front_tire.Fz"][0]
    fy = pacejka_torch(a, Fz)
    for al in [-0.3, -0.02, 1e-5, 0.07, 0.25]:
        out = np.zeros(3)
        ht.lib().mrh_pacejka(P(a), Fz, al, 0, out.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        t = torch.tensor(al, dtype=torch.float64)
        d1 = torch.func.grad(fy)(t)
        d2 = torch.func.grad(torch.func.grad(fy))(t)
        ref = np.array([float(fy(t)), float(d1), float(d2)])
        np.testing.assert_allclose(out, ref, rtol=1e-9, atol=1e-9 * max(1.0, abs(ref[1])))
        out32 = np.zeros(3)
        ht.lib().mrh_pacejka(P(a), Fz, al, 1, out32.ctypes.data_as(ctypes.POINTER(ctypes.c_double)))
        assert abs(out32[0] - ref[0]) <= 2e-6 * max(1.0, abs(ref[0]))  # fp32 form is usable (naive is not)


def _compare(name, n, tol=1e-10, parity=1e-6):
    cfg = wl.CONFIGS[name]
    b = wl.make_batch(name, limit=n)
    c = ht.config(cfg["N"], cfg["model"], "fp64", cfg["lane"], cfg["Ts"], tol=tol)
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    out = ht.solve(c, b, tyres=tyres)
    assert (out["status"] == 0).all(), out["status"]
    for i, inst in enumerate(wl.instance_dicts(b)):
        p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=cfg["N"],
                       Ts=cfg["Ts"], model=cfg["model"], lane_bounds=cfg["lane"], tyres=tyres,
                       )
        r = solve_ipopt(p, tol=1e-10, max_iter=1000, acceptable_iter=0, rules=PRODUCT)
        assert r.status == 0
        X, U, S, eC, eL = p.unpack(r.w)
        dU = np.abs(U - out["U"][:, :, i])
        dU[0, -1] = 0.0  # last throttle: cost-insensitive direction, fixed by the barrier only
        assert dU.max() < parity, (i, dU.max())
        assert np.abs(X[:, :-1] - out["X"][:, :-1, i]).max() < parity
        assert np.abs(np.delete(X[:, -1], 3) - np.delete(out["X"][:, -1, i], 3)).max() < parity
        assert np.abs(S - out["S"][:, i]).max() < parity
        assert np.abs(eC - out["eC"][:, i]).max() < parity and np.abs(eL - out["eL"][:, i]).max() < parity
        assert abs(r.obj - out["obj"][i]) <= 1e-8 * max(1.0, abs(r.obj))


def test_config1_dynamic_and_kinematic_vs_oracle():
    """C1: script/test_mpc.py inputs (N = 20, Ts = 0.1), reference dynamic NLP and kinematic variant."""
    b = wl.make_batch("C1")
    inst = wl.instance_dicts(b)[0]
    for model in ("dyn", "kin"):
        c = ht.config(20, model, "fp64", False, 0.1, tol=1e-10)
        out = ht.solve(c, b)
        assert out["status"][0] == 0
        p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=20, Ts=0.1,
                       model=model)
        r = solve_ipopt(p, tol=1e-10, max_iter=1000, acceptable_iter=0, rules=PRODUCT)
        X, U, S, eC, eL = p.unpack(r.w)
        dU = np.abs(U - out["U"][:, :, 0])
        dU[0, -1] = 0.0
        assert dU.max() < 1e-6 and np.abs(S - out["S"][:, 0]).max() < 1e-6
        # the wrap-around rate row of MPC.py:142-143 is active at this solution: U1_0 - U1_{N-1} = 0.2
        assert abs((out["U"][1, 0, 0] - out["U"][1, -1, 0]) - 0.2) < 1e-6


def test_c2_kinematic_vs_oracle():
    _compare("C2", 3)


def _golden(name):
    return dict(np.load(os.path.join(HERE, "golden", f"solutions_{name}.npz")))


def _vs_golden(name, idx, scalar, parity=1e-6, trace=False):
    """Host build (wave emulation or scalar) on instances idx of the config vs the oracle's IPOPT solutions."""
    g = _golden(name)
    cfg = wl.CONFIGS[name]
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    full = wl.make_batch(name, limit=max(idx) + 1)
    b = {k: (v[..., idx].copy() if v is not None else None) for k, v in full.items()}
    c = ht.config(cfg["N"], cfg["model"], "fp64", cfg["lane"], cfg["Ts"], tol=1e-10)
    N = cfg["N"]
    outs = []
    for j, i in enumerate(idx):
        o = ht.solve(c, b, tyres=tyres, nthreads=8, scalar=scalar, trace_instance=j if trace else -1,
                     trace_cap=600 if trace else 0)
        assert o["status"][j] == 0, (i, o["status"][j])
        dU = np.abs(g["U"][..., i] - o["U"][..., j])
        dU[0, N - 1] = 0.0  # last throttle: cost-insensitive direction, fixed by the barrier only
        dX = np.abs(g["X"][..., i] - o["X"][..., j])
        dX[3, N] = 0.0
        assert dU.max() < parity and dX.max() < parity, (i, dU.max(), dX.max())
        assert np.abs(g["S"][:, i] - o["S"][:, j]).max() < parity
        assert np.abs(g["eC"][:, i] - o["eC"][:, j]).max() < parity and np.abs(g["eL"][:, i] - o["eL"][:, j]).max() < parity
        assert abs(g["obj"][i] - o["obj"][j]) <= 1e-8 * max(1.0, abs(g["obj"][i]))
        outs.append(o)
        if not trace:
            break  # one solve covers the whole subset
    return outs


@pytest.mark.parametrize("scalar", [False, True])
def test_c3_restoration_phase_vs_oracle(scalar):
    """Hard lane rows (the commented MPC.py:135) from the reference's initial guess: instances 0 and 1
    of C3 start far outside the lane (S_i = s0 + i Ts v_max, MPC.py:127, for a slow car), the filter line
    search fails, and IPOPT's restoration phase takes over -- in the oracle's dense restatement (2 and 1
    restoration iterations, tests/golden/solutions_C3.npz) and in both host builds of the product,
    which must enter it (trace marker -300) and end at the oracle's solution."""
    for o in _vs_golden("C3", [0, 1], scalar, trace=True):
        col = o["trace"][:, 7]
        assert (col == -300).any(), "restoration phase not entered"
        assert ((col <= -200) & (col > -300)).any()  # at least one restoration-phase step (-200 - trials)


def test_c2_vs_golden_wave_twin():
    _vs_golden("C2", list(range(4)), scalar=False)


@pytest.mark.slow
def test_c4_c5_fp64_vs_golden():
    _vs_golden("C4", [0, 1], scalar=False)
    _vs_golden("C5", [0], scalar=False)


def test_fp32_close_to_fp64():
    """fp32 and fp64 under the same options (the reference's tol 1e-4 / acceptable 1e-2 / 15) end with the
    same IPOPT status on >= 90 % of a C4 sample -- about half of them status 3: with C4's objective scaling
    (df ~ 1e-3) the unscaled complementarity at IPOPT's mu floor stays above compl_inf_tol and the
    acceptable level, the iterate stalls at an almost-feasible point and IPOPT ends in restoration failure
     -- and where both converge the controls agree to 5e-2 (median 1e-3)."""
    b = wl.make_batch("C4", limit=16)
    o64 = ht.solve(ht.config(40, "blend", "fp64", tol=1e-4, acceptable_iter=15, acceptable_tol=1e-2), b)
    o32 = ht.solve(ht.config(40, "blend", "fp32", tol=1e-4, acceptable_iter=15, acceptable_tol=1e-2), b)
    assert (o64["status"] == o32["status"]).mean() >= 0.9, (o64["status"], o32["status"])
    assert set(np.unique(o32["status"])) <= {0, 1, 3}
    ok = (o64["status"] <= 1) & (o32["status"] <= 1)
    assert ok.sum() >= 4
    dU = np.abs(o32["U"] - o64["U"])[:, :-1, ok]
    assert np.median(dU) < 1e-3 and dU.max() < 5e-2


def test_second_order_corrections_wave_matches_scalar():
    """IPOPT's linear second-order corrections (up to 4 per line search, continued while theta falls by
    kappa_soc) take the same decisions in the emulated wave kernel as in the scalar solver: C4 instance
    4765 at the reference's options in fp64 (a long solve at mu 2.8e-3 whose line searches reject the
    full step and correct it) -- every iteration's kkt, mu, alpha, delta, theta, phi and marker equal to
    1e-6 over 150 iterations, with corrections accepted (marker >= 100)."""
    cfg = wl.CONFIGS["C4"]
    i = 4765
    b = wl.make_batch("C4", limit=i + 1)
    sub = {k: (v[..., i:i + 1].copy() if v is not None else None) for k, v in b.items()}
    c = ht.config(cfg["N"], cfg["model"], "fp64", cfg["lane"], cfg["Ts"], tol=1e-4, acceptable_iter=15,
                  acceptable_tol=1e-2, max_iter=150)
    a = ht.solve(c, sub, nthreads=1, scalar=True, trace_instance=0, trace_cap=200)
    w = ht.solve(c, sub, nthreads=1, scalar=False, trace_instance=0, trace_cap=200)
    n = int(a["iters"][0])
    assert int(w["iters"][0]) == n and int(w["status"][0]) == int(a["status"][0])
    ta, tw = a["trace"][:n], w["trace"][:n]
    assert (ta[:, 7] >= 100).sum() >= 5  # corrections accepted
    np.testing.assert_array_equal(ta[:, 7], tw[:, 7])
    np.testing.assert_allclose(tw[:, :7], ta[:, :7], rtol=1e-6, atol=1e-12)


def test_max_iter_beyond_filter_capacity_rejected():
    """A max_iter the line-search filter cannot hold (mr_solver.h FCAP) is an error of the solve call (the GPU
    library's mr_create rejects it too, test_gpu.py::test_abi_errors), not a silent loss of filter entries."""
    b = wl.make_batch("C2", limit=1)
    for scalar in (False, True):
        with pytest.raises(AssertionError):
            ht.solve(ht.config(20, "kin", max_iter=10000), b, nthreads=1, scalar=scalar)


def test_restoration_exit_reports_the_restoration_iterate_objective():
    """A solve that ends inside the restoration phase (C3 instance 706 of tests/golden/c3_sample_ipopt.npz, IPOPT's
    local infeasibility there) returns the restoration iterate; its reported objective is the reference's
    objective (control/MPC.py:84-98) at exactly that returned point, not the last regular iteration's."""
    from oracle.nlp import MPCProblem
    import torch
    cfg = wl.CONFIGS["C3"]
    i = 706
    b = wl.make_batch("C3", limit=i + 1)
    sub = {k: (v[..., i:i + 1].copy() if v is not None else None) for k, v in b.items()}
    for scalar in (False, True):
        o = ht.solve(ht.config(cfg["N"], cfg["model"], "fp64", cfg["lane"], cfg["Ts"], tol=1e-8, acceptable_tol=1e-6,
                               acceptable_iter=15), sub, nthreads=1, scalar=scalar, trace_instance=0, trace_cap=520)
        # the emulated wave ends with IPOPT's local infeasibility (4), the scalar build with restoration failure
        # (3); both inside the restoration phase (trace code <= -200: a restoration iteration)
        it = o["iters"][0]
        assert o["status"][0] in (3, 4) and o["trace"][it - 1, 7] <= -200, (o["status"], o["trace"][it - 1])
        inst = wl.instance_dicts(b)[i]
        p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=cfg["N"],
                       Ts=cfg["Ts"], model=cfg["model"], lane_bounds=cfg["lane"])
        w = np.concatenate([o["U"][:, :, 0].ravel(), o["S"][:, 0], o["X"][:, :, 0].ravel()])
        f = float(p.f(torch.tensor(w)))
        np.testing.assert_allclose(o["obj"][0], f, rtol=1e-9, atol=1e-9)
