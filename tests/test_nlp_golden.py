"""The oracle NLP pinned to the reference's own MPC.__init__.

Fixtures: tests/golden/make_nlp_golden.py ran the reference's control/MPC.py in
the build container with a recording casadi stand-in (tests/golden/casadi_standin.py)
and stored, per case and evaluation point, the objective J (MPC.py:86-98), every
constraint row in Opti call order with its bounds (MPC.py:101-149), the initial
guess (MPC.py:109-131) and the ret tuple (MPC.py:166-170); plus G6 (f_vehicle,
f_vehicle_kinematic, Fx, steer_cmd_to_angle at 1000 seeded points, MPC.py:186-283)
and G9b (Pacejka.forward in float64, learning/vehicle.py:79-92).

Tolerances: the model pieces are the same fp64 operations in the same order, so G6
is compared at 1e-13 relative.  The oracle evaluates the global-s centerline
quartic after an exact Taylor shift to sigma = s - s0 (oracle/nlp.py ``errors``);
the reference evaluates it in global s, where its own rounding is
~eps * sum_j |c_j| s^j (~1e-9 m at s ~ 1e3).  Rows and ret values that depend on the
polynomial are therefore compared against that bound, computed per case.
"""
import json
import os

import numpy as np
import pytest
import torch

from oracle import dynamics as dyn
from oracle.nlp import MPCProblem, solve_ipm, solve_slsqp, kkt_residuals

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "nlp_golden.npz"))
META = json.load(open(os.path.join(HERE, "golden", "nlp_golden.json")))
CASES = {c["name"]: c for c in META["cases"]}
EPS = np.finfo(np.float64).eps


def _problem(c):
    st = c["state0"]
    names = ["x", "y", "yaw", "v_x", "v_y", "yaw_dot", "throttle", "steer"]
    return MPCProblem({n: v for n, v in zip(names, st)}, c["s0"], c["cx"], c["cy"], c["max_error"], N=c["N"],
                      Ts=c["Ts"], model=c["model"], last_controls=c.get("last_controls"))


def _w(key):
    return np.concatenate([G[key + "U"].reshape(-1), G[key + "S"], G[key + "X"].reshape(-1)])


def _poly_noise(c, S):
    """Rounding bound of the reference's global-s polynomial and its derivative at S."""
    s = np.abs(np.asarray(S))
    tot = 0.0
    for coeffs in (c["cx"], c["cy"]):
        a = np.abs(np.asarray(coeffs[::-1]))
        val = sum(a[j] * s ** j for j in range(5))
        der = sum(j * a[j] * s ** (j - 1) for j in range(1, 5))
        tot = np.maximum(tot, 8 * EPS * (val + der * 10.0))
    return tot


def test_g6_model_pieces():
    x, u, Ts = G["g6_x"], G["g6_u"], G["g6_Ts"]
    fd = np.array([dyn.f_vehicle(x[i], u[i], Ts[i]) for i in range(len(Ts))])
    fk = np.array([dyn.f_vehicle_kinematic(x[i], u[i], Ts[i]) for i in range(len(Ts))])
    np.testing.assert_allclose(fd, G["g6_fdyn"], rtol=1e-13, atol=1e-12)
    np.testing.assert_allclose(fk, G["g6_fkin"], rtol=1e-13, atol=1e-12)
    assert np.array_equal([dyn.Fx(u[i, 0], x[i, 3]) for i in range(len(Ts))], G["g6_Fx"])
    assert np.array_equal([dyn.steer_cmd_to_angle(u[i, 1], x[i, 3], x[i, 4]) for i in range(len(Ts))],
                          G["g6_delta"])


@pytest.mark.parametrize("name", ["pacejka-1", "pacejka-2"])
def test_g9b_pacejka_forward(name):
    """The reference's Pacejka.forward in float64 equals oracle.dynamics.pacejka_naive bit for bit;
    the cancellation-free oracle form (pacejka_torch, exact to 1e-12 vs mpmath in
    test_oracle_golden.py) agrees with it within the naive form's own rounding,
    4 eps |E| |alpha| |BCD| (|E| ~ 1e9..6e10 makes that up to ~1 N)."""
    import math
    from oracle.nlp import pacejka_torch
    gj = json.load(open(os.path.join(HERE, "golden", "golden.json")))
    al = G["g9b_alpha"]
    for side in ("front_tire", "back_tire"):
        t = gj["tyres"][name]
        a, Fz = t[side + ".a"], t[side + ".Fz"][0]
        ref = G[f"g9b_{name}_{side}"]
        assert np.array_equal([dyn.pacejka_naive(x, a, Fz) for x in al], ref)
        fy = pacejka_torch(a, Fz)
        mine = np.array([float(fy(torch.tensor(x, dtype=torch.float64))) if x != 0 else 0.0 for x in al])
        E = a[6] * Fz ** 2 + a[7] * Fz + a[8]
        BCD = a[3] * math.sin(a[4] * math.atan(a[5] * Fz))
        bound = 4 * EPS * abs(E) * np.abs(al) * abs(BCD) + 1e-9
        assert np.all(np.abs(mine - ref) <= bound), np.abs(mine - ref).max()


@pytest.mark.parametrize("name", list(CASES))
def test_initial_guess(name):
    c = CASES[name]
    p = _problem(c)
    w = p.initial_guess()
    ref = np.concatenate([G[name + "/init_U"].reshape(-1), G[name + "/init_S"], G[name + "/init_X"].reshape(-1)])
    np.testing.assert_allclose(w, ref, rtol=1e-13, atol=1e-12)


@pytest.mark.parametrize("name", list(CASES))
@pytest.mark.parametrize("pt", [0, 1, 2])
def test_objective_rows_ret(name, pt):
    c = CASES[name]
    p = _problem(c)
    key = f"{name}/p{pt}/"
    w = _w(key)
    U, S, X = G[key + "U"], G[key + "S"], G[key + "X"]
    # rows in Opti order, with bounds
    g, lo, hi = p.opti_rows(w)
    assert len(g) == c["n_rows"] == c["n_dual"]
    if c["state0"][6] is not None and c["state0"][7] is not None:
        assert len(g) == 13 * c["N"] + 9
    assert np.array_equal(lo, G[key + "lbg"]) and np.array_equal(hi, G[key + "ubg"])
    np.testing.assert_allclose(g, G[key + "g"], rtol=1e-13, atol=1e-11)
    # ret tuple (e_hat rows use the polynomial: bound by the reference's own rounding)
    Xo, Uo, So, eC, eL = p.unpack(w)
    assert np.array_equal(Xo, G[key + "ret_X"]) and np.array_equal(Uo, G[key + "ret_U"])
    assert np.array_equal(So, G[key + "ret_S"])
    tol = _poly_noise(c, S[:-1]) * (1 + np.abs(X[0, :-1]) + np.abs(X[1, :-1]))
    assert np.all(np.abs(eC - G[key + "ret_eC"]) <= tol + 1e-12)
    assert np.all(np.abs(eL - G[key + "ret_eL"]) <= tol + 1e-12)
    # objective: term-wise bound on the polynomial rounding
    J = float(p.f(torch.tensor(w)))
    Jr = float(G[key + "J"])
    eCa = np.abs(np.concatenate([eC, [0.0]])) + 1.0
    bound = 1e-13 * abs(Jr) + float(np.sum(2 * (1000 + 500) * eCa * _poly_noise(c, S) * 10))
    assert abs(J - Jr) <= bound, (J, Jr, bound)


def test_row_structure_c1():
    c = CASES["C1_dyn"]
    N = c["N"]
    # subject_to calls: S0, 6 x X0, then per i: dynamics (6 rows), Delta-S; then per i: 6 control rows
    # (4 comparisons + 2 bounded), then the two state0 rows
    calls = c["row_of_call"]
    assert calls[:7] == list(range(7))
    assert len(calls) == 7 + 2 * N + 6 * N + 2
    assert c["ipopt_options"] == {"max_iter": 500, "print_level": 4, "tol": 1e-4, "acceptable_tol": 1e-2,
                                  "warm_start_init_point": "no", "check_derivatives_for_naninf": "yes"}


@pytest.mark.parametrize("name,start", [("C1_kin", "init"), ("C1_dyn", "near"), ("C2_0", "near")])
def test_slsqp_crosscheck(name, start):
    """The oracle's IPM and scipy SLSQP (independent algorithm) reach the same local optimum of
    the pinned NLP; the IPM point satisfies KKT to 1e-8.  SLSQP starts from the reference's
    initial guess where it converges from there (C1 kinematic); on the dynamic-model cases it
    hits its iteration limit from that start, so it starts from the IPM optimum with the controls
    and progress perturbed by 1e-2 and the states re-rolled (it must return to the same point)."""
    c = CASES[name]
    p = _problem(c)
    r = solve_ipm(p, tol=1e-10)
    assert r.status == 0
    k = kkt_residuals(p, r.w, r.nu, r.lam)
    assert k["stat"] < 1e-6 and k["eq"] < 1e-9 and k["ineq"] < 1e-9, k
    w0 = None
    if start == "near":
        rng = np.random.default_rng(5)
        N = c["N"]
        w0 = r.w.copy()
        w0[:3 * N + 1] += 1e-2 * rng.standard_normal(3 * N + 1)
        w0[2 * N] = c["s0"]
        w0 = p.rollout(w0)
    s = solve_slsqp(p, w0=w0)
    assert s.status in (0, 8), s.message  # 8: no further fp64 descent (judged by the point below)
    T = lambda a: torch.tensor(a, dtype=torch.float64)  # noqa: E731
    assert np.abs(p.g(T(s.x)).numpy()).max() < 1e-8 and p.d(T(s.x)).numpy().min() > -1e-8
    Xa, Ua, Sa, _, _ = p.unpack(r.w)
    Xb, Ub, Sb, _, _ = p.unpack(s.x)
    dU = np.abs(Ua - Ub)
    dU[0, -1] = 0.0  # last throttle: only the barrier fixes it
    assert dU.max() < 1e-6, dU.max()
    dX = np.abs(Xa - Xb)
    dX[3, -1] = 0.0  # vx_N: driven only by that throttle
    assert dX.max() < 1e-5 and np.abs(Sa - Sb).max() < 1e-5  # SLSQP stops at ftol 1e-12 (scaled)
    assert abs(r.obj - s.fun) <= 1e-9 * max(1.0, abs(r.obj))
    # the multipliers in the reference's lam_g layout
    lg = p.lam_g(r.nu, r.lam)
    assert lg.shape == (13 * c["N"] + 9,)
