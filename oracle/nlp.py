"""Oracle restatement of the reference's MPC NLP and a dense IPM solver for it.

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

``MPCProblem`` restates ``control/MPC.py:30-161`` in the reference's own
decision variables ``w = [U (2xN), S_hat (N+1), States (6x(N+1))]``
(MPC.py:62-64), with torch expressions so exact first/second derivatives come
from autograd (independent of the product's generated derivative code):

* cost: terminal terms MPC.py:86-90, stage terms i = 1..N-1 MPC.py:93-98;
* equalities: S_0 = s0, X_0 = x0 (MPC.py:101-107), X_i = f(X_{i-1}, U_{i-1})
  for i = 1..N (MPC.py:133);
* inequalities: 0.1 <= S_i - S_{i-1} <= Ts*v_max (MPC.py:58-59,134);
  optional lane row |e_C(S_i, X_i)| <= max_error (the commented MPC.py:135);
  throttle/steer boxes with the *class attribute* d_max (MPC.py:50,138-141);
  rate rows with Python index i-1, so i = 0 couples U[:,0] and U[:,N-1]
  (MPC.py:142-143); rate rows against state0 throttle/steer (MPC.py:145-149);
* initial guess exactly as MPC.py:109-131 (shifted last_controls or
  (throttle0, steer0) repeated, S_i = s0 + i*Ts*v_max, state rollout).

``solve_ipm`` is a dense primal-dual interior-point method in the spirit of
the IPOPT configuration of MPC.py:151-161 (monotone Fiacco-McCormick barrier
update, fraction-to-boundary rule, inertia-corrected Newton steps) run to a
tight tolerance; ``solve_slsqp`` cross-checks the same NLP with scipy.
"""
import math
from dataclasses import dataclass

import numpy as np
import torch

from . import dynamics as dyn


@dataclass
class Fixed:
    """control/ControllerParameters.py:3-23."""
    lambda_s: float = 300
    alpha_L: float = 500
    min_steer: float = -0.9
    max_steer: float = 0.9
    min_throttle: float = -1.0
    max_steer_delta: float = 0.2
    min_steer_delta: float = -0.2
    max_throttle_delta: float = 2.0
    min_throttle_delta: float = -0.4
    q_v_max: float = 2
    v_max: float = 50
    Ts: float = 0.05
    N: int = 30
    max_iter: int = 500


@dataclass
class Runtime:
    """control/ControllerParameters.py:25-32."""
    alpha_c: float = 1000
    d_max: float = 0.85
    q_v_y: float = 50
    n: int = 2
    beta_delta: float = 5000


def _poly(c, s):
    # control/util.py:4-8: coefficients highest order first
    d = len(c) - 1
    out = 0.0
    for j, cj in enumerate(c):
        out = out + cj * s ** (d - j)
    return out


def _dpoly(c, s):
    d = len(c) - 1
    out = 0.0
    for j, cj in enumerate(c[:-1]):
        out = out + (d - j) * cj * s ** (d - j - 1)
    return out


def taylor_shift(c_desc, s0):
    """Coefficients (ascending powers of sigma) of p(s0 + sigma) for the
    highest-first global-s coefficients c_desc, computed exactly in rationals
    and rounded once to float64."""
    from fractions import Fraction
    from math import comb
    c = [Fraction(v) for v in reversed(c_desc)]
    s0 = Fraction(float(s0))
    d = len(c) - 1
    return [float(sum(c[j] * comb(j, k) * s0 ** (j - k) for j in range(k, d + 1))) for k in range(d + 1)]


def _poly_asc(a, x):
    out = 0.0
    for ak in reversed(a):
        out = out * x + ak
    return out


def _dpoly_asc(a, x):
    out = 0.0
    for k in range(len(a) - 1, 0, -1):
        out = out * x + k * a[k]
    return out


def pacejka_torch(a, Fz):
    """The magic formula of learning/vehicle.py:79-92 rewritten without its fp64
    cancellation: phi = alpha*(1 + E*(atan(x)/x - 1)), x = B*alpha, and
    Fy = BCD*phi*sin(C*atan(y))/(C*y), y = B*phi (series near 0). Same value
    in exact arithmetic; checked against mpmath in tests."""
    a = [float(v) for v in a]
    C = a[0]
    D = (a[1] * Fz + a[2]) * Fz
    BCD = a[3] * math.sin(a[4] * math.atan(a[5] * Fz))
    B = BCD / (C * D)
    E = a[6] * Fz ** 2 + a[7] * Fz + a[8]
    K2 = E * B * B

    def fy(alpha):
        x = B * alpha
        small = abs(B) * 1.0 < 1e-3
        if small:
            x2 = x * x
            eg = K2 * alpha * alpha * (-1.0 / 3.0 + x2 / 5.0 - x2 * x2 / 7.0)
        else:
            eg = E * (torch.atan(x) / x - 1.0)
        phi = alpha * (1.0 + eg)
        y = B * phi
        y2 = y * y
        if small:
            # sin(C atan y)/(C y) = 1 - (1/3 + C^2/6) y^2 + O(y^4)
            c2 = C * C
            h = 1.0 - y2 * (1.0 / 3.0 + c2 / 6.0) + y2 * y2 * (1.0 / 5.0 + c2 / 6.0 + c2 * c2 / 120.0)
        else:
            h = torch.sin(C * torch.atan(y)) / (C * y)
        return BCD * phi * h
    return fy


class MPCProblem:
    def __init__(self, state0, s0, cx, cy, max_error, runtime=None, N=None, Ts=None,
                 model="dyn", tyres=None, lane_bounds=False, last_controls=None,
                 fixed=None, d_max_class=0.85, elastic=None):
        self.fp = fixed or Fixed()
        self.rp = runtime or Runtime()
        self.N = self.fp.N if N is None else int(N)
        self.Ts = self.fp.Ts if Ts is None else float(Ts)
        self.model = model
        self.s0 = float(s0)
        self.cx = [float(c) for c in cx]
        self.cy = [float(c) for c in cy]
        self.ax = taylor_shift(self.cx, self.s0)
        self.ay = taylor_shift(self.cy, self.s0)
        self.max_error = float(max_error)
        self.lane = bool(lane_bounds)
        # elastic lane rows: |e_C| <= max_error + t_i, t_i >= 0, cost elastic * sum t_i (exact penalty)
        self.elastic = float(elastic) if (elastic and self.lane) else None
        self.state0 = dict(state0)
        self.d_max = float(d_max_class)  # MPC.py:50 reads the class attribute
        self.last_controls = last_controls
        N = self.N
        self.n = 9 * N + 7 + (N if self.elastic else 0)
        self.tyre_fns = None
        if tyres is not None:
            (af, Fzf), (ar, Fzr) = tyres
            self.tyre_fns = (pacejka_torch(af, Fzf), pacejka_torch(ar, Fzr))
        self._rows()

    # ---- index helpers (MPC.py:62-64) ----
    def iU(self, r, i):
        return r * self.N + i

    def iS(self, i):
        return 2 * self.N + i

    def iX(self, j, i):
        return 2 * self.N + self.N + 1 + j * (self.N + 1) + i

    def split(self, w):
        N = self.N
        U = w[:2 * N].reshape(2, N)
        S = w[2 * N:3 * N + 1]
        X = w[3 * N + 1:9 * N + 7].reshape(6, N + 1)
        return U, S, X

    def _rows(self):
        """Inequality rows (c(w) in [lo, hi]) in MPC.py's order."""
        fp, N, Ts = self.fp, self.N, self.Ts
        rows = []  # (kind, i, lo, hi)
        for i in range(1, N + 1):
            rows.append(("ds", i, 0.1, Ts * fp.v_max))
            if self.lane and not self.elastic:
                rows.append(("lane", i, -self.max_error, self.max_error))
        for i in range(N):
            rows.append(("thr", i, fp.min_throttle, self.d_max))
            rows.append(("steer", i, fp.min_steer, fp.max_steer))
            rows.append(("dthr", i, fp.min_throttle_delta, fp.max_throttle_delta))
            rows.append(("dsteer", i, fp.min_steer_delta, fp.max_steer_delta))
        if self.state0.get("throttle") is not None:
            rows.append(("thr0", 0, fp.min_throttle_delta, fp.max_throttle_delta))
        if self.state0.get("steer") is not None:
            rows.append(("steer0", 0, fp.min_steer_delta, fp.max_steer_delta))
        self.rows = rows
        self.lo = np.array([r[2] for r in rows])
        self.hi = np.array([r[3] for r in rows])

    # ---- model pieces ----
    def F(self, Xs, Us, M):
        """Stage dynamics vectorised over columns (6 x K states, 2 x K controls)."""
        Ts = self.Ts
        x = [Xs[j] for j in range(6)]
        u = [Us[0], Us[1]]
        if self.model == "kin":
            return dyn.f_vehicle_kinematic(x, u, Ts, M)
        tyres = self.tyre_fns
        fd = dyn.f_vehicle(x, u, Ts, M, tyres)
        if self.model in ("dyn", "dyn_pacejka"):
            return fd
        fk = dyn.f_vehicle_kinematic(x, u, Ts, M)
        vel = torch.sqrt(x[3] ** 2 + x[4] ** 2)
        vmin, vmax = dyn.VP.Vblendmin, dyn.VP.Vblendmax
        lam = torch.where(vel <= vmin, torch.zeros_like(vel),
                          torch.where(vel >= vmax, torch.ones_like(vel), (vel - vmin) / (vmax - vmin)))
        return lam * fd + (1 - lam) * fk

    def errors(self, S, X0, X1):
        """e_hat_C, e_hat_L of MPC.py:78-79.  The polynomials of util.make_poly are
        in global s (coefficients highest first); they are evaluated here in the
        local coordinate sigma = s - s0 after an exact rational Taylor shift
        (``taylor_shift``), the same polynomial without make_poly's cancellation
        noise (~1e-9 m in G at s ~ 1e3, enough to stall a 1e-10 KKT test)."""
        sig = S - self.s0
        gx, gy = _poly_asc(self.ax, sig), _poly_asc(self.ay, sig)
        dgx, dgy = _dpoly_asc(self.ax, sig), _dpoly_asc(self.ay, sig)
        eC = dgy * (X0 - gx) - dgx * (X1 - gy)
        eL = -dgx * (X0 - gx) - dgy * (X1 - gy)
        return eC, eL

    def f(self, w):
        fp, rp, N = self.fp, self.rp, self.N
        U, S, X = self.split(w)
        eC, eL = self.errors(S, X[0], X[1])
        J = -fp.lambda_s * S[N]
        J = J + rp.q_v_y * X[4, N] ** 2 + rp.alpha_c * eC[N] ** rp.n + fp.alpha_L * eL[N] ** 2
        J = J + torch.exp(fp.q_v_max * (X[3, N] - fp.v_max))
        if N > 1:
            sl = slice(1, N)
            J = J + torch.sum(rp.q_v_y * X[4, sl] ** 2 + rp.alpha_c * eC[sl] ** rp.n
                              + fp.alpha_L * eL[sl] ** 2
                              + rp.beta_delta * (U[1, 1:N] - U[1, 0:N - 1]) ** 2
                              + torch.exp(fp.q_v_max * (X[3, sl] - fp.v_max)))
        if self.elastic:
            J = J + self.elastic * torch.sum(w[9 * N + 7:])
        return J

    def g(self, w):
        U, S, X = self.split(w)
        st = self.state0
        x0 = torch.tensor([st["x"], st["y"], st["yaw"], st["v_x"], st["v_y"], st["yaw_dot"]],
                          dtype=w.dtype)
        M = dyn._torch_ns()
        Fk = self.F(X[:, :-1], U, M)
        return torch.cat([(S[0] - self.s0).reshape(1), X[:, 0] - x0, (X[:, 1:] - Fk).T.reshape(-1)])

    def c(self, w):
        U, S, X = self.split(w)
        st = self.state0
        N = self.N
        out = []
        eC = None
        if self.lane:
            eC, _ = self.errors(S, X[0], X[1])
        for kind, i, _, _ in self.rows:
            if kind == "ds":
                out.append(S[i] - S[i - 1])
            elif kind == "lane":
                out.append(eC[i])
            elif kind == "thr":
                out.append(U[0, i])
            elif kind == "steer":
                out.append(U[1, i])
            elif kind == "dthr":
                out.append(U[0, i] - U[0, (i - 1) % N])  # U[:, -1] at i = 0
            elif kind == "dsteer":
                out.append(U[1, i] - U[1, (i - 1) % N])
            elif kind == "thr0":
                out.append(U[0, 0] - st["throttle"])
            elif kind == "steer0":
                out.append(U[1, 0] - st["steer"])
        return torch.stack(out)

    def d(self, w):
        """One-sided form d(w) >= 0: [c - lo ; hi - c]."""
        cw = self.c(w)
        lo = torch.tensor(self.lo, dtype=w.dtype)
        hi = torch.tensor(self.hi, dtype=w.dtype)
        out = [cw - lo, hi - cw]
        if self.elastic:
            N = self.N
            U, S, X = self.split(w)
            eC, _ = self.errors(S, X[0], X[1])
            t = w[9 * N + 7:]
            out += [eC[1:] + self.max_error + t, self.max_error - eC[1:] + t, t]
        return torch.cat(out)

    # ---- IPOPT's view of the Opti problem (casadi 3.6.5 Opti -> nlpsol 'ipopt') ----
    def ipopt_ineq(self):
        """The inequality rows as casadi's Opti hands them to IPOPT: one row per ``subject_to`` call with
        a constant side moved into the bounds, so ``opti.bounded(lb, e, ub)`` (MPC.py:134, :142-143,
        :145-149; the lane row :135 when enabled) is ONE row with two finite bounds, while
        ``U[0, i] < d_max`` and ``U[0, i] > min_throttle`` (MPC.py:138-141) are two separate one-sided
        rows.  Equality rows are ``g`` (S_0, X_0, the dynamics).  Returns (d(w), dL, dU, kinds) with
        -inf / +inf for a missing side; the row order is grouped by kind (IPOPT's iterates do not depend
        on it)."""
        fp, N, Ts = self.fp, self.N, self.Ts
        inf = math.inf
        kinds, lo, hi = [], [], []

        def grp(kind, n, lb, ub):
            kinds.extend([kind] * n)
            lo.extend([lb] * n)
            hi.extend([ub] * n)
        grp("ds", N, 0.1, Ts * fp.v_max)
        if self.lane:
            grp("lane", N, -self.max_error, self.max_error)
        grp("thr_hi", N, -inf, self.d_max)
        grp("thr_lo", N, fp.min_throttle, inf)
        grp("steer_hi", N, -inf, fp.max_steer)
        grp("steer_lo", N, fp.min_steer, inf)
        grp("dthr", N, fp.min_throttle_delta, fp.max_throttle_delta)
        grp("dsteer", N, fp.min_steer_delta, fp.max_steer_delta)
        st = self.state0
        has_t, has_s = st.get("throttle") is not None, st.get("steer") is not None
        if has_t:
            grp("thr0", 1, fp.min_throttle_delta, fp.max_throttle_delta)
        if has_s:
            grp("steer0", 1, fp.min_steer_delta, fp.max_steer_delta)

        def d(w):
            U, S, X = self.split(w)
            out = [S[1:] - S[:-1]]
            if self.lane:
                eC, _ = self.errors(S, X[0], X[1])
                out.append(eC[1:])
            out += [U[0], U[0], U[1], U[1],
                    U[0] - torch.roll(U[0], 1), U[1] - torch.roll(U[1], 1)]  # Python index i-1: U[:, -1] at i = 0
            if has_t:
                out.append((U[0, 0] - st["throttle"]).reshape(1))
            if has_s:
                out.append((U[1, 0] - st["steer"]).reshape(1))
            return torch.cat(out)
        return d, np.array(lo, dtype=np.float64), np.array(hi, dtype=np.float64), kinds

    # ---- the reference's own row order (CasADi Opti call order, MPC.py:101-149) ----
    def opti_rows(self, w):
        """(g, lbg, ubg) in the order the reference's ``subject_to`` calls create them, with
        Opti's canonical rows (a constant side becomes the bound): S_0, X_{:,0} (:101-107);
        for i = 1..N the 6 dynamics rows X_i - f(X_{i-1}, U_{i-1}) and the Delta-S row (:133-134);
        for i = 0..N-1 thr < d_max, thr > min, steer < max, steer > min, the two rate rows with
        Python index i-1 (:137-143); the state0 rate rows (:145-149).  13N+9 rows when both
        state0 controls are given.  Lane rows are not part of the reference NLP (:135 commented)."""
        fp, N, Ts = self.fp, self.N, self.Ts
        wt = torch.as_tensor(np.asarray(w, dtype=np.float64))
        U, S, X = (t.numpy() for t in self.split(wt))
        gk = self.g(wt).numpy()  # [S0 - s0, X0 - x0 (6), defects (6 per stage)]
        st = self.state0
        x0 = [st["x"], st["y"], st["yaw"], st["v_x"], st["v_y"], st["yaw_dot"]]
        inf = math.inf
        g, lo, hi = [S[0]], [self.s0], [self.s0]
        for j in range(6):
            g.append(X[j, 0]); lo.append(x0[j]); hi.append(x0[j])
        for i in range(1, N + 1):
            for j in range(6):
                g.append(gk[7 + 6 * (i - 1) + j]); lo.append(0.0); hi.append(0.0)
            g.append(S[i] - S[i - 1]); lo.append(0.1); hi.append(Ts * fp.v_max)
        for i in range(N):
            g += [U[0, i], U[0, i], U[1, i], U[1, i], U[0, i] - U[0, i - 1], U[1, i] - U[1, i - 1]]
            lo += [-inf, fp.min_throttle, -inf, fp.min_steer, fp.min_throttle_delta, fp.min_steer_delta]
            hi += [self.d_max, inf, fp.max_steer, inf, fp.max_throttle_delta, fp.max_steer_delta]
        if st.get("throttle") is not None:
            g.append(U[0, 0] - st["throttle"]); lo.append(fp.min_throttle_delta); hi.append(fp.max_throttle_delta)
        if st.get("steer") is not None:
            g.append(U[1, 0] - st["steer"]); lo.append(fp.min_steer_delta); hi.append(fp.max_steer_delta)
        return np.array(g, dtype=np.float64), np.array(lo), np.array(hi)

    def lam_g(self, nu, lam):
        """The oracle's multipliers (Lagrangian f + nu.g - lam.d, d = [c - lo; hi - c]) as the
        reference's ``opti.lam_g`` (MPC.py:171) in ``opti_rows`` order, CasADi's sign
        convention (Lagrangian f + lam_g . g: positive at an active upper bound)."""
        N = self.N
        nr = len(self.rows)
        llo, lhi = np.asarray(lam[:nr]), np.asarray(lam[nr:2 * nr])
        idx = {(kind, i): r for r, (kind, i, _, _) in enumerate(self.rows)}
        out = list(np.asarray(nu[:7]))
        for i in range(1, N + 1):
            out += list(np.asarray(nu[7 + 6 * (i - 1):7 + 6 * i]))
            r = idx[("ds", i)]
            out.append(lhi[r] - llo[r])
        for i in range(N):
            rt, rs = idx[("thr", i)], idx[("steer", i)]
            rdt, rds = idx[("dthr", i)], idx[("dsteer", i)]
            out += [lhi[rt], -llo[rt], lhi[rs], -llo[rs], lhi[rdt] - llo[rdt], lhi[rds] - llo[rds]]
        for kind in ("thr0", "steer0"):
            if (kind, 0) in idx:
                r = idx[(kind, 0)]
                out.append(lhi[r] - llo[r])
        return np.array(out, dtype=np.float64)

    def lam_g_ipopt(self, nu, yd):
        """oracle.ipopt.solve_ipopt's multipliers (``nu`` on ``g``, ``yd`` on the ``ipopt_ineq`` rows, IPOPT's
        sign: positive at an active upper bound) as the reference's ``opti.lam_g`` (MPC.py:171) in
        ``opti_rows`` order.  A two-bounded ``opti.bounded`` row carries one multiplier, as in CasADi; the
        lane rows are not Opti rows of the reference and are dropped."""
        N = self.N
        _d, _lo, _hi, kinds = self.ipopt_ineq()
        yd = np.asarray(yd)
        k = np.array(kinds)
        by = {kind: yd[k == kind] for kind in dict.fromkeys(kinds)}
        out = list(np.asarray(nu[:7]))
        for i in range(1, N + 1):
            out += list(np.asarray(nu[7 + 6 * (i - 1):7 + 6 * i]))
            out.append(by["ds"][i - 1])
        for i in range(N):
            out += [by["thr_hi"][i], by["thr_lo"][i], by["steer_hi"][i], by["steer_lo"][i], by["dthr"][i],
                    by["dsteer"][i]]
        for kind in ("thr0", "steer0"):
            if kind in by:
                out.append(by[kind][0])
        return np.array(out, dtype=np.float64)

    def push(self):
        """IPOPT-style slack push per one-sided row (kappa = 1e-2)."""
        rng = np.concatenate([self.hi - self.lo, self.hi - self.lo])
        bnd = np.concatenate([np.abs(self.lo), np.abs(self.hi)])
        p = np.minimum(1e-2 * np.maximum(1.0, bnd), 1e-2 * rng)
        if self.elastic:
            N = self.N
            p = np.concatenate([p, np.full(2 * N, 1e-2 * max(1.0, self.max_error)), np.full(N, 1e-2)])
        return p

    def initial_guess(self):
        """MPC.py:109-131."""
        N, Ts, fp = self.N, self.Ts, self.fp
        st = self.state0
        w = np.zeros(self.n)
        if self.last_controls is not None:
            lc = list(self.last_controls)
            up = lc[1:] + [lc[-1]]
        else:
            up = [(st["throttle"], st["steer"]) for _ in range(N)]
        up = np.array(up, dtype=np.float64).T  # 2 x N
        w[:2 * N] = up.reshape(-1)
        x = np.array([st["x"], st["y"], st["yaw"], st["v_x"], st["v_y"], st["yaw_dot"]], dtype=np.float64)
        w[self.iS(0)] = self.s0
        for j in range(6):
            w[self.iX(j, 0)] = x[j]
        M = dyn._torch_ns()
        for i in range(1, N + 1):
            w[self.iS(i)] = self.s0 + i * Ts * fp.v_max
            xt = torch.tensor(x).reshape(6, 1)
            ut = torch.tensor(up[:, i - 1]).reshape(2, 1)
            x = self.F(xt, ut, M).reshape(6).numpy()
            for j in range(6):
                w[self.iX(j, i)] = x[j]
        if self.elastic:
            U, S, X = self.split(torch.tensor(w))
            eC, _ = self.errors(S, X[0], X[1])
            w[9 * N + 7:] = np.maximum(np.abs(eC.numpy()[1:]) - self.max_error, 0.0) + 1e-2
        return w

    def rollout(self, w):
        """Same controls / progress, states re-simulated from X_0 (zero defects)."""
        w = np.array(w, dtype=np.float64)
        N = self.N
        U, _, X = self.split(w)
        M = dyn._torch_ns()
        x = torch.tensor(X[:, 0].copy()).reshape(6, 1)
        for i in range(1, N + 1):
            x = self.F(x, torch.tensor(U[:, i - 1].copy()).reshape(2, 1), M)
            xi = x.reshape(6).numpy()
            for j in range(6):
                w[self.iX(j, i)] = xi[j]
        return w

    def unpack(self, w):
        """(States 6x(N+1), U 2xN, S_hat, e_hat_C[0..N-1], e_hat_L[0..N-1]) as MPC.py:166-170."""
        wt = torch.tensor(w)
        U, S, X = self.split(wt)
        eC, eL = self.errors(S, X[0], X[1])
        return (X.numpy().copy(), U.numpy().copy(), S.numpy().copy(),
                eC.numpy()[:self.N].copy(), eL.numpy()[:self.N].copy())


@dataclass
class IPMResult:
    w: np.ndarray
    nu: np.ndarray
    lam: np.ndarray
    s: np.ndarray
    iters: int
    status: int  # 0 solved, 2 max_iter, 3 failure
    kkt: float
    obj: float


def solve_ipm(prob, tol=1e-10, max_iter=300, w0=None, verbose=False, soc=True):
    """Dense primal-dual IPM on prob.f / prob.g / prob.d (float64).

    IPOPT-like rules (Waechter & Biegler 2006): gradient-based objective
    scaling, slack push, monotone Fiacco-McCormick barrier update, fraction to
    the boundary, inertia correction of the KKT matrix, and a filter line
    search (switching condition + Armijo on the barrier objective, filter of
    (theta, phi) pairs reset when mu changes) with a second-order correction
    that re-rolls the multiple-shooting states through the dynamics.
    """
    from scipy.linalg import ldl
    tfun = torch.func
    g, d = prob.g, prob.d
    # IPOPT's default gradient-based NLP scaling (nlp_scaling_max_gradient = 100):
    # the objective is multiplied by min(1, 100 / ||grad f(w0)||_inf).
    w_init = np.array(prob.initial_guess() if w0 is None else w0, dtype=np.float64)
    gmax = float(torch.func.grad(prob.f)(torch.tensor(w_init)).abs().max())
    obj_scale = min(1.0, 100.0 / gmax) if gmax > 0 else 1.0

    def f(w):
        return obj_scale * prob.f(w)
    grad_f = tfun.grad(f)
    jac_g = tfun.jacrev(g)
    jac_d = tfun.jacrev(d)

    def lag(w, nu, lam):
        return f(w) + torch.dot(nu, g(w)) - torch.dot(lam, d(w))
    hess_L = tfun.hessian(lag, argnums=0)

    T = lambda a: torch.tensor(a, dtype=torch.float64)  # noqa: E731
    w = w_init.copy()
    n = w.size
    gw = g(T(w)).numpy()
    me = gw.size
    dw = d(T(w)).numpy()
    mi = dw.size
    # slack push (IPOPT bound_push style, kappa = 1e-2 relative to the bound range)
    s = np.maximum(dw, prob.push())
    lam = np.ones(mi)
    nu = np.zeros(me)
    mu = 0.1
    kappa_eps, kappa_mu, theta_mu, kappa_sigma = 10.0, 0.2, 1.5, 1e10
    mu_min = tol / 10.0
    delta_last = 0.0
    status = 2
    it = 0
    kkt = np.inf

    def theta_of(ww, ss):
        wt2 = T(ww)
        return float(np.abs(g(wt2).numpy()).sum() + np.abs(d(wt2).numpy() - ss).sum())

    def phi_of(ww, ss):
        return float(f(T(ww))) - mu * float(np.log(ss).sum())

    th0 = theta_of(w, s)
    theta_max = 1e4 * max(1.0, th0)
    theta_min = 1e-4 * max(1.0, th0)
    s_phi, s_theta, delta_sw, eta, g_th, g_ph = 2.3, 1.1, 1.0, 1e-4, 1e-5, 1e-5
    filt = []
    for it in range(max_iter + 1):
        wt = T(w)
        fv = float(f(wt))
        gf = grad_f(wt).numpy()
        gw = g(wt).numpy()
        Jg = jac_g(wt).numpy()
        dw = d(wt).numpy()
        Jd = jac_d(wt).numpy()
        rd = dw - s
        stat = gf + Jg.T @ nu - Jd.T @ lam
        sd = max(100.0, (np.abs(nu).sum() + np.abs(lam).sum()) / (me + mi)) / 100.0
        sc = max(100.0, np.abs(lam).sum() / mi) / 100.0
        inf_pr = max(np.abs(gw).max(), np.abs(rd).max())

        def err(m):
            return max(np.abs(stat).max() / sd, inf_pr, np.abs(s * lam - m).max() / sc)
        kkt = err(0.0)
        if verbose:
            print(f"it {it:3d} f {fv: .10e} kkt {kkt:.3e} mu {mu:.2e} pr {inf_pr:.2e}")
        if not np.isfinite(kkt):
            status = 3
            break
        if kkt <= tol:
            status = 0
            break
        if it == max_iter:
            break
        mu_old = mu
        while err(mu) <= kappa_eps * mu and mu > mu_min:
            mu = max(mu_min, min(kappa_mu * mu, mu ** theta_mu))
        if mu != mu_old:
            filt = []
        W = hess_L(wt, T(nu), T(lam)).numpy()
        Sig = lam / s
        H = W + Jd.T @ (Sig[:, None] * Jd)
        ghat = gf + Jd.T @ (Sig * rd - mu / s)
        # inertia-corrected KKT solve
        delta = 0.0
        first = True
        while True:
            K = np.zeros((n + me, n + me))
            K[:n, :n] = H + delta * np.eye(n)
            K[:n, n:] = Jg.T
            K[n:, :n] = Jg
            _lu, D, _perm = ldl(K, lower=True)
            ev = np.linalg.eigvalsh(D)
            if int((ev > 0).sum()) == n and int((ev < 0).sum()) == me:
                break
            if first:
                delta = 1e-4 if delta_last == 0.0 else max(1e-20, delta_last / 3.0)
                first = False
            else:
                delta *= (100.0 if delta_last == 0.0 else 8.0)
            if delta > 1e40:
                status = 3
                break
        if status == 3:
            break
        if delta > 0:
            delta_last = delta
        sol = np.linalg.solve(K, -np.concatenate([ghat, gw]))
        dz = sol[:n]
        nu_new = sol[n:]
        ds = Jd @ dz + rd
        dlam = mu / s - lam - Sig * ds
        tau = max(0.99, 1.0 - mu)

        def ftb(v, dv):
            neg = dv < 0
            if not neg.any():
                return 1.0
            return float(min(1.0, np.min(-tau * v[neg] / dv[neg])))
        ap = ftb(s, ds)
        ad = ftb(lam, dlam)
        # ---- filter line search ----
        th = float(np.abs(gw).sum() + np.abs(rd).sum())
        ph = fv - mu * float(np.log(s).sum())
        gphi = float(gf @ dz - mu * np.sum(ds / s))
        if gphi < 0:
            a_min = 0.05 * min(g_th, g_ph * th / (-gphi), delta_sw * th ** s_theta / (-gphi) ** s_phi)
        else:
            a_min = 0.05 * g_th
        alpha = ap
        accepted = False
        f_type = False
        w_new = s_new = None
        nls = 0
        while alpha >= a_min and alpha >= 1e-30:  # same floor as mr_solver.h / mr_wave.h
            cands = [(w + alpha * dz, s + alpha * ds)]
            if nls == 0 and soc:
                pass
            for ci, (wc, sc_) in enumerate(cands):
                th_t = theta_of(wc, sc_)
                ph_t = phi_of(wc, sc_)
                ok = th_t <= theta_max and not any(th_t >= a and ph_t >= b for a, b in filt)
                if ok:
                    sw = gphi < 0 and alpha * (-gphi) ** s_phi > delta_sw * th ** s_theta
                    if th <= theta_min and sw:
                        ok = ph_t <= ph + eta * alpha * gphi + 1e-14 * abs(ph)
                        f_type = True
                    else:
                        ok = th_t <= (1 - g_th) * th or ph_t <= ph - g_ph * th + 1e-14 * abs(ph)
                        f_type = False
                if ok:
                    accepted = True
                    w_new, s_new = wc, sc_
                    break
                if nls == 0 and soc and th_t >= th:
                    # second-order correction: re-roll states through the dynamics
                    wsoc = prob.rollout(wc)
                    ssoc = sc_ + (d(T(wsoc)).numpy() - d(T(wc)).numpy())
                    if np.all(ssoc >= (1.0 - tau) * s * (1 + 1e-12) - 1e-300) or np.all(ssoc > 0):
                        th_s = theta_of(wsoc, ssoc)
                        ph_s = phi_of(wsoc, ssoc)
                        ok = th_s <= theta_max and not any(th_s >= a and ph_s >= b for a, b in filt)
                        if ok:
                            sw = gphi < 0 and alpha * (-gphi) ** s_phi > delta_sw * th ** s_theta
                            if th <= theta_min and sw:
                                ok = ph_s <= ph + eta * alpha * gphi + 1e-14 * abs(ph)
                                f_type = True
                            else:
                                ok = th_s <= (1 - g_th) * th or ph_s <= ph - g_ph * th + 1e-14 * abs(ph)
                                f_type = False
                        if ok and np.all(ssoc > 0):
                            accepted = True
                            w_new, s_new = wsoc, ssoc
                            break
            if accepted:
                break
            alpha *= 0.5
            nls += 1
        if not accepted:
            # no restoration phase: take the shortest tried step (reported via verbose)
            alpha = max(alpha, a_min)
            w_new, s_new = w + alpha * dz, s + alpha * ds
            f_type = False
        if not f_type:
            filt.append(((1 - g_th) * th, ph - g_ph * th))
        if verbose:
            print(f"    ap {ap:.3e} ad {ad:.3e} alpha {alpha:.3e} acc {accepted} ftype {f_type} "
                  f"delta {delta:.1e} th {th:.2e} |dz| {np.abs(dz).max():.2e} nfilt {len(filt)}")
        w, s = w_new, s_new
        nu = nu + alpha * (nu_new - nu)
        lam = lam + ad * dlam
        lam = np.clip(lam, mu / (kappa_sigma * s), kappa_sigma * mu / s)
    # multipliers reported for the unscaled objective
    return IPMResult(w=w, nu=nu / obj_scale, lam=lam / obj_scale, s=s, iters=it, status=status,
                     kkt=float(kkt), obj=float(prob.f(T(w))))


def kkt_residuals(prob, w, nu, lam):
    """Unscaled KKT pieces of a candidate (w, nu, lam): stationarity, equality
    and inequality violation, complementarity (for full-batch property checks)."""
    T = lambda a: torch.tensor(a, dtype=torch.float64)  # noqa: E731
    wt = T(w)
    gf = torch.func.grad(prob.f)(wt).numpy()
    Jg = torch.func.jacrev(prob.g)(wt).numpy()
    Jd = torch.func.jacrev(prob.d)(wt).numpy()
    dw = prob.d(wt).numpy()
    gw = prob.g(wt).numpy()
    stat = gf + Jg.T @ nu - Jd.T @ lam
    return {"stat": float(np.abs(stat).max()), "eq": float(np.abs(gw).max()),
            "ineq": float(max(0.0, -dw.min())), "compl": float(np.abs(dw * lam).max())}


def solve_slsqp(prob, w0=None, ftol=1e-12, maxiter=500, scale=1e-3):
    """Independent cross-check: scipy SLSQP on the same restated NLP (objective multiplied by
    ``scale``: at the objective's natural size ~1e5 SLSQP's QP subproblems stall far from the
    optimum).  SLSQP typically ends with status 8 ("positive directional derivative") once it
    can no longer improve in fp64; callers judge the returned point, not the flag."""
    from scipy.optimize import minimize
    T = lambda a: torch.tensor(a, dtype=torch.float64)  # noqa: E731
    gf = torch.func.grad(prob.f)
    jg = torch.func.jacrev(prob.g)
    jd = torch.func.jacrev(prob.d)
    cons = [{"type": "eq", "fun": lambda w: prob.g(T(w)).numpy(), "jac": lambda w: jg(T(w)).numpy()},
            {"type": "ineq", "fun": lambda w: prob.d(T(w)).numpy(), "jac": lambda w: jd(T(w)).numpy()}]
    w0 = prob.initial_guess() if w0 is None else w0
    r = minimize(lambda w: scale * float(prob.f(T(w))), w0, jac=lambda w: scale * gf(T(w)).numpy(),
                 constraints=cons, method="SLSQP", options={"ftol": ftol, "maxiter": maxiter})
    r.fun = r.fun / scale
    return r
