"""Dense restatement of IPOPT's algorithm as the reference configures it (control/MPC.py:151-161).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference solves its NLP with IPOPT 3.x under casadi 3.6.5 (requirements.txt:8), options
max_iter 500, tol 1e-4, acceptable_tol 1e-2 and IPOPT's defaults otherwise.  casadi / IPOPT are not
importable here, so this module restates the published algorithm (Waechter & Biegler, Math. Prog.
106 (2006) 25-57, and the IPOPT option defaults) densely, on ``oracle.nlp.MPCProblem`` (the reference's
variables and constraint rows, pinned to the reference's own MPC.__init__ by tests/test_nlp_golden.py):

* primal-dual barrier method, slacks s for the inequality rows d(w) >= 0, gradient-based objective
  scaling (nlp_scaling_max_gradient 100), slack push (bound_push / bound_frac 1e-2);
* monotone Fiacco-McCormick barrier update (mu_init 0.1, kappa_mu 0.2, theta_mu 1.5, barrier_tol_factor
  10, several decreases per iteration), fraction to the boundary tau = max(0.99, 1 - mu);
* inertia correction delta_w (first 1e-4, then delta_last / 3, x100 / x8; tried 0 first);
* filter line search with the switching / Armijo conditions, theta_max / theta_min, one second-order
  correction that re-rolls the shooting states (the multiple-shooting form of IPOPT's SOC), the
  filter-reset heuristic (filter_reset_trigger 5, max_filter_resets 5);
* the watchdog (watchdog_shortened_iter_trigger 10, watchdog_trial_iter_max 3);
* the feasibility restoration phase: on a failed line search at an infeasible point, the l1 restoration
  NLP of W&B 2006 sec. 3.3 over the reference's variables --
      min rho sum(p + n) + zeta/2 ||D_R (w - w_R)||^2  s.t.  g(w) - p_g + n_g = 0,
                                                          d(w) - s - p_d + n_d = 0,  s, p, n >= 0,
  rho = 1000, zeta = sqrt(mu), D_R = diag(min(1, 1/|w_R|)) -- every equality row of the reference
  (including S_0 = s0, X_0 = state0) and every inequality row relaxed, solved by the same method with
  its own filter and barrier parameter max(mu, ||c||_inf) (p, n started in closed form), returning when
  theta <= 0.9 theta(w_R) and the point is acceptable to the original filter (augmented with w_R);
  bound multipliers afterwards mu/s, reset to 1 when they change by more than 1000, equality
  multipliers 0; status 4 when the restoration NLP converges without that.

It is an independent dense implementation (full-space KKT matrix, LDL inertia, torch autograd
derivatives) of the same rules the product restates stage-wise (csrc/mr_solver.h, csrc/mr_wave.h).
"""
import math
from dataclasses import dataclass

import numpy as np
import torch

from .nlp import IPMResult  # (round-3 restatement, kept for the rule-by-rule regression of oracle.ipopt)

RHO = 1000.0
KAPPA_RESTO = 0.9
MULT_RESET = 1000.0
WD_TRIGGER, WD_TRIAL_MAX = 10, 3
FILTER_RESET_TRIGGER, MAX_FILTER_RESETS = 5, 5
S_PHI, S_THETA, DELTA_SW, ETA, G_TH, G_PH = 2.3, 1.1, 1.0, 1e-4, 1e-5, 1e-5
KAPPA_EPS, KAPPA_MU, THETA_MU, KAPPA_SIGMA = 10.0, 0.2, 1.5, 1e10


def _T(a):
    return torch.tensor(np.asarray(a, dtype=np.float64), dtype=torch.float64)


class _NLP:
    """min f(w) s.t. g(w) = 0, d(w) >= 0 with autograd derivatives; ``lag_hess(w, nu, y)`` is the
    Hessian of f + nu.g - y.d in w."""

    def __init__(self, f, g, d, n, soc_roll=None, lag_hess=None, pre_eval=None):
        self.f, self.g, self.d, self.n = f, g, d, n
        self.grad_f = torch.func.grad(f)
        self.jac_g = torch.func.jacrev(g)
        self.jac_d = torch.func.jacrev(d)
        self.soc_roll = soc_roll
        self.pre_eval = pre_eval  # called with mu before each iteration's evaluation
        if lag_hess is not None:
            self.lag_hess = lag_hess
        else:
            def lag(w, nu, y):
                return f(w) + torch.dot(nu, g(w)) - torch.dot(y, d(w))
            self._hess = torch.func.hessian(lag, argnums=0)

    def lag_hess(self, w, nu, y):
        return self._hess(_T(w), _T(nu), _T(y)).numpy()


@dataclass
class _State:
    w: np.ndarray
    s: np.ndarray
    lam: np.ndarray  # bound duals of the slacks (= the inequality multipliers y in the regular phase)
    nu: np.ndarray
    mu: float


def _ftb(v, dv, tau):
    neg = dv < 0
    if not neg.any():
        return 1.0
    return float(min(1.0, np.min(-tau * v[neg] / dv[neg])))


class _Filter:
    def __init__(self):
        self.e = []

    def ok(self, th, ph):
        return not any(th >= a and ph >= b for a, b in self.e)

    def add(self, th, ph):
        self.e.append((th, ph))


def _kkt(stat, inf_pr, s, lam, nu, m, me, mi):
    sd = max(100.0, (np.abs(nu).sum() + np.abs(lam).sum()) / max(me + mi, 1)) / 100.0
    sc = max(100.0, np.abs(lam).sum() / max(mi, 1)) / 100.0
    cerr = np.abs(s * lam - m).max() if mi else 0.0
    return max(np.abs(stat).max() / sd, inf_pr, cerr / sc)


def _newton(nlp, w, s, lam, nu, y, mu, delta_last, gf, gw, Jg, dw, Jd):
    """Inertia-corrected primal-dual Newton step (slacks condensed); y: the multipliers in the Hessian."""
    from scipy.linalg import ldl
    n, me = w.size, gw.size
    W = nlp.lag_hess(w, nu, y)
    Sig = lam / s
    rd = dw - s
    H = W + Jd.T @ (Sig[:, None] * Jd)
    ghat = gf + Jd.T @ (Sig * rd - mu / s)
    delta, first = 0.0, True
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
            return None
    sol = np.linalg.solve(K, -np.concatenate([ghat, gw]))
    dz, nu_new = sol[:n], sol[n:]
    ds = Jd @ dz + rd
    dlam = mu / s - lam - Sig * ds
    return dz, nu_new, ds, dlam, delta


def _run(nlp, st, tol, max_iter, it0, filt, theta_max, theta_min, obj_scale, trace, exit_test=None,
         resto_factory=None, y_sep=None):
    """The IPM loop on ``nlp`` from state ``st``.  exit_test(w, s) -> bool ends it successfully after an
    accepted step (restoration phase); resto_factory(st, th, ph, filt) runs the restoration phase and
    returns (status, st, it) -- None disables it.  y_sep: separate inequality multipliers for the
    Hessian (the restoration phase's y_d, started at 0, stepped with the primal step size).
    Returns (status, st, it, kkt)."""
    w, s, lam, nu, mu = st.w.copy(), st.s.copy(), st.lam.copy(), st.nu.copy(), st.mu
    y = None if y_sep is None else y_sep.copy()
    me, mi = len(nlp.g(_T(w))), len(nlp.d(_T(w)))
    mu_min = tol / 10.0
    delta_last = 0.0
    it = it0
    status, kkt = 2, math.inf
    acc_count = 0
    filt_rej_iters = filt_resets = 0
    in_wd, wd_short, wd_trial, wd = False, 0, 0, None

    def theta_phi(ww, ss, m):
        wt = _T(ww)
        th = float(np.abs(nlp.g(wt).numpy()).sum() + np.abs(nlp.d(wt).numpy() - ss).sum())
        ph = float(nlp.f(wt)) - m * float(np.log(ss).sum())
        return th, ph

    while True:
        if nlp.pre_eval is not None:
            nlp.pre_eval(mu)
        wt = _T(w)
        fv = float(nlp.f(wt))
        gf = nlp.grad_f(wt).numpy()
        gw = nlp.g(wt).numpy()
        Jg = nlp.jac_g(wt).numpy()
        dw = nlp.d(wt).numpy()
        Jd = nlp.jac_d(wt).numpy()
        rd = dw - s
        yy = lam.copy()
        if y is not None:
            yy[:y.size] = y
        stat = gf + Jg.T @ nu - Jd.T @ yy
        inf_pr = max(np.abs(gw).max() if me else 0.0, np.abs(rd).max() if mi else 0.0)
        kkt = _kkt(stat if y is None else np.concatenate([stat, y - lam[:y.size]]), inf_pr, s, lam, nu, 0.0, me, mi)
        if not np.isfinite(kkt):
            status = 3
            break
        if kkt <= tol:
            status = 0 if exit_test is None else 4
            break
        if exit_test is None and trace is not None and trace.get("acc_iter", 0) > 0:
            acc_count = acc_count + 1 if kkt <= trace["acc_tol"] else 0
            if acc_count >= trace["acc_iter"]:
                status = 1
                break
        if it >= max_iter:
            status = 2
            break

        def err(m):
            return _kkt(stat if y is None else np.concatenate([stat, y - lam[:y.size]]), inf_pr, s, lam, nu, m, me,
                        mi)
        mu_old = mu
        while err(mu) <= KAPPA_EPS * mu and mu > mu_min:
            mu = max(mu_min, min(KAPPA_MU * mu, mu ** THETA_MU))
        if mu != mu_old:
            filt.e = []
            in_wd, wd_short = False, 0
        stp = _newton(nlp, w, s, lam, nu, yy, mu, delta_last, gf, gw, Jg, dw, Jd)
        if stp is None:
            status = 3
            break
        dz, nu_new, ds, dlam, delta = stp
        if delta > 0:
            delta_last = delta
        tau = max(0.99, 1.0 - mu)
        ap, ad = _ftb(s, ds, tau), _ftb(lam, dlam, tau)
        th = float(np.abs(gw).sum() + np.abs(rd).sum())
        ph = fv - mu * float(np.log(s).sum())
        gphi = float(gf @ dz - mu * np.sum(ds / s))
        th_pow = th ** S_THETA
        if gphi < 0:  # W&B 2006 eq. 23: the switching term only at theta <= theta_min
            a_min = 0.05 * min(G_TH, G_PH * th / (-gphi))
            if th <= theta_min:
                a_min = min(a_min, 0.05 * DELTA_SW * th_pow / (-gphi) ** S_PHI)
        else:
            a_min = 0.05 * G_TH

        def accept(th_t, ph_t, alpha, th_r, ph_r, gphi_r, thpow_r):
            if not th_t <= theta_max:
                return False, False, False
            sw = gphi_r < 0 and alpha * (-gphi_r) ** S_PHI > DELTA_SW * thpow_r
            if th_r <= theta_min and sw:
                ok, ft = ph_t <= ph_r + ETA * alpha * gphi_r + 1e-14 * abs(ph_r), True
            else:
                ok, ft = th_t <= (1 - G_TH) * th_r or ph_t <= ph_r - G_PH * th_r + 1e-14 * abs(ph_r), False
            if ok and not filt.ok(th_t, ph_t):
                return False, ft, True
            return ok, ft, False

        def backtrack(w0, s0, dz0, ds0, a0, nls0, a_minr, th_r, ph_r, gphi_r, thpow_r):
            alpha, nls, rej = a0, nls0, False
            while alpha >= a_minr and alpha >= 1e-30:
                wc, sc_ = w0 + alpha * dz0, s0 + alpha * ds0
                if (sc_ > 0).all():
                    th_t, ph_t = theta_phi(wc, sc_, mu)
                    ok, ft, rj = accept(th_t, ph_t, alpha, th_r, ph_r, gphi_r, thpow_r)
                    rej |= rj
                    if ok:
                        return True, alpha, wc, sc_, ft, nls, rej
                else:
                    th_t = math.inf
                if nls == 0 and nlp.soc_roll is not None and th_t >= th_r:
                    wsoc = nlp.soc_roll(wc)
                    ssoc = sc_ + (nlp.d(_T(wsoc)).numpy() - nlp.d(_T(wc)).numpy())
                    if (ssoc > 0).all():
                        th_s, ph_s = theta_phi(wsoc, ssoc, mu)
                        ok, ft, rj = accept(th_s, ph_s, alpha, th_r, ph_r, gphi_r, thpow_r)
                        rej |= rj
                        if ok:
                            return True, alpha, wsoc, ssoc, ft, nls, rej
                alpha *= 0.5
                nls += 1
            return False, alpha, None, None, False, nls, rej

        take_anyway = False
        if exit_test is None and not in_wd and wd_short >= WD_TRIGGER:
            wd = dict(w=w.copy(), s=s.copy(), lam=lam.copy(), nu=nu.copy(), dz=dz.copy(), ds=ds.copy(),
                      dlam=dlam.copy(), nu_new=nu_new.copy(), th=th, ph=ph, gphi=gphi, ap=ap, ad=ad,
                      a_min=a_min, th_pow=th_pow)
            in_wd, wd_trial = True, 0
        if in_wd:
            acc, alpha, wn, sn, ftype, nls, rej = backtrack(w, s, dz, ds, ap, 0, ap, wd["th"], wd["ph"], wd["gphi"],
                                                            wd["th_pow"])
            if acc:
                in_wd, wd_short = False, 0
                th, ph = wd["th"], wd["ph"]
            else:
                wd_trial += 1
                if wd_trial <= WD_TRIAL_MAX:
                    take_anyway = True
                    alpha, wn, sn, ftype = ap, w + ap * dz, s + ap * ds, False
                else:
                    w, s, lam, nu = wd["w"], wd["s"], wd["lam"], wd["nu"]
                    dz, ds, dlam, nu_new = wd["dz"], wd["ds"], wd["dlam"], wd["nu_new"]
                    th, ph, gphi, ap, ad, a_min, th_pow = (wd[k] for k in ("th", "ph", "gphi", "ap", "ad", "a_min",
                                                                           "th_pow"))
                    in_wd, wd_short = False, 0
                    acc, alpha, wn, sn, ftype, nls, rej = backtrack(w, s, dz, ds, 0.5 * ap, 1, a_min, th, ph, gphi,
                                                                    th_pow)
        else:
            acc, alpha, wn, sn, ftype, nls, rej = backtrack(w, s, dz, ds, ap, 0, a_min, th, ph, gphi, th_pow)
        if exit_test is not None and not acc:
            status = 3  # restoration failed
            break
        if not acc and not take_anyway:
            if resto_factory is not None and inf_pr > tol:
                filt.add((1 - G_TH) * th, ph - G_PH * th)
                rstat, st2, it = resto_factory(_State(w, s, lam, nu, mu), th, ph, filt, inf_pr, it + 1)
                if rstat != 0:
                    status = rstat
                    w, s = st2.w, st2.s
                    break
                w, s, lam, nu = st2.w, st2.s, st2.lam, st2.nu
                in_wd, wd_short, acc_count, filt_rej_iters = False, 0, 0, 0
                continue
            alpha = min(max(alpha, a_min), ap)  # the shortest tried step (feasible point)
            wn, sn, ftype = w + alpha * dz, s + alpha * ds, False
        if not take_anyway:
            wd_short = wd_short + 1 if (acc and alpha < ap) else 0
        if filt_resets < MAX_FILTER_RESETS:
            filt_rej_iters = filt_rej_iters + 1 if rej else 0
            if filt_rej_iters >= FILTER_RESET_TRIGGER:
                filt.e = []
                filt_resets += 1
                filt_rej_iters = 0
        if not ftype and not take_anyway:
            filt.add((1 - G_TH) * th, ph - G_PH * th)
        if y is not None:
            y = y + alpha * (lam[:y.size] + dlam[:y.size] - y)
        w, s = wn, sn
        nu = nu + alpha * (nu_new - nu)
        lam = lam + ad * dlam
        lam = np.clip(lam, mu / (KAPPA_SIGMA * s), KAPPA_SIGMA * mu / s)
        it += 1
        if trace is not None and "log" in trace:
            trace["log"].append((it, kkt, mu, alpha, delta, th, ph, exit_test is not None))
        if exit_test is not None and exit_test(w, s):
            status = 0
            break
    return status, _State(w, s, lam, nu, mu), it, kkt


def solve_ipopt(prob, tol=1e-8, max_iter=500, acceptable_tol=1e-6, acceptable_iter=15, w0=None, log=False):
    """IPOPT's algorithm (module docstring) on MPCProblem ``prob``; returns nlp.IPMResult with status
    0 solved, 1 acceptable, 2 max_iter, 3 failed, 4 infeasible (the product's MR_STATUS_* codes)."""
    w_init = np.array(prob.initial_guess() if w0 is None else w0, dtype=np.float64)
    gmax = float(torch.func.grad(prob.f)(_T(w_init)).abs().max())
    obj_scale = min(1.0, 100.0 / gmax) if gmax > 0 else 1.0

    def f(w):
        return obj_scale * prob.f(w)
    nlp = _NLP(f, prob.g, prob.d, w_init.size, soc_roll=prob.rollout)
    n = w_init.size
    dw0 = prob.d(_T(w_init)).numpy()
    me, mi = len(prob.g(_T(w_init))), dw0.size
    s0 = np.maximum(dw0, prob.push())
    st = _State(w_init, s0, np.ones(mi), np.zeros(me), 0.1)
    th0 = float(np.abs(prob.g(_T(w_init)).numpy()).sum() + np.abs(dw0 - s0).sum())
    trace = {"acc_tol": acceptable_tol, "acc_iter": acceptable_iter}
    if log:
        trace["log"] = []

    def resto(st_o, th_o, ph_o, filt_o, inf_pr, it0):
        """IPOPT's restoration phase from st_o (module docstring)."""
        wR, sR = st_o.w.copy(), st_o.s.copy()
        mu_r = max(st_o.mu, inf_pr)
        D2 = np.minimum(1.0, 1.0 / np.maximum(np.abs(wR), 1e-30)) ** 2
        zeta_box = [math.sqrt(mu_r)]
        cg = prob.g(_T(wR)).numpy()
        cd = prob.d(_T(wR)).numpy() - sR

        def pn(c):
            b = (mu_r - RHO * c) / (2 * RHO)
            q = mu_r * c / (2 * RHO)
            r = np.sqrt(b * b + q)
            nn = np.where(b >= 0, b + r, q / np.where(r - b > 0, r - b, 1.0))
            return c + nn, nn
        pg, ng = pn(cg)
        pd, nd = pn(cd)
        # augmented variables v = [w, pg, ng, pd, nd]; rows: g(w) - pg + ng = 0; d(w) - pd + nd >= 0 (slack s),
        # and pg, ng, pd, nd >= 0 (bounds as rows whose slacks are the variables themselves)
        ia = np.cumsum([0, n, me, me, mi, mi])
        wRt, D2t = _T(wR), _T(D2)

        def fR(v):
            w = v[:n]
            return RHO * torch.sum(v[n:]) + 0.5 * zeta_box[0] * torch.sum(D2t * (w - wRt) ** 2)

        def gR(v):
            return prob.g(v[:n]) - v[ia[1]:ia[2]] + v[ia[2]:ia[3]]

        def dR(v):
            return torch.cat([prob.d(v[:n]) - v[ia[3]:ia[4]] + v[ia[4]:ia[5]], v[n:]])
        def lagw(w, nu, yd):  # the constraints' curvature in w (p, n enter linearly)
            return torch.dot(nu, prob.g(w)) - torch.dot(yd, prob.d(w))
        hw = torch.func.hessian(lagw, argnums=0)

        def hessR(v, nu, y):
            H = np.zeros((ia[5], ia[5]))
            H[:n, :n] = hw(_T(v[:n]), _T(nu), _T(y[:mi])).numpy() + np.diag(zeta_box[0] * D2)
            return H

        def pre(mu):
            zeta_box[0] = math.sqrt(mu)  # IPOPT: resto_proximity_weight sqrt(mu)
        nlpR = _NLP(fR, gR, dR, ia[5], lag_hess=hessR, pre_eval=pre)
        v0 = np.concatenate([wR, pg, ng, pd, nd])
        pnv = v0[n:]
        sRt = np.concatenate([sR, pnv])
        lamR = np.concatenate([mu_r / sR, mu_r / pnv])
        stR = _State(v0, sRt, lamR, np.zeros(me), mu_r)
        ysep = np.zeros(mi)  # the relaxed rows' multipliers y_d start at 0 (the bounds' are their duals)
        thR0 = float(np.abs(gR(_T(v0)).numpy()).sum() + np.abs(dR(_T(v0)).numpy() - sRt).sum())
        filtR = _Filter()

        def exit_test(v, sv):
            w, s = v[:n], sv[:mi]
            th = float(np.abs(prob.g(_T(w)).numpy()).sum() + np.abs(prob.d(_T(w)).numpy() - s).sum())
            ph = float(f(_T(w))) - st_o.mu * float(np.log(s).sum())
            return th <= KAPPA_RESTO * th_o and filt_o.ok(th, ph)

        rstat, stR2, it, _ = _run(nlpR, stR, tol, max_iter, it0, filtR, 1e4 * max(1.0, thR0),
                                  1e-4 * max(1.0, thR0), 1.0, trace, exit_test=exit_test, y_sep=ysep)
        w, s = stR2.w[:n], stR2.s[:mi]
        if rstat != 0:
            return rstat, _State(w, s, st_o.lam, st_o.nu, st_o.mu), it
        lam_o = stR2.lam[:mi]
        lam_n = st_o.mu / s
        lam_n = np.where(np.abs(lam_n - lam_o) > MULT_RESET, 1.0, lam_n)
        return 0, _State(w, s, lam_n, np.zeros(me), st_o.mu), it

    status, st2, it, kkt = _run(nlp, st, tol, max_iter, 0, _Filter(), 1e4 * max(1.0, th0), 1e-4 * max(1.0, th0),
                                obj_scale, trace, resto_factory=resto)
    r = IPMResult(w=st2.w, nu=st2.nu / obj_scale, lam=st2.lam / obj_scale, s=st2.s, iters=it, status=status,
                  kkt=float(kkt), obj=float(prob.f(_T(st2.w))))
    if log:
        r.log = trace["log"]
    return r
