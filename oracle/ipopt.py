"""IPOPT restated densely: the algorithm the reference's ``opti.solve()`` runs (control/MPC.py:151-161).

TEST INFRASTRUCTURE ONLY (see oracle/__init__.py).

The reference calls IPOPT 3.14 through casadi 3.6.5 (requirements.txt:8) with max_iter 500, tol 1e-4,
acceptable_tol 1e-2, warm_start_init_point no, check_derivatives_for_naninf yes and IPOPT's defaults
otherwise.  casadi / IPOPT are not importable here, so this module restates the published
algorithm (Waechter & Biegler, Math. Prog. 106 (2006) 25-57; the IPOPT 3.14 option defaults) on the
problem exactly as casadi's Opti hands it to IPOPT (``oracle.nlp.MPCProblem.ipopt_ineq``: equality rows
S_0, X_0, the dynamics; one inequality row per ``subject_to`` with its constant side as the bound, so
``opti.bounded`` rows keep ONE slack with two bounds and ``U < d_max`` / ``U > min`` are two one-sided
rows; no variable bounds).  Dense linear algebra: a full-space KKT matrix, inertia from scipy's LDL^T.

IPOPT's rules, with the option (default) or the source routine they restate; ``Rules`` switches each one
so its effect on the iterates can be attributed (``R3`` = the round-3 restatement's rules):

problem / start (OrigIpoptNLP, DefaultIterateInitializer)
  * bound_relax_factor 1e-8: every inequality bound relaxed by min(constr_viol_tol, 1e-8 max(1, |b|));
  * nlp_scaling_method gradient-based, nlp_scaling_max_gradient 100 (min value 1e-8): objective factor
    min(1, 100 / ||grad f(x0)||_inf) and the same per constraint row (no row of this NLP exceeds 100 on
    the reference's inputs: ``Solve.max_row_gradient`` records it);
  * slack_bound_push / slack_bound_frac 1e-2: s0 = d(x0) projected into [d_L + p_L, d_U - p_U],
    p = min(1e-2 max(1, |b|), 1e-2 (d_U - d_L)) (the range term only for two-sided rows);
  * bound_mult_init_val 1 (v_L, v_U, z_L), mu_init 0.1;
  * constr_mult_init_max 1000: y_c, y_d = the least-square multipliers (W = 0, D_x = D_s = I augmented
    system: minimise ||grad_x L||^2 + ||grad_s L||^2), zero if their max exceeds 1000.
iteration (IpoptAlgorithm, PDFullSpaceSolver, PDPerturbationHandler, MonotoneMuUpdate)
  * y_d (multiplier of d(x) - s = 0) is an iterate of its own, stepped with the primal step size
    (alpha_for_y primal) and used in the Hessian and grad_x L; v_L, v_U (slack bound duals) take the dual
    step; kappa_sigma 1e10 safeguard on the bound duals;
  * kappa_d 1e-5: linear damping kappa_d mu (s - d_L) / (d_U - s) of one-sided slacks in the barrier
    objective, its gradient and the Newton right-hand side;
  * inertia correction: delta_x = delta_s (the slack block too), first 1e-4 (delta_xs_init) or
    delta_last / 3 (max 1e-20), then x100 (first_inc_fact, also when delta > 1e5 delta_last) or x8, give up
    above 1e40; delta_c = delta_d = 1e-8 mu^0.25 when the matrix is singular;
  * optimality error (curr_nlp_error): max(dual_inf / s_d, constraint violation of d(x) w.r.t. its
    bounds and |c|, compl / s_c), s_max 100, s_d over y_c, y_d, z, v; termination also requires the
    unscaled dual_inf_tol 1, constr_viol_tol 1e-4, compl_inf_tol 1e-4; acceptable level:
    acceptable_tol with acceptable_dual_inf_tol 1e10, acceptable_constr_viol_tol 1e-2,
    acceptable_compl_inf_tol 1e-2 for acceptable_iter (15) consecutive iterations;
  * monotone barrier update: while the barrier error <= barrier_tol_factor (10) mu, mu = max(floor,
    min(0.2 mu, mu^1.5)), floor = max(mu_min 1e-11, min(tol, compl_inf_tol) / 11); fraction to the boundary
    tau = max(0.99, 1 - mu); a new mu resets the line search (filter, watchdog, soft restoration).
line search (BacktrackingLineSearch, FilterLSAcceptor)
  * filter (unbounded) with theta_max / theta_min = 1e4 / 1e-4 max(1, theta_0), gamma_theta = gamma_phi =
    1e-5, s_phi 2.3, s_theta 1.1, delta 1, eta_phi 1e-4, alpha_min_frac 0.05, Compare_le tolerance
    10 eps |ref|, obj_max_inc 5; the first trial point is always tested; the filter is augmented unless the
    accepted step is f-type with the Armijo condition (UpdateForNextIteration);
  * max_soc 4 linear second-order corrections on the stored factorisation (kappa_soc 0.99), first trial
    only, when theta did not decrease;
  * filter_reset_trigger 5 / max_filter_resets 5; watchdog (shortened_iter_trigger 10, trial_iter_max 3,
    one trial point per watchdog iteration, f-type / Armijo tests at the watchdog point's step size);
  * tiny steps (tiny_step_tol 10 eps): accepted without line search, forcing a barrier decrease;
  * on a failed line search: the soft restoration phase (soft_resto_pderror_reduction_factor 0.9999,
    max_soft_resto_iters 10: the full primal-dual step with one step size, accepted by the filter or by a
    primal-dual error reduction); then "acceptable point reached" if the current point passes the
    acceptable tests (status 1); at an almost feasible point (theta <= 1e-2 tol) the stored acceptable
    point or restoration failure; otherwise the restoration phase; also when the inertia correction
    fails;
restoration phase (RestoMinC_1Nrm, RestoIpoptNLP, RestoIterateInitializer, RestoConvergenceCheck)
  * min rho ||p + n||_1 + zeta/2 ||D_R (x - x_R)||^2 s.t. c(x) - p_c + n_c = 0, d_L <= d(x) - p_d + n_d <= d_U,
    p, n >= 0 (variable bounds), rho = 1000, zeta = sqrt(mu_R), D_R = min(1, 1/|x_R|); every row of the
    reference relaxed, the initial-state rows included; mu_R = max(mu, ||c, d - s||_inf); p, n in closed
    form; slack bound duals min(rho, v); y by least squares; its own filter / watchdog;
  * returns when the original theta <= 0.9 theta(x_R) at a point the original filter (augmented with x_R)
    and x_R accept; then bound duals by a complementarity Newton step over the whole restoration (dual
    fraction to the boundary), all reset to 1 if one exceeds bound_mult_reset_threshold 1000, y = 0
    (constr_mult_reset_threshold 0);
  * the restoration problem converged: status 3 (restoration failed) if the original primal infeasibility
    is <= 1e2 tol, else 4 (local infeasibility); a failed restoration line search: 3.

Restated from the published algorithm and IPOPT's documented defaults, not from IPOPT's source (not
vendored in the reference): parity with IPOPT itself stays UNPINNED.  Not restated
(irrelevant here or unreachable): variable bounds of the regular problem (none), the Jacobian-degeneracy
bookkeeping (degen_iters_max), iterative refinement, slack_move, the adaptive barrier strategies.
"""
import math
from dataclasses import dataclass, replace

import numpy as np
import torch
from scipy.linalg import ldl, lu_factor, lu_solve

from .nlp import IPMResult

EPS = float(np.finfo(np.float64).eps)
S_PHI, S_THETA, DELTA_SW, ETA_PHI, G_TH, G_PH = 2.3, 1.1, 1.0, 1e-4, 1e-5, 1e-5
KAPPA_EPS, KAPPA_MU, THETA_MU, KAPPA_SIGMA = 10.0, 0.2, 1.5, 1e10
RHO, KAPPA_RESTO, MULT_RESET = 1000.0, 0.9, 1000.0
WD_TRIGGER, WD_TRIAL_MAX, FILTER_RESET_TRIGGER, MAX_FILTER_RESETS = 10, 3, 5, 5
KAPPA_SOC, SOFT_RESTO_FACTOR, MAX_SOFT_RESTO = 0.99, 0.9999, 10
CONSTR_VIOL_TOL, COMPL_INF_TOL, DUAL_INF_TOL = 1e-4, 1e-4, 1.0
ACC_DUAL_INF, ACC_CONSTR_VIOL, ACC_COMPL = 1e10, 1e-2, 1e-2


@dataclass(frozen=True)
class Rules:
    opti_rows: bool = True            # IPOPT's rows (two-bounded slacks); False: the one-sided d(w) >= 0 form
    bound_relax_factor: float = 1e-8
    constr_scaling: bool = True
    ls_mult_init: bool = True         # constr_mult_init_max 1000
    separate_yd: bool = True          # y_d its own iterate; False: y_d = v_U - v_L
    sd_count_yd: bool = True          # s_d sums y_d too
    kappa_d: float = 1e-5
    delta_s: bool = True              # delta on the slack block
    delta_inc_1e5: bool = True        # x100 also when delta > 1e5 delta_last
    unscaled_tests: bool = True       # dual_inf_tol / constr_viol_tol / compl_inf_tol (+ acceptable_*)
    mu_floor: str = "ipopt"           # "ipopt" or "tol10"
    nlp_error_viol: bool = True       # the error's primal part is the violation of d(x)'s bounds
    max_soc: int = 4                  # linear SOCs; -1: one nonlinear re-roll of the shooting states
    ftype_rule: str = "ipopt"         # "ipopt": augment unless f-type & Armijo; "r3": unless theta<=theta_min & f-type
    first_trial: bool = True          # always test the first trial point
    obj_max_inc: float = 5.0          # 0: off
    compare_eps: bool = True          # Compare_le (10 eps |ref|); False: 1e-14 |phi| on the phi tests
    soc_in_watchdog: bool = False
    tiny_step: bool = True
    soft_resto: bool = True
    acceptable_on_fail: bool = True
    resto_on_fact_fail: bool = True
    shortest_step_if_feasible: bool = False   # round 3: no restoration at inf_pr <= tol, take the shortest step
    resto_feasible_status: bool = True
    resto_mult: str = "newton"        # "newton" (IPOPT) or "mu_s" (round 3)
    resto_v_init: str = "min_rho"     # "min_rho" (IPOPT) or "mu_s" (round 3)
    resto_ls_mult: bool = True
    resto_watchdog: bool = True
    resto_soc: bool = True
    resto_relax_x0: bool = True       # the initial-state rows S_0 = s0, X_0 = state0 relaxed in the restoration
                                      # phase too (IPOPT relaxes every equality row; the product eliminates x_0)
    push_range_one_sided: bool = False  # round 3 pushed one-sided rows by min(1e-2 max(1,|b|), 1e-2 range)


IPOPT = Rules()
# the rules of the product (csrc/mr_solver.h, csrc/mr_wave.h): IPOPT's, less the tiny-step termination (compiled
# out, MR_TINY_STEP 0: it reads the step's rounding floor) and with the restoration phase's
# documented simplifications; the restoration phase's own iterates are not compared (the product also relaxes a
# two-sided row's distances separately).  Every field here must mirror a compile-time rule of the kernel:
# tests/test_rules_label.py reads them back from mr_solver.h.
PRODUCT = replace(IPOPT, tiny_step=False, resto_ls_mult=False, resto_soc=False, resto_watchdog=False,
                  resto_relax_x0=False)
R3 = Rules(opti_rows=False, bound_relax_factor=0.0, constr_scaling=False, ls_mult_init=False, separate_yd=False,
           sd_count_yd=False, kappa_d=0.0, delta_s=False, delta_inc_1e5=False, unscaled_tests=False, mu_floor="tol10",
           nlp_error_viol=False, max_soc=-1, ftype_rule="r3", first_trial=False, obj_max_inc=0.0, compare_eps=False,
           soc_in_watchdog=True, tiny_step=False, soft_resto=False, acceptable_on_fail=False,
           resto_on_fact_fail=False, shortest_step_if_feasible=True, resto_feasible_status=False, resto_mult="mu_s",
           resto_v_init="mu_s", resto_ls_mult=False, resto_watchdog=False, resto_soc=False,
           push_range_one_sided=True)


def _T(a):
    return torch.tensor(np.asarray(a, dtype=np.float64), dtype=torch.float64)


class Problem:
    """min f(x) s.t. c(x) = 0, d_L <= d(x) <= d_U (+-inf: no bound), x_i >= x_L,i (x_L,i > -inf).
    f, c, d: torch functions; lag_hess(x, wf, yc, yd) -> Hessian of wf f + yc.c + yd.d (numpy), optional;
    soc_roll(x) -> x with the shooting states re-simulated (round-3 SOC), optional."""

    def __init__(self, n, f, c, d, dL, dU, xL=None, lag_hess=None, soc_roll=None, push=None, x0_rows=0):
        self.n, self.f, self.c, self.d = n, f, c, d
        self.x0_rows = x0_rows  # leading equality rows that fix the initial state (Rules.resto_relax_x0)
        self.dL, self.dU = np.asarray(dL, np.float64), np.asarray(dU, np.float64)
        self.xL = np.full(n, -np.inf) if xL is None else np.asarray(xL, np.float64)
        self.soc_roll, self.push = soc_roll, push
        self._g = torch.func.grad(f)
        self._jc = torch.func.jacrev(c)
        self._jd = torch.func.jacrev(d)
        if lag_hess is None:
            def lag(x, wf, yc, yd):
                return wf * f(x) + torch.dot(yc, c(x)) + torch.dot(yd, d(x))
            h = torch.func.hessian(lag, argnums=0)
            lag_hess = lambda x, wf, yc, yd: h(_T(x), torch.tensor(float(wf), dtype=torch.float64), _T(yc),  # noqa: E731
                                               _T(yd)).numpy()
        self.lag_hess = lag_hess

    def evaluate(self, x):
        xt = _T(x)
        return dict(f=float(self.f(xt)), gf=self._g(xt).numpy(), c=self.c(xt).numpy(), Jc=self._jc(xt).numpy(),
                    d=self.d(xt).numpy(), Jd=self._jd(xt).numpy())

    def primal(self, x):
        xt = _T(x)
        return float(self.f(xt)), self.c(xt).numpy(), self.d(xt).numpy()


def _scaled(P, x0, rules):
    """IPOPT's gradient-based scaling of P at x0: (scaled problem, df, dc, dd, max row gradient)."""
    ev = P.evaluate(x0)
    gmax = float(np.abs(ev["gf"]).max()) if P.n else 0.0
    df = max(1e-8, min(1.0, 100.0 / gmax)) if gmax > 0 else 1.0

    def rowf(J):
        if J.size == 0:
            return np.ones(J.shape[0]), 0.0
        m = np.abs(J).max(axis=1)
        f = np.where(m > 100.0, np.maximum(1e-8, 100.0 / np.maximum(m, 1e-300)), 1.0)
        return f, float(m.max())
    dc, mc = rowf(ev["Jc"])
    dd, md = rowf(ev["Jd"])
    if not rules.constr_scaling:
        dc, dd = np.ones_like(dc), np.ones_like(dd)
    dct, ddt = _T(dc), _T(dd)
    f, c, d, lh = P.f, P.c, P.d, P.lag_hess
    S = Problem(P.n, lambda x: df * f(x), lambda x: dct * c(x), lambda x: ddt * d(x), dd * P.dL, dd * P.dU, P.xL,
                lag_hess=lambda x, wf, yc, yd: lh(x, wf * df, np.asarray(yc) * dc, np.asarray(yd) * dd),
                soc_roll=P.soc_roll, push=P.push, x0_rows=P.x0_rows)
    return S, df, dc, dd, max(mc, md)


@dataclass
class _It:
    x: np.ndarray
    s: np.ndarray
    yc: np.ndarray
    yd: np.ndarray
    zL: np.ndarray
    vL: np.ndarray
    vU: np.ndarray

    def copy(self):
        return _It(*(a.copy() for a in (self.x, self.s, self.yc, self.yd, self.zL, self.vL, self.vU)))


class _Filter:
    def __init__(self):
        self.e = []

    def ok(self, th, ph):
        return all(th < a or ph < b for a, b in self.e)

    def add(self, th, ph):
        self.e.append(((1.0 - G_TH) * th, ph - G_PH * th))


def _ftb(v, dv, tau):
    neg = dv < 0
    if not neg.any():
        return 1.0
    return float(min(1.0, np.min(-tau * v[neg] / dv[neg])))


def _inertia(D):
    n = D.shape[0]
    pos = neg = zero = 0
    i = 0
    while i < n:
        if i + 1 < n and D[i + 1, i] != 0.0:
            ev = np.linalg.eigvalsh(D[i:i + 2, i:i + 2])
            vals = list(ev)
            i += 2
        else:
            vals = [D[i, i]]
            i += 1
        for v in vals:
            if v == 0.0:  # an exactly singular pivot (MUMPS' null-pivot detection is off by default)
                zero += 1
            elif v > 0:
                pos += 1
            else:
                neg += 1
    return pos, neg, zero


def _pn(c, mu, rho):
    """IPOPT's closed-form start of (p, n) for a row residual c (so that c - p + n = 0)."""
    b = (mu - rho * c) / (2 * rho)
    q = mu * c / (2 * rho)
    r = np.sqrt(b * b + q)
    n = np.where(b >= 0, b + r, q / np.where(r - b > 0, r - b, 1.0))
    return c + n, n


class _Alg:
    """IPOPT's main loop on a (scaled) Problem.  ``resto`` = the restoration context when this is the
    restoration phase's algorithm."""

    def __init__(self, P, rules, tol, max_iter, acc_tol, acc_iter, log, unscale=(1.0, None, None), resto=None):
        self.P, self.R, self.tol, self.max_iter = P, rules, tol, max_iter
        self.acc_tol, self.acc_iter, self.log = acc_tol, acc_iter, log
        self.df, self.dc, self.dd = unscale
        self.resto = resto
        self.mL, self.mU = np.isfinite(P.dL), np.isfinite(P.dU)
        self.mx = np.isfinite(P.xL)
        self.oneL, self.oneU = self.mL & ~self.mU, self.mU & ~self.mL
        self.mu = 0.1
        self.delta_last = 0.0
        self.filt = _Filter()
        self.theta_max = self.theta_min = None
        self.in_wd, self.wd_short, self.wd_trial, self.wd = False, 0, 0, None
        self.in_soft, self.soft_count = False, 0
        self.filt_rej_iters = self.filt_resets = 0
        self.acc_count = 0
        self.acc_point = None
        self.tiny_flag = False
        self.pre_eval = None
        self.first_iter = True
        self.why = self.resto_why = ""
        self.stats = dict(soc_tries=0, soc_acc=0, soft=0, soft_acc=0, wd_start=0, wd_stop=0, tiny=0, delta_pos=0,
                          resto=0, ls_fail=0, filt_max=0, filt_resets=0)
        self.mu_floor = (max(1e-11, min(tol, COMPL_INF_TOL) / (KAPPA_EPS + 1.0)) if rules.mu_floor == "ipopt"
                         else tol / 10.0)

    # ---------------- pieces of IpoptCalculatedQuantities ----------------
    def dist(self, it):
        P = self.P
        return (it.s - P.dL)[self.mL], (P.dU - it.s)[self.mU], (it.x - P.xL)[self.mx]

    def yd_of(self, it):
        if self.R.separate_yd:
            return it.yd
        return it.vU - it.vL

    def barrier(self, f, x, s, mu):
        P, kd = self.P, self.R.kappa_d
        SL, SU, X = (s - P.dL)[self.mL], (P.dU - s)[self.mU], (x - P.xL)[self.mx]
        if (SL <= 0).any() or (SU <= 0).any() or (X <= 0).any():
            return math.inf
        ph = f - mu * (np.log(SL).sum() + np.log(SU).sum() + np.log(X).sum())
        if kd:
            ph += kd * mu * ((s - P.dL)[self.oneL].sum() + (P.dU - s)[self.oneU].sum() + X.sum())
        return float(ph)

    def grad_barrier(self, ev, it, mu):
        P, kd = self.P, self.R.kappa_d
        gx = ev["gf"].copy()
        SL, SU, X = self.dist(it)
        gx[self.mx] += -mu / X + kd * mu
        gs = np.zeros_like(it.s)
        gs[self.mL] -= mu / SL
        gs[self.mU] += mu / SU
        if kd:
            gs[self.oneL] += kd * mu
            gs[self.oneU] -= kd * mu
        return gx, gs

    def measure(self, it):
        """Everything the convergence test, the barrier update and the line search need at ``it``."""
        P = self.P
        ev = P.evaluate(it.x)
        yd = self.yd_of(it)
        SL, SU, X = self.dist(it)
        glx = ev["gf"] + ev["Jc"].T @ it.yc + ev["Jd"].T @ yd
        glx[self.mx] -= it.zL[self.mx]
        gls = -yd.copy()
        gls[self.mL] -= it.vL[self.mL]
        gls[self.mU] += it.vU[self.mU]
        rd = ev["d"] - it.s
        dual_inf = max(np.abs(glx).max(initial=0.0), np.abs(gls).max(initial=0.0))
        pr_inf = max(np.abs(ev["c"]).max(initial=0.0), np.abs(rd).max(initial=0.0))
        viol_d = np.maximum(0.0, np.maximum(np.where(self.mL, P.dL - ev["d"], 0.0),
                                            np.where(self.mU, ev["d"] - P.dU, 0.0)))
        nlp_viol = max(np.abs(ev["c"]).max(initial=0.0), viol_d.max(initial=0.0))
        prods = np.concatenate([it.vL[self.mL] * SL, it.vU[self.mU] * SU, it.zL[self.mx] * X])
        nb = prods.size
        bsum = np.abs(it.vL[self.mL]).sum() + np.abs(it.vU[self.mU]).sum() + np.abs(it.zL[self.mx]).sum()
        ysum = np.abs(it.yc).sum() + (np.abs(yd).sum() if self.R.sd_count_yd else 0.0)
        ny = it.yc.size + (yd.size if self.R.sd_count_yd else 0)
        s_d = max(100.0, (ysum + bsum) / max(ny + nb, 1)) / 100.0
        s_c = max(100.0, bsum / max(nb, 1)) / 100.0

        def compl(mu):
            return float(np.abs(prods - mu).max()) if nb else 0.0
        th = float(np.abs(ev["c"]).sum() + np.abs(rd).sum())
        E = dict(ev=ev, glx=glx, gls=gls, rd=rd, dual_inf=dual_inf, pr_inf=pr_inf, nlp_viol=nlp_viol, s_d=s_d,
                 s_c=s_c, compl=compl, theta=th, yd=yd, viol_d=viol_d)
        E["nlp_err"] = max(dual_inf / s_d, nlp_viol if self.R.nlp_error_viol else pr_inf, compl(0.0) / s_c)
        if self.R.unscaled_tests and self.dc is not None:
            du = max(np.abs(glx).max(initial=0.0), np.abs(self.dd * gls).max(initial=0.0)) / self.df
            cv = max(np.abs(ev["c"] / self.dc).max(initial=0.0), (viol_d / self.dd).max(initial=0.0))
            E["unscaled"] = (du, cv, compl(0.0) / self.df)
        else:
            E["unscaled"] = (0.0, 0.0, 0.0)
        return E

    def barrier_error(self, E, mu):
        return max(E["dual_inf"] / E["s_d"], E["pr_inf"], E["compl"](mu) / E["s_c"])

    def is_acceptable(self, E):
        du, cv, co = E["unscaled"]
        return (E["nlp_err"] <= self.acc_tol and du <= ACC_DUAL_INF and cv <= ACC_CONSTR_VIOL and co <= ACC_COMPL)

    # ---------------- the Newton system ----------------
    def factorize(self, it, E, mu, delta_c=0.0):
        """PDPerturbationHandler + PDFullSpaceSolver: returns (solver, delta_x) or None."""
        P, R = self.P, self.R
        ev = E["ev"]
        n, mc = P.n, ev["c"].size
        W = P.lag_hess(it.x, 1.0, it.yc, self.yd_of(it))
        SL, SU, X = self.dist(it)
        sig_s = np.zeros_like(it.s)
        sig_s[self.mL] += it.vL[self.mL] / SL
        sig_s[self.mU] += it.vU[self.mU] / SU
        sig_x = np.zeros(n)
        sig_x[self.mx] = it.zL[self.mx] / X
        Jd, Jc = ev["Jd"], ev["Jc"]
        base = W + np.diag(sig_x)
        delta, first = 0.0, True
        while True:
            ds_ = delta if R.delta_s else 0.0
            D = sig_s + ds_
            H = base + delta * np.eye(n) + Jd.T @ (D[:, None] * Jd)
            K = np.zeros((n + mc, n + mc))
            K[:n, :n] = H
            K[:n, n:] = Jc.T
            K[n:, :n] = Jc
            K[n:, n:] = -delta_c * np.eye(mc)
            _lu, Dm, _p = ldl(K, lower=True)
            pos, neg, zero = _inertia(Dm)
            if zero == 0 and pos == n and neg == mc:
                break
            if zero > 0 and delta_c == 0.0 and not (delta > 0):
                delta_c = 1e-8 * mu ** 0.25  # jacobian_regularization_value / _exponent
                continue
            if first:
                delta = 1e-4 if self.delta_last == 0.0 else max(1e-20, self.delta_last / 3.0)
                first = False
            else:
                if self.delta_last == 0.0 or (R.delta_inc_1e5 and 1e5 * self.delta_last < delta):
                    delta *= 100.0
                else:
                    delta *= 8.0
            if delta > 1e40:
                return None
        if delta > 0:
            self.delta_last = delta
            self.stats["delta_pos"] += 1
        self.stats["filt_max"] = max(self.stats["filt_max"], len(self.filt.e))
        return dict(lu=lu_factor(K), K=K, D=D, sig_s=sig_s, sig_x=sig_x, delta=delta, delta_c=delta_c, n=n, mc=mc)

    def solve(self, F, it, E, mu, c_rhs, r_rhs):
        """The search direction for constraint right-hand sides c_rhs (c) and r_rhs (d - s)."""
        ev = E["ev"]
        n = F["n"]
        gx, gs = self.grad_barrier(ev, it, mu)
        D = F["D"]
        rx = -(gx + ev["Jd"].T @ (D * r_rhs + gs))
        rc = -c_rhs - F["delta_c"] * it.yc
        rhs = np.concatenate([rx, rc])
        sol = lu_solve(F["lu"], rhs)
        # iterative refinement (PDFullSpaceSolver: min_refinement_steps 1, up to max_refinement_steps 10 while
        # the residual improves)
        res_old = math.inf
        for _r in range(10):
            res = rhs - F["K"] @ sol
            rn = float(np.abs(res).max())
            if _r >= 1 and not (rn < 0.5 * res_old):
                break
            sol = sol + lu_solve(F["lu"], res)
            res_old = rn
        dx, yc_new = sol[:n], sol[n:]
        ds = ev["Jd"] @ dx + r_rhs
        yd = self.yd_of(it)
        dyd = D * ds + gs - yd
        SL, SU, X = self.dist(it)
        dvL = np.zeros_like(it.s)
        dvU = np.zeros_like(it.s)
        dvL[self.mL] = mu / SL - it.vL[self.mL] - (it.vL[self.mL] / SL) * ds[self.mL]
        dvU[self.mU] = mu / SU - it.vU[self.mU] + (it.vU[self.mU] / SU) * ds[self.mU]
        dzL = np.zeros(n)
        dzL[self.mx] = mu / X - it.zL[self.mx] - F["sig_x"][self.mx] * dx[self.mx]
        return dict(x=dx, s=ds, yc=yc_new - it.yc, yd=dyd, zL=dzL, vL=dvL, vU=dvU)

    def alpha_primal_max(self, it, dr, tau):
        SL, SU, X = self.dist(it)
        return min(_ftb(SL, dr["s"][self.mL], tau), _ftb(SU, -dr["s"][self.mU], tau),
                   _ftb(X, dr["x"][self.mx], tau))

    def alpha_dual_max(self, it, dr, tau):
        return min(_ftb(it.vL[self.mL], dr["vL"][self.mL], tau), _ftb(it.vU[self.mU], dr["vU"][self.mU], tau),
                   _ftb(it.zL[self.mx], dr["zL"][self.mx], tau))

    def grad_barr_t_delta(self, E, it, dr, mu):
        gx, gs = self.grad_barrier(E["ev"], it, mu)
        return float(gx @ dr["x"] + gs @ dr["s"])

    # ---------------- acceptability (FilterLSAcceptor) ----------------
    def cmp_le(self, lhs, rhs, bas):
        return lhs - rhs <= 10.0 * EPS * abs(bas)

    def is_ftype(self, a_test, ref):
        g = ref["gphi"]
        return g < 0 and a_test * (-g) ** S_PHI > DELTA_SW * ref["th"] ** S_THETA

    def armijo(self, ph_t, a_test, ref):
        if self.R.compare_eps:
            return self.cmp_le(ph_t - ref["ph"], ETA_PHI * a_test * ref["gphi"], ref["ph"])
        return ph_t <= ref["ph"] + ETA_PHI * a_test * ref["gphi"] + 1e-14 * abs(ref["ph"])

    def acc_to_iterate(self, th_t, ph_t, ref, from_resto=False):
        th_r, ph_r = ref["th"], ref["ph"]
        if self.R.obj_max_inc and not from_resto and ph_t > ph_r:
            bas = math.log10(abs(ph_r)) if abs(ph_r) > 10.0 else 1.0
            if math.log10(ph_t - ph_r) > self.R.obj_max_inc + bas:
                return False
        if self.R.compare_eps:
            return self.cmp_le(th_t, (1 - G_TH) * th_r, th_r) or self.cmp_le(ph_t - ph_r, -G_PH * th_r, ph_r)
        return th_t <= (1 - G_TH) * th_r or ph_t <= ph_r - G_PH * th_r + 1e-14 * abs(ph_r)

    def check_acceptability(self, th_t, ph_t, a_test, ref):
        """(accept, rejected by the filter)."""
        if not (th_t <= self.theta_max):
            return False, False
        if a_test > 0 and self.is_ftype(a_test, ref) and ref["th"] <= self.theta_min:
            ok = self.armijo(ph_t, a_test, ref)
        else:
            ok = self.acc_to_iterate(th_t, ph_t, ref)
        if not ok:
            return False, False
        if not self.filt.ok(th_t, ph_t):
            return False, True
        return True, False

    def alpha_min(self, E, gphi):
        th = E["theta"]
        a = G_TH
        if gphi < 0:
            a = min(G_TH, G_PH * th / (-gphi))
            if th <= self.theta_min:
                a = min(a, DELTA_SW * th ** S_THETA / (-gphi) ** S_PHI)
        return 0.05 * a

    # ---------------- trial points ----------------
    def trial(self, it, dr, alpha):
        t = it.copy()
        t.x = it.x + alpha * dr["x"]
        t.s = it.s + alpha * dr["s"]
        f, c, d = self.P.primal(t.x)
        th = float(np.abs(c).sum() + np.abs(d - t.s).sum())
        ph = self.barrier(f, t.x, t.s, self.mu)
        if not (np.isfinite(th) and np.isfinite(ph)):
            return t, math.inf, math.inf, False
        return t, th, ph, True

    def dual_step(self, it, t, dr, a_p, a_d, mu):
        t.vL = it.vL + a_d * dr["vL"]
        t.vU = it.vU + a_d * dr["vU"]
        t.zL = it.zL + a_d * dr["zL"]
        t.yc = it.yc + a_p * dr["yc"]
        t.yd = it.yd + a_p * dr["yd"] if self.R.separate_yd else it.yd

    def kappa_sigma(self, t, mu):
        SL, SU, X = self.dist(t)
        t.vL[self.mL] = np.clip(t.vL[self.mL], mu / (KAPPA_SIGMA * SL), KAPPA_SIGMA * mu / SL)
        t.vU[self.mU] = np.clip(t.vU[self.mU], mu / (KAPPA_SIGMA * SU), KAPPA_SIGMA * mu / SU)
        t.zL[self.mx] = np.clip(t.zL[self.mx], mu / (KAPPA_SIGMA * X), KAPPA_SIGMA * mu / X)

    def pd_error(self, it, mu):
        """primal_dual_system_error (1-norms averaged), for the soft restoration phase."""
        E = self.measure(it)
        SL, SU, X = self.dist(it)
        prods = np.concatenate([it.vL[self.mL] * SL, it.vU[self.mU] * SU, it.zL[self.mx] * X])
        num = (np.abs(E["glx"]).sum() + np.abs(E["gls"]).sum() + np.abs(E["ev"]["c"]).sum()
               + np.abs(E["rd"]).sum() + np.abs(prods - mu).sum())
        den = it.x.size + it.s.size + it.yc.size + it.s.size + prods.size
        return num / max(den, 1)

    def try_soc(self, it, E, F, dr, a_trial, th_trial, a_test, ref):
        """TrySecondOrderCorrection: up to max_soc linear corrections on the stored factorisation."""
        c_soc = E["ev"]["c"].copy()
        r_soc = E["rd"].copy()
        a_soc = a_trial
        count, th_old = 0, 0.0
        tau = max(0.99, 1.0 - self.mu)
        last = None
        while count < self.R.max_soc and (count == 0 or th_trial <= KAPPA_SOC * th_old):
            th_old = th_trial
            xt = it.x + a_soc * dr["x"] if last is None else last[0].x
            st = it.s + a_soc * dr["s"] if last is None else last[0].s
            _f, ct, dt = self.P.primal(xt)
            c_soc = a_soc * c_soc + ct
            r_soc = a_soc * r_soc + (dt - st)
            ds = self.solve(F, it, E, self.mu, c_soc, r_soc)
            self.stats["soc_tries"] += 1
            a_soc = self.alpha_primal_max(it, ds, tau)
            t, th_t, ph_t, fin = self.trial(it, ds, a_soc)
            if not fin:
                break
            ok, rj = self.check_acceptability(th_t, ph_t, a_test, ref)
            self.last_rej = self.last_rej or rj
            if ok:
                self.stats["soc_acc"] += 1
                return True, a_soc, ds, t
            count += 1
            th_trial = th_t
            last = (t,)
        return False, None, None, None

    def try_reroll(self, it, t_plain, th_t, a_test, ref):
        """Round-3 SOC: the trial controls / progress kept, the shooting states re-simulated."""
        xs = self.P.soc_roll(t_plain.x)
        _f, _c, d_plain = self.P.primal(t_plain.x)
        f2, c2, d2 = self.P.primal(xs)
        ss = t_plain.s + (d2 - d_plain)
        t = t_plain.copy()
        t.x, t.s = xs, ss
        th = float(np.abs(c2).sum() + np.abs(d2 - ss).sum())
        ph = self.barrier(f2, xs, ss, self.mu)
        if not np.isfinite(ph):
            return False, None
        ok, rj = self.check_acceptability(th, ph, a_test, ref)
        self.last_rej = self.last_rej or rj
        return ok, t

    def backtrack(self, it, E, F, dr, ref, skip_first):
        """DoBacktrackingLineSearch: (accept, trial, alpha, a_test, dr, n_steps)."""
        tau = max(0.99, 1.0 - self.mu)
        a_max = self.alpha_primal_max(it, dr, tau)
        a_min = a_max if self.in_wd else self.alpha_min(E, ref["gphi_cur"])
        alpha = a_max * (0.5 if skip_first else 1.0)
        n_steps = 0
        th_cur = E["theta"]
        while n_steps < 1100:
            if self.R.first_trial:
                if not (alpha > a_min or n_steps == 0):
                    break
            elif not (alpha >= a_min and alpha >= 1e-30):
                break
            a_test = self.wd["a_test"] if self.in_wd else alpha
            t, th_t, ph_t, fin = self.trial(it, dr, alpha)
            ok = False
            if fin:
                ok, rj = self.check_acceptability(th_t, ph_t, a_test, ref)
                self.last_rej = self.last_rej or rj
            if ok:
                return True, t, alpha, a_test, dr, n_steps
            if self.in_wd and not self.R.soc_in_watchdog:
                break
            if self.R.max_soc > 0:
                if fin and alpha == a_max and th_cur <= th_t:
                    ok, a2, d2, t2 = self.try_soc(it, E, F, dr, alpha, th_t, a_test, ref)
                    if ok:
                        return True, t2, a2, a_test, d2, n_steps
            elif self.R.max_soc < 0 and self.P.soc_roll is not None and n_steps == 0 and not skip_first:
                if th_t >= ref["th"] and not self.resto:
                    ok, t2 = self.try_reroll(it, t, th_t, a_test, ref)
                    if ok:
                        return True, t2, alpha, a_test, dr, n_steps
            if self.in_wd:
                break
            alpha *= 0.5
            n_steps += 1
        return False, None, alpha, alpha, dr, n_steps

    def try_soft_resto(self, it, E, dr):
        """TrySoftRestoStep: (accept, satisfies the original criterion, trial)."""
        tau = max(0.99, 1.0 - self.mu)
        self.stats["soft"] += 1
        a = min(self.alpha_primal_max(it, dr, tau), self.alpha_dual_max(it, dr, tau))
        t, th_t, ph_t, fin = self.trial(it, dr, a)
        if not fin:
            return False, False, None, a
        self.dual_step(it, t, dr, a, a, self.mu)
        ref = dict(th=E["theta"], ph=E["phi"], gphi=E["gphi"])
        ok, _rj = self.check_acceptability(th_t, ph_t, 0.0, ref)
        if ok:
            self.stats["soft_acc"] += 1
            return True, True, t, a
        if self.pd_error(t, self.mu) <= SOFT_RESTO_FACTOR * self.pd_error(it, self.mu):
            return True, False, t, a
        return False, False, None, a

    # ---------------- the restoration phase ----------------
    def restoration(self, it, E, k):
        """RestoMinC_1Nrm::PerformRestoration from ``it``: (status, iterate, iteration count)."""
        P, R = self.P, self.R
        self.stats["resto"] += 1
        n = P.n
        ev = E["ev"]
        mc, md = ev["c"].size, ev["d"].size
        mu_r = max(self.mu, E["pr_inf"])
        xR = it.x.copy()
        DR2 = np.minimum(1.0, 1.0 / np.maximum(np.abs(xR), 1e-300)) ** 2
        rel = np.ones(mc, dtype=bool)  # the relaxed equality rows
        if not R.resto_relax_x0:
            rel[:P.x0_rows] = False
        mr = int(rel.sum())
        rel_t = torch.tensor(np.nonzero(rel)[0], dtype=torch.long)
        pc, nc = _pn(ev["c"][rel], mu_r, RHO)
        pd, nd = _pn(ev["d"] - it.s, mu_r, RHO)
        ia = np.cumsum([0, n, mr, mr, md, md])
        zeta = [math.sqrt(mu_r)]
        xRt, DR2t = _T(xR), _T(DR2)
        f, c, d, lh = P.f, P.c, P.d, P.lag_hess

        def fR(v):
            return RHO * torch.sum(v[n:]) + 0.5 * zeta[0] * torch.sum(DR2t * (v[:n] - xRt) ** 2)

        def cR(v):
            return c(v[:n]).index_add(0, rel_t, -v[ia[1]:ia[2]] + v[ia[2]:ia[3]])

        def dR(v):
            return d(v[:n]) - v[ia[3]:ia[4]] + v[ia[4]:ia[5]]

        def hR(v, wf, yc, yd):
            H = np.zeros((ia[5], ia[5]))
            H[:n, :n] = lh(v[:n], 0.0, yc, yd) + np.diag(wf * zeta[0] * DR2)
            return H
        xLR = np.concatenate([np.full(n, -np.inf), np.zeros(ia[5] - n)])
        PR = Problem(ia[5], fR, cR, dR, P.dL, P.dU, xLR, lag_hess=hR)
        rules_r = replace(R, soft_resto=False, acceptable_on_fail=False, resto_on_fact_fail=False,
                          shortest_step_if_feasible=False, unscaled_tests=False,
                          max_soc=R.max_soc if R.resto_soc else 0)
        A = _Alg(PR, rules_r, self.tol, self.max_iter, self.acc_tol, 0, self.log, unscale=(1.0, None, None),
                 resto=self)
        A.mu = mu_r
        A.first_iter = True

        def pre(mu):
            zeta[0] = math.sqrt(mu)
        A.pre_eval = pre
        v0 = np.concatenate([xR, pc, nc, pd, nd])
        pnv = v0[n:]
        vL = np.where(A.mL, it.vL, 0.0)
        vU = np.where(A.mU, it.vU, 0.0)
        if R.resto_v_init == "min_rho":
            vL, vU = np.minimum(vL, RHO), np.minimum(vU, RHO)
        else:
            SL, SU, _X = self.dist(it)
            vL = np.zeros_like(it.s)
            vU = np.zeros_like(it.s)
            vL[A.mL] = mu_r / SL
            vU[A.mU] = mu_r / SU
        zL = np.concatenate([np.zeros(n), mu_r / pnv])
        itR = _It(v0, it.s.copy(), np.zeros(mc), np.zeros(md), zL, vL, vU)
        if R.resto_ls_mult:
            A.ls_mults(itR)
        A.orig_ref = dict(th=E["theta"], ph=E["phi"])
        A.orig_mu = self.mu
        status, itR2, k2 = A.optimize(itR, k)
        self.resto_why = getattr(A, "why", "")
        x_new, s_new = itR2.x[:n], itR2.s
        if status != 0:
            out = it.copy()
            out.x, out.s = x_new, s_new
            return status, out, k2
        t = it.copy()
        t.x, t.s = x_new, s_new
        if R.resto_mult == "newton":
            # the whole restoration as one primal Newton step: dz = mu/S - z - z/S dS at the entry point
            SL, SU, X = self.dist(it)
            SL2, SU2, X2 = self.dist(t)
            dr = dict(vL=np.zeros_like(it.vL), vU=np.zeros_like(it.vU), zL=np.zeros_like(it.zL))
            dr["vL"][self.mL] = self.mu / SL - it.vL[self.mL] - it.vL[self.mL] / SL * (SL2 - SL)
            dr["vU"][self.mU] = self.mu / SU - it.vU[self.mU] - it.vU[self.mU] / SU * (SU2 - SU)
            dr["zL"][self.mx] = self.mu / X - it.zL[self.mx] - it.zL[self.mx] / X * (X2 - X)
            a_d = self.alpha_dual_max(it, dr, max(0.99, 1.0 - self.mu))
            t.vL, t.vU, t.zL = it.vL + a_d * dr["vL"], it.vU + a_d * dr["vU"], it.zL + a_d * dr["zL"]
            bmax = max(np.abs(t.vL).max(initial=0.0), np.abs(t.vU).max(initial=0.0), np.abs(t.zL).max(initial=0.0))
            if bmax > MULT_RESET:
                t.vL = np.where(self.mL, 1.0, 0.0)
                t.vU = np.where(self.mU, 1.0, 0.0)
                t.zL = np.where(self.mx, 1.0, 0.0)
        else:  # round 3: mu / S, reset where the change exceeds 1000
            SL2, SU2, X2 = self.dist(t)
            vR = itR2.vL
            t.vL = np.zeros_like(it.vL)
            t.vL[self.mL] = np.where(np.abs(self.mu / SL2 - vR[self.mL]) > MULT_RESET, 1.0, self.mu / SL2)
            t.vU = np.zeros_like(it.vU)
            t.vU[self.mU] = self.mu / SU2
        t.yc = np.zeros_like(it.yc)
        t.yd = np.zeros_like(it.yd)
        self.kappa_sigma(t, self.mu)
        return 0, t, k2

    def resto_progress(self, it):
        """RestoConvergenceCheck: the accepted restoration iterate seen by the original problem."""
        O = self.resto
        n = O.P.n
        x, s = it.x[:n], it.s
        f, c, d = O.P.primal(x)
        th = float(np.abs(c).sum() + np.abs(d - s).sum())
        ph = O.barrier(f, x, s, self.orig_mu)
        if not (th <= KAPPA_RESTO * self.orig_ref["th"]):
            return False
        if not O.filt.ok(th, ph):
            return False
        return O.acc_to_iterate(th, ph, self.orig_ref, from_resto=True)

    # ---------------- initialisation ----------------
    def ls_mults(self, it):
        """least_square_mults: y minimising ||grad_x L||^2 + ||grad_s L||^2; zero if max |y| > 1000."""
        ev = self.P.evaluate(it.x)
        n, mc, md = it.x.size, it.yc.size, it.yd.size
        rx = -(ev["gf"] - np.where(self.mx, it.zL, 0.0))
        rs = np.where(self.mL, it.vL, 0.0) - np.where(self.mU, it.vU, 0.0)
        A = np.zeros((n + md, mc + md))
        A[:n, :mc] = ev["Jc"].T
        A[:n, mc:] = ev["Jd"].T
        A[n:, mc:] = -np.eye(md)
        y = np.linalg.lstsq(A, np.concatenate([rx, rs]), rcond=None)[0]
        if np.abs(y).max(initial=0.0) > 1000.0 or not np.isfinite(y).all():
            y = np.zeros_like(y)
        it.yc, it.yd = y[:mc].copy(), y[mc:].copy()

    def initial_iterate(self, x0):
        P = self.P
        _f, c, d = P.primal(x0)
        s = d.copy()
        if P.push is not None:
            s = np.maximum(s, P.push)
        else:
            rng = P.dU - P.dL
            bL = np.where(self.mL, np.abs(P.dL), 0.0)
            bU = np.where(self.mU, np.abs(P.dU), 0.0)
            two = self.mL & self.mU
            pL = 1e-2 * np.maximum(1.0, bL)
            pU = 1e-2 * np.maximum(1.0, bU)
            pL = np.where(two, np.minimum(pL, 1e-2 * np.where(two, rng, 1.0)), pL)
            pU = np.where(two, np.minimum(pU, 1e-2 * np.where(two, rng, 1.0)), pU)
            s = np.where(self.mL, np.maximum(s, P.dL + pL), s)
            s = np.where(self.mU, np.minimum(s, P.dU - pU), s)
        it = _It(np.asarray(x0, np.float64).copy(), s, np.zeros(c.size), np.zeros(d.size),
                 np.where(self.mx, 1.0, 0.0), np.where(self.mL, 1.0, 0.0), np.where(self.mU, 1.0, 0.0))
        if self.R.ls_mult_init:
            self.ls_mults(it)
        return it

    # ---------------- the main loop ----------------
    def update_mu(self, E):
        mu_old = self.mu
        err = self.barrier_error(E, self.mu)
        tiny = self.tiny_flag
        self.tiny_flag = False
        if self.resto is not None and self.first_iter:
            return False
        changed_any = False
        while (err <= KAPPA_EPS * self.mu or tiny):
            new = max(self.mu_floor, min(KAPPA_MU * self.mu, self.mu ** THETA_MU))
            changed = new != self.mu
            if not changed and tiny:
                return "tiny"
            self.mu = new
            tiny = False
            if not changed:
                break
            changed_any = True
            err = self.barrier_error(E, self.mu)
        if self.mu != mu_old:
            self.reset_ls()
        return changed_any

    def reset_ls(self):
        self.filt.e = []
        self.in_wd, self.wd_short, self.wd = False, 0, None
        self.in_soft, self.soft_count = False, 0

    def optimize(self, it, k):
        R = self.R
        status, kkt = 2, math.inf
        while True:
            if self.pre_eval is not None:
                self.pre_eval(self.mu)
            E = self.measure(it)
            E["phi"] = self.barrier(E["ev"]["f"], it.x, it.s, self.mu)
            kkt = E["nlp_err"]
            if not (np.isfinite(kkt) and np.isfinite(E["ev"]["f"])):
                status, self.why = 3, "nonfinite"
                break
            # RestoConvergenceCheck (after the first restoration iteration)
            if self.resto is not None and not self.first_iter and self.resto_progress(it):
                status, self.why = 0, "resto_return"
                break
            du, cv, co = E["unscaled"]
            if kkt <= self.tol and (not R.unscaled_tests or self.resto is not None
                                    or (du <= DUAL_INF_TOL and cv <= CONSTR_VIOL_TOL and co <= COMPL_INF_TOL)):
                if self.resto is None:
                    status = 0
                else:
                    n = self.resto.P.n
                    _f, c, d = self.resto.P.primal(it.x[:n])
                    prinf = max(np.abs(c).max(initial=0.0), np.abs(d - it.s).max(initial=0.0))
                    status = 3 if (R.resto_feasible_status and prinf <= 1e2 * self.tol) else 4
                    self.why = "resto_converged_feasible" if status == 3 else "locally_infeasible"
                break
            if self.resto is None and self.acc_iter > 0:
                self.acc_count = self.acc_count + 1 if self.is_acceptable(E) else 0
                if self.acc_count >= self.acc_iter:
                    status, self.why = 1, "acceptable_iter"
                    break
            if k >= self.max_iter:
                status, self.why = 2, "max_iter"
                break
            if self.update_mu(E) == "tiny":
                status, self.why = 3, "tiny_step"  # Search_Direction_Becomes_Too_Small
                break
            self.first_iter = False
            E["phi"] = self.barrier(E["ev"]["f"], it.x, it.s, self.mu)
            F = self.factorize(it, E, self.mu)
            if F is None:
                if self.resto is None and R.resto_on_fact_fail:
                    self.filt.add(E["theta"], E["phi"])
                    st, it2, k = self.restoration(it, E, k + 1)
                    if st != 0:
                        status, it = st, it2
                        break
                    it = it2
                    self.after_resto()
                    continue
                status, self.why = 3, "factorization"
                break
            dr = self.solve(F, it, E, self.mu, E["ev"]["c"], E["rd"])
            E["gphi"] = self.grad_barr_t_delta(E, it, dr, self.mu)
            if self.theta_max is None:
                self.theta_max = 1e4 * max(1.0, E["theta"])
                self.theta_min = 1e-4 * max(1.0, E["theta"])
            res = self.line_search(it, E, F, dr, k)
            if res[0] == "stop":
                status, it = res[1], res[2]
                self.why = res[3]
                break
            if res[0] == "resto":
                self.filt.add(E["theta"], E["phi"])
                st, it2, k = self.restoration(it, E, k + 1)
                if st != 0:
                    status, it = st, it2
                    break
                it = it2
                self.after_resto()
                continue
            _tag, t, alpha, delta = res
            it = t
            k += 1
            if self.log is not None:
                self.log.append((k, kkt, self.mu, alpha, F["delta"], self.log_ref[0], self.log_ref[1],
                                 self.resto is not None))
        return status, it, k

    def after_resto(self):
        self.in_wd, self.wd_short, self.wd = False, 0, None
        self.in_soft, self.soft_count = False, 0
        self.acc_count = 0
        self.filt_rej_iters = 0

    def line_search(self, it, E, F, dr, k):
        """FindAcceptableTrialPoint: ("ok", iterate, alpha, delta) / ("resto",) / ("stop", status, iterate)."""
        R = self.R
        self.last_rej = False
        self.log_ref = (E["theta"], E["phi"])
        if R.acceptable_on_fail and self.resto is None and self.is_acceptable(E):
            self.acc_point = it.copy()
        cur_ref = dict(th=E["theta"], ph=E["phi"], gphi=E["gphi"], gphi_cur=E["gphi"])
        accept, soft_step, take_anyway, tiny = False, False, False, False
        a_test = 0.0
        t = alpha = None
        n_steps = 0
        tau = max(0.99, 1.0 - self.mu)
        ref = cur_ref
        ws = WD_TRIGGER if (self.resto is None or R.resto_watchdog) else 0
        if self.in_soft:
            self.soft_count += 1
            if self.soft_count <= MAX_SOFT_RESTO:
                accept, orig, t, alpha = self.try_soft_resto(it, E, dr)
                if accept:
                    soft_step = True
                    if orig:
                        self.in_soft, self.soft_count = False, 0
        else:
            if ws and not self.in_wd and self.wd_short >= ws:
                self.stats["wd_start"] += 1
                self.in_wd, self.wd_trial = True, 0
                self.wd = dict(it=it.copy(), E=E, F=F, dr=dr, ref=dict(cur_ref),
                               a_test=self.alpha_primal_max(it, dr, tau))
            if self.in_wd:
                ref = dict(self.wd["ref"], gphi_cur=E["gphi"])
            if R.tiny_step and self.detect_tiny(it, E, dr):
                alpha = self.alpha_primal_max(it, dr, tau)
                t, _th, _ph, _fin = self.trial(it, dr, alpha)
                accept, tiny, a_test = True, True, alpha
                # tiny_step_y_tol 1e-2: the flag (a forced barrier decrease, or the stop) only when the
                # constraint multipliers' step is small too
                self.tiny_flag = (np.abs(dr["yc"]).max(initial=0.0) < 1e-2
                                  and np.abs(dr["yd"]).max(initial=0.0) < 1e-2)
                self.stats["tiny"] += 1
            else:
                skip_first = False
                while True:
                    accept, t, alpha, a_test, dr2, n_steps = self.backtrack(it, E, F, dr, ref, skip_first)
                    if self.in_wd:
                        if accept:
                            self.in_wd, self.wd_short = False, 0
                        else:
                            self.wd_trial += 1
                            if self.wd_trial > WD_TRIAL_MAX:
                                self.stats["wd_stop"] += 1
                                w = self.wd
                                it, E, F, dr = w["it"], w["E"], w["F"], w["dr"]
                                self.in_wd, self.wd_short, self.wd = False, 0, None
                                ref = cur_ref = dict(w["ref"], gphi_cur=w["ref"]["gphi"])
                                skip_first = True
                                continue
                            take_anyway = True
                            alpha = self.alpha_primal_max(it, dr, tau)
                            t, _th, _ph, _fin = self.trial(it, dr, alpha)
                            accept = True
                            dr2 = dr
                    dr = dr2
                    break
            if not accept and R.soft_resto and self.resto is None:
                accept, orig, t, alpha = self.try_soft_resto(it, E, dr)
                if accept:
                    soft_step = True
                    self.in_soft = not orig
                    self.soft_count = 0
        if not accept:
            self.stats["ls_fail"] += 1
            if self.resto is not None:
                return ("stop", 3, it, "resto_line_search")
            if R.acceptable_on_fail:
                if self.is_acceptable(E):
                    return ("stop", 1, it, "acceptable_at_ls_failure")
                if E["theta"] <= 1e-2 * self.tol:
                    if self.acc_point is not None:
                        return ("stop", 1, self.acc_point, "acceptable_point_restored")
                    return ("stop", 3, it, "almost_feasible_ls_failure")
            if R.shortest_step_if_feasible and E["pr_inf"] <= self.tol:
                alpha = min(max(alpha, self.alpha_min(E, E["gphi"])), self.alpha_primal_max(it, dr, tau))
                t, _th, _ph, _fin = self.trial(it, dr, alpha)
                a_test = alpha
                accept = True
                self.dual_step(it, t, dr, alpha, self.alpha_dual_max(it, dr, tau), self.mu)
                self.kappa_sigma(t, self.mu)
                self.wd_short = 0
                self.filt_reset_check()
                self.filt.add(cur_ref["th"], cur_ref["ph"])
                return ("ok", t, alpha, F["delta"])
            return ("resto",)
        # the accepted point: dual step, kappa_sigma, watchdog counter, filter
        if not soft_step:
            a_d = self.alpha_dual_max(it, dr, tau)
            self.dual_step(it, t, dr, alpha, a_d, self.mu)
        self.kappa_sigma(t, self.mu)
        if not take_anyway and not soft_step and not tiny:
            self.wd_short = self.wd_short + 1 if alpha < self.alpha_primal_max(it, dr, tau) else 0
        self.filt_reset_check()
        self.log_ref = (ref["th"], ref["ph"])
        if not take_anyway:
            if soft_step:
                if not self.in_soft:  # 'S': accepted by the original criterion (alpha_test 0: h-type)
                    self.filt.add(ref["th"], ref["ph"])
            elif not tiny:
                if R.ftype_rule == "ipopt":
                    _f, _c, _d = self.P.primal(t.x)
                    ph_t = self.barrier(_f, t.x, t.s, self.mu)
                    if not (self.is_ftype(a_test, ref) and self.armijo(ph_t, a_test, ref)):
                        self.filt.add(ref["th"], ref["ph"])
                else:
                    if not (ref["th"] <= self.theta_min and self.is_ftype(a_test, ref)):
                        self.filt.add(ref["th"], ref["ph"])
        return ("ok", t, alpha, F["delta"])

    def filt_reset_check(self):
        if self.filt_resets < MAX_FILTER_RESETS:
            self.filt_rej_iters = self.filt_rej_iters + 1 if self.last_rej else 0
            if self.filt_rej_iters >= FILTER_RESET_TRIGGER:
                self.filt.e = []
                self.filt_resets += 1
                self.stats["filt_resets"] += 1
                self.filt_rej_iters = 0

    def detect_tiny(self, it, E, dr):
        if np.abs(dr["x"] / (1.0 + np.abs(it.x))).max(initial=0.0) > 10 * EPS:
            return False
        if np.abs(dr["s"] / (1.0 + np.abs(it.s))).max(initial=0.0) > 10 * EPS:
            return False
        return E["pr_inf"] <= 1e-4


def make_problem(prob, rules=IPOPT):
    """The reference's NLP (oracle.nlp.MPCProblem) as IPOPT receives it (rules.opti_rows) or in the
    round-3 one-sided form."""
    n = prob.n
    if rules.opti_rows:
        d, dL, dU, _kinds = prob.ipopt_ineq()
        bl = rules.bound_relax_factor
        if bl:
            rl = np.minimum(CONSTR_VIOL_TOL, bl * np.maximum(1.0, np.abs(dL)))
            ru = np.minimum(CONSTR_VIOL_TOL, bl * np.maximum(1.0, np.abs(dU)))
            dL = np.where(np.isfinite(dL), dL - rl, dL)
            dU = np.where(np.isfinite(dU), dU + ru, dU)
        return Problem(n, prob.f, prob.g, d, dL, dU, soc_roll=prob.rollout, x0_rows=7)  # g: S_0, X_0, dynamics
    mi = prob.push().size
    return Problem(n, prob.f, prob.g, prob.d, np.zeros(mi), np.full(mi, np.inf), soc_roll=prob.rollout,
                   push=prob.push())


def solve_ipopt(prob, tol=1e-8, max_iter=500, acceptable_tol=1e-6, acceptable_iter=15, w0=None, log=False,
                rules=IPOPT):
    """IPOPT on MPCProblem ``prob`` (module docstring); returns nlp.IPMResult with status 0 solved,
    1 acceptable, 2 max_iter, 3 failed, 4 infeasible (the product's MR_STATUS_* codes).  ``nu`` = the
    equality multipliers y_c, ``lam`` = the inequality multipliers y_d (IPOPT's sign: L = f + y.g), both
    for the unscaled objective; ``r.max_row_gradient`` = the largest constraint-row gradient at w0."""
    w_init = np.array(prob.initial_guess() if w0 is None else w0, dtype=np.float64)
    P0 = make_problem(prob, rules)
    PS, df, dc, dd, mrg = _scaled(P0, w_init, rules)
    logl = [] if log else None
    A = _Alg(PS, rules, tol, max_iter, acceptable_tol, acceptable_iter, logl, unscale=(df, dc, dd))
    it0 = A.initial_iterate(w_init)
    status, it, k = A.optimize(it0, 0)
    why = getattr(A, "why", "")
    if getattr(A, "resto_why", None):
        why = why + "/" + A.resto_why if why else A.resto_why
    Ef = A.measure(it)
    r = IPMResult(w=it.x, nu=it.yc * dc / df, lam=A.yd_of(it) * dd / df, s=it.s / dd, iters=k, status=status,
                  kkt=float(Ef["nlp_err"]), obj=float(prob.f(_T(it.x))))
    r.max_row_gradient = mrg
    r.why = why
    r.stats = A.stats
    r.obj_scale = df
    if log:
        r.log = logl
    return r
