"""Oracle restatement of the reference's centerline geometry (test infrastructure only).

Follows ``splines/ParameterizedLine.py`` / ``splines/ParameterizedCenterline.py``
of the reference and the scipy 1.15 algorithms they call:

* cubic B-spline evaluation: interval search (scipy ``_find_interval``) +
  Cox-de Boor basis recursion (scipy ``_deBoor_D`` with m = 0), summed in the
  order scipy uses;
* ``BSpline.derivative()``: the knot-dropping coefficient rule of scipy
  ``splder`` (the reference rebuilds the derivative spline on every call,
  ``ParameterizedLine.py:27-41``);
* ``np.polyfit`` (``ParameterizedLine.py:43-64``) — numpy is the pinned
  third-party dependency, so the oracle calls it on its own spline samples;
* bounded Brent (scipy ``_minimize_scalar_bounded``, xatol 1e-5, maxiter 500)
  as used by ``projection_local`` (``ParameterizedLine.py:80-97``);
* ``lookup_error`` with Python round-half-even (``ParameterizedCenterline.py:61-80``);
* the lane-width table build (``script/make_lane_width_lookup_table.py:12-16`` ->
  ``ParameterizedCenterline.get_errors(lane, s, 0)`` :41-58 -> ``projection_global``
  ``ParameterizedLine.py:99-105``): scipy's ``dual_annealing`` (unseeded) is restated as a
  deterministic global search -- nearest of the knot-interval start/midpoint samples, then the
  bounded Brent in its bracket.  Pinned against the reference's committed
  ``lanes/<track>_max_error.csv`` tables (tests/test_lane_table.py, 1e-4 m).
"""
import bisect
import math

import numpy as np


class Spline:
    """A scipy-layout B-spline (t, c, k) with extrapolate=True."""

    def __init__(self, t, c, k):
        self.t = np.asarray(t, dtype=np.float64)
        self.c = np.asarray(c, dtype=np.float64)
        self.k = int(k)
        self._tl = self.t.tolist()

    def span(self, x):
        """Interval index l with t[l] <= x < t[l+1], clamped to [k, n-1] (scipy _find_interval)."""
        t, k = self.t, self.k
        n = len(t) - k - 1
        if x != x:
            return k
        # largest l in [k, n-1] with t[l] <= x (bisection on the sorted knots)
        l = bisect.bisect_right(self._tl, x) - 1
        return min(max(l, k), n - 1)

    def __call__(self, x):
        t, c, k = self.t, self.c, self.k
        x = float(x)
        ell = self.span(x)
        h = [0.0] * (k + 1)
        h[0] = 1.0
        for j in range(1, k + 1):
            hh = h[:j]
            h[0] = 0.0
            for n in range(1, j + 1):
                ind = ell + n
                xb = t[ind]
                xa = t[ind - j]
                if xb == xa:
                    h[n] = 0.0
                    continue
                w = hh[n - 1] / (xb - xa)
                h[n - 1] += w * (xb - x)
                h[n] = w * (x - xa)
        acc = 0.0
        for a in range(k + 1):
            acc += c[ell + a - k] * h[a]
        return acc

    def derivative(self):
        t, c, k = self.t, self.c, self.k
        c = np.r_[c, np.zeros(len(t) - len(c))] if len(t) > len(c) else c.copy()
        dt = t[k + 1:-1] - t[1:-k - 1]
        cn = (c[1:-1 - k] - c[:-2 - k]) * k / dt
        cn = np.r_[cn, np.zeros(k)]
        return Spline(t[1:-1], cn, k - 1)


class Centerline:
    """Geometry queries of ParameterizedCenterline on a fixed spline table."""

    def __init__(self, t, cx, cy, length, err_ss=None, err_left=None, err_right=None):
        self.sx = Spline(t, cx, 3)
        self.sy = Spline(t, cy, 3)
        self.dsx = self.sx.derivative()
        self.dsy = self.sy.derivative()
        self.ddsx = self.dsx.derivative()
        self.ddsy = self.dsy.derivative()
        self.length = float(length)
        if err_ss is not None:
            self.err = {float(s): (float(l), float(r)) for s, l, r in zip(err_ss, err_left, err_right)}

    def _m(self, s):
        return s % self.length  # Python float modulo, as ``s % self.length`` in ParameterizedLine.py:20

    def Gx(self, s):
        return self.sx(self._m(s))

    def Gy(self, s):
        return self.sy(self._m(s))

    def dGx(self, s):
        return self.dsx(self._m(s))

    def dGy(self, s):
        return self.dsy(self._m(s))

    def ddGx(self, s):
        return self.ddsx(self._m(s))

    def ddGy(self, s):
        return self.ddsy(self._m(s))

    def x_as_coeffs(self, s, lookahead, deg=4):
        ss = np.linspace(0, lookahead, 50) + s
        return list(np.polyfit(ss, np.array([self.Gx(q) for q in ss]), deg=deg))

    def y_as_coeffs(self, s, lookahead, deg=4):
        ss = np.linspace(0, lookahead, 50) + s
        return list(np.polyfit(ss, np.array([self.Gy(q) for q in ss]), deg=deg))

    def dist(self, s, X, Y):
        return math.sqrt((self.Gx(s) - X) ** 2 + (self.Gy(s) - Y) ** 2)

    def projection_local(self, X, Y, bounds):
        xs = brent_bounded(lambda s: self.dist(s, X, Y), bounds[0], bounds[1])
        return xs, self.dist(xs, X, Y)

    def unit_tangent(self, s):
        d = np.array([self.dGx(s), self.dGy(s)])
        return d / np.linalg.norm(d)

    def unit_tangent_yaw(self, s):
        ut = self.unit_tangent(s)
        return float(np.arctan2(ut[1], ut[0]))

    def curvature(self, s):
        return abs(self.dGx(s) * self.ddGy(s) - self.dGy(s) * self.ddGx(s))

    def mean_curvature(self, s, lookahead, N=10):
        return (1 / N) * sum(self.curvature(q) for q in np.linspace(s, s + lookahead, N))

    def unit_principal_normal(self, s):
        ux, uy = self.unit_tangent(s)
        return uy, -ux

    def error_sign(self, X, Y, s):
        n = np.array(self.unit_principal_normal(s))
        d = np.array([X - self.Gx(s), Y - self.Gy(s)])
        return 1 if np.linalg.norm(d - n) < np.linalg.norm(d + n) else -1

    def lookup_error(self, s, lookahead):
        def r2(x):
            return round(x * 2) / 2  # Python round: half-to-even
        s_round = r2(s)
        la = r2(lookahead)
        left_min = 10000
        right_min = 10000
        for q in np.arange(s_round, s + la, 0.5):
            key = r2(q % self.length)
            left, right = self.err[key]  # pandas .loc row lookup
            if left < left_min:
                left_min = left
            if right < right_min:
                right_min = right
        return min(right_min, left_min)


def brent_bounded(func, x1, x2, xatol=1e-5, maxiter=500):
    """Bounded Brent minimiser, step-for-step scipy ``_minimize_scalar_bounded``."""
    sqrt_eps = math.sqrt(2.2e-16)
    golden_mean = 0.5 * (3.0 - math.sqrt(5.0))
    a, b = float(x1), float(x2)
    fulc = a + golden_mean * (b - a)
    nfc = xf = fulc
    rat = e = 0.0
    fx = func(xf)
    num = 1
    ffulc = fnfc = fx
    xm = 0.5 * (a + b)
    tol1 = sqrt_eps * abs(xf) + xatol / 3.0
    tol2 = 2.0 * tol1
    while abs(xf - xm) > (tol2 - 0.5 * (b - a)):
        golden = True
        if abs(e) > tol1:
            golden = False
            r = (xf - nfc) * (fx - ffulc)
            q = (xf - fulc) * (fx - fnfc)
            p = (xf - fulc) * q - (xf - nfc) * r
            q = 2.0 * (q - r)
            if q > 0.0:
                p = -p
            q = abs(q)
            r = e
            e = rat
            if abs(p) < abs(0.5 * q * r) and p > q * (a - xf) and p < q * (b - xf):
                rat = (p + 0.0) / q
                x = xf + rat
                if (x - a) < tol2 or (b - x) < tol2:
                    si = (1.0 if xm - xf > 0 else (-1.0 if xm - xf < 0 else 0.0)) + (1.0 if xm == xf else 0.0)
                    rat = tol1 * si
            else:
                golden = True
        if golden:
            e = (a - xf) if xf >= xm else (b - xf)
            rat = golden_mean * e
        si = (1.0 if rat > 0 else (-1.0 if rat < 0 else 0.0)) + (1.0 if rat == 0 else 0.0)
        x = xf + si * max(abs(rat), tol1)
        fu = func(x)
        num += 1
        if fu <= fx:
            if x >= xf:
                a = xf
            else:
                b = xf
            fulc, ffulc = nfc, fnfc
            nfc, fnfc = xf, fx
            xf, fx = x, fu
        else:
            if x < xf:
                a = x
            else:
                b = x
            if fu <= fnfc or nfc == xf:
                fulc, ffulc = nfc, fnfc
                nfc, fnfc = x, fu
            elif fu <= ffulc or fulc == xf or fulc == nfc:
                fulc, ffulc = x, fu
        xm = 0.5 * (a + b)
        tol1 = sqrt_eps * abs(xf) + xatol / 3.0
        tol2 = 2.0 * tol1
        if num >= maxiter:
            break
    return xf


def from_golden(g, track):
    """Oracle centerline built from the reference-produced golden spline table (G1)."""
    p = f"{track}/"
    return Centerline(g[p + "t"], g[p + "cx"], g[p + "cy"], float(g[p + "L"]))


class Lane:
    """A lane boundary (ParameterizedLane): the spline of lanes/<track>_{left,right}.csv."""

    def __init__(self, t, cx, cy, length):
        self.sx = Spline(t, cx, 3)
        self.sy = Spline(t, cy, 3)
        self.length = float(length)
        k = 3
        nspan = len(self.sx.t) - 2 * k - 1
        t = self.sx.t
        u = []
        for m in range(2 * nspan + 1):  # knot-interval starts and midpoints, then L
            if m >= 2 * nspan:
                u.append(float(t[k + nspan]))
            else:
                l = k + (m >> 1)
                u.append(float(t[l] + 0.5 * (t[l + 1] - t[l])) if m & 1 else float(t[l]))
        self.u = u
        self.px = np.array([self.sx(q) for q in u])
        self.py = np.array([self.sy(q) for q in u])

    def dist(self, s, X, Y):
        m = s % self.length
        return math.sqrt((self.sx(m) - X) ** 2 + (self.sy(m) - Y) ** 2)

    def distance_global(self, X, Y):
        """projection_global's minimum distance: nearest sample (first on ties), Brent in its bracket."""
        dx = self.px - X
        dy = self.py - Y
        mb = int(np.argmin(dx * dx + dy * dy))
        M = len(self.u)
        lo, hi = self.u[max(mb - 1, 0)], self.u[min(mb + 1, M - 1)]
        xs = brent_bounded(lambda q: self.dist(q, X, Y), lo, hi)
        return self.dist(xs, X, Y), xs


def lane_errors(center, lane, ss):
    """ParameterizedCenterline.get_errors(lane, s, 0) for each s (one row of the lane-width table)."""
    out = []
    for s in ss:
        X, Y = center.Gx(float(s)), center.Gy(float(s))
        out.append(lane.distance_global(X, Y)[0])
    return np.array(out)
