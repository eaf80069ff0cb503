"""Drop-in ``splines.ParameterizedLine`` (splines/ParameterizedLine.py:12-178) whose queries run on
the GPU (``mpcracing.geometry.DeviceTrack``, kernels in ``csrc/mr_track.h``).

Same attributes (``spline_x, spline_y, length, waypoints``) and methods.  ``from_waypoints``
(:162-178) builds the chord-length not-a-knot cubic in the library's host code
(``mr_spline_from_waypoints``: knots and length bit-exact with scipy's ``make_interp_spline``,
G1); ``spline_x`` / ``spline_y`` are scipy ``BSpline`` views of the same tables (host-side
callers such as ``TrackSegments``).  Query methods take scalars (scalar results) or arrays.

Differences from the reference, both documented in DESIGN.md: ``projection_global`` (:99-105,
scipy's unseeded ``dual_annealing``) is a deterministic search -- the local bounded Brent on every
5 m window, best distance wins; ``x_as_coeffs`` / ``y_as_coeffs`` take degrees 0..10 on the device
(``mr_track_polyfit_deg``; the agent uses the quartic), the reference's ``np.polyfit`` any degree.
"""
import numpy as np

from splines.util import euclidean  # noqa: F401  (re-exported like the reference module)


def _out(v, scalar):
    a = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
    return float(a.reshape(-1)[0]) if scalar else a


class ParameterizedLine:
    def __init__(self):
        self.spline_x = None
        self.spline_y = None
        self.length = None
        self.waypoints = None
        self._tables = None   # (t, cx, cy, L, err_left, err_right)
        self._dev = None
        self.device = 0

    # ---- construction ----
    def from_file(self, fp):
        raise NotImplementedError()

    def from_waypoints(self, waypoints):
        from mpcracing import abi
        from mpcracing.geometry import native_spline
        x = np.array([p[0] for p in waypoints], dtype=np.float64)
        y = np.array([p[1] for p in waypoints], dtype=np.float64)
        t, cx, cy, L = native_spline(abi.load_product(), x, y, close_loop=False)
        self._set_tables(t, cx, cy, L)
        self.waypoints = list(zip(x, y))

    def _set_tables(self, t, cx, cy, L, err_left=None, err_right=None):
        from scipy.interpolate import BSpline
        self._tables = (np.asarray(t), np.asarray(cx), np.asarray(cy), float(L), err_left, err_right)
        self.spline_x = BSpline(np.asarray(t), np.asarray(cx), 3)
        self.spline_y = BSpline(np.asarray(t), np.asarray(cy), 3)
        self.length = float(L)
        self._dev = None

    @property
    def dev(self):
        if self._dev is None:
            from mpcracing.geometry import DeviceTrack
            if self._tables is None:
                raise RuntimeError("line not built: call from_waypoints / from_file first")
            self._dev = DeviceTrack(device=self.device, tables=self._tables)
        return self._dev

    @property
    def host_track(self):
        """Host evaluation of the same spline (scipy BSpline), for setup-time helpers."""
        return _HostLine(self)

    # ---- spline values (:19-41) ----
    def _eval(self, s, j):
        out, _ = self.dev.eval(s)
        return _out(out[j], np.ndim(s) == 0)

    def Gx(self, s):
        return self._eval(s, 0)

    def Gy(self, s):
        return self._eval(s, 1)

    def dGx(self, s):
        return self._eval(s, 2)

    def dGy(self, s):
        return self._eval(s, 3)

    def ddGx(self, s):
        return self._eval(s, 4)

    def ddGy(self, s):
        return self._eval(s, 5)

    # ---- local polynomial (:43-64) ----
    def x_as_coeffs(self, s, lookahead, deg=4):
        """deg 0..10 on the device (mr_track_polyfit_deg); the reference's np.polyfit takes any degree but
        warns that high ones are ill-conditioned -- above 10 the global-s monomial coefficients carry no
        digits in fp64."""
        cx, _ = self.dev.polyfit([s], lookahead, deg=int(deg))
        return list(cx[:, 0].cpu().numpy())

    def y_as_coeffs(self, s, lookahead, deg=4):
        _, cy = self.dev.polyfit([s], lookahead, deg=int(deg))
        return list(cy[:, 0].cpu().numpy())

    # ---- projection (:66-105) ----
    def projection(self, X, Y, bounds=None):
        if bounds is None or 5 < abs(bounds[1] - bounds[0]):
            return self.projection_global(X, Y)
        return self.projection_local(X, Y, bounds=bounds)

    def projection_local(self, X, Y, bounds=None, warn=True):
        if bounds is None:
            bounds = (0, self.length)
        if warn is True and (bounds[1] - bounds[0]) > 10:
            print("Warning: local projection over with large bounds", bounds)
        s, d, _ = self.dev.projection([X], [Y], [bounds[0]], [bounds[1]])
        return float(s[0]), float(d[0])

    def projection_global(self, X, Y):
        lo = np.arange(0.0, self.length, 5.0)
        hi = np.minimum(lo + 5.0, self.length)
        n = len(lo)
        s, d, _ = self.dev.projection(np.full(n, X), np.full(n, Y), lo, hi)
        i = int(np.argmin(d.cpu().numpy()))
        return float(s[i]), float(d[i])

    # ---- frame (:107-149) ----
    def unit_tangent(self, s):
        out, _ = self.dev.eval([s])
        d = out[2:4, 0].cpu().numpy()
        return d / np.linalg.norm(d)

    def unit_tangent_yaw(self, s):
        return float(self.dev.frame([s])["yaw"][0])

    def curvature(self, s):
        f = self.dev.frame(np.atleast_1d(s))["curvature"]
        return _out(f, np.ndim(s) == 0)

    def mean_curvature(self, s, lookahead, N=10):
        if N == 10:
            return float(self.dev.frame([s], mc_lookahead=lookahead)["mean_curvature"][0])
        ks = self.dev.frame(np.linspace(s, s + lookahead, N))["curvature"].cpu().numpy()
        return (1 / N) * sum(ks.tolist())

    def unit_principal_normal(self, s):
        f = self.dev.frame([s])
        return float(f["nx"][0]), float(f["ny"][0])


class _HostLine:
    """dGx / dGy / ddGx / ddGy / Gx / Gy of a ParameterizedLine on the host (s mod L, scipy)."""

    def __init__(self, line):
        self.length = line.length
        self._x, self._y = line.spline_x, line.spline_y
        self._dx, self._dy = self._x.derivative(), self._y.derivative()
        self._ddx, self._ddy = self._dx.derivative(), self._dy.derivative()

    def Gx(self, s):
        return self._x(s % self.length)

    def Gy(self, s):
        return self._y(s % self.length)

    def dGx(self, s):
        return self._dx(s % self.length)

    def dGy(self, s):
        return self._dy(s % self.length)

    def ddGx(self, s):
        return self._ddx(s % self.length)

    def ddGy(self, s):
        return self._ddy(s % self.length)
