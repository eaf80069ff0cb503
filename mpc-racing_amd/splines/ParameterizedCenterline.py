"""Drop-in ``splines.ParameterizedCenterline`` whose per-tick queries run on the GPU.

Same constructor and query methods as the reference class
(splines/ParameterizedCenterline.py:12-105, ParameterizedLine.py:12-178) that the
agent calls every tick (agent.py:156-168, 271-274): ``Gx/Gy/dGx/dGy/ddGx/ddGy``,
``x_as_coeffs/y_as_coeffs``, ``projection`` (local bounded Brent), ``lookup_error``,
``error_sign``, ``unit_tangent``, ``unit_tangent_yaw``, ``curvature``,
``mean_curvature``, ``unit_principal_normal``.  Scalars in, scalars out (arrays
give arrays), computed by the kernels of ``mpcracing.geometry.DeviceTrack``.

``projection`` with bounds wider than 5 m (or none) falls to the reference's
``projection_global`` (scipy dual_annealing, unseeded and therefore not
reproducible); here it is a deterministic global search: the local Brent over
each 5 m window of the track, best distance wins.
"""
import numpy as np

from mpcracing.geometry import DeviceTrack


def _out(v, scalar):
    a = v.detach().cpu().numpy()
    return float(a.reshape(-1)[0]) if scalar else a


class ParameterizedCenterline:
    def __init__(self, track: str = "shanghai_intl_circuit", lanes=True, error=True, device=0):
        self.dev = DeviceTrack(track, device=device)
        self.length = self.dev.length
        self.track = track

    def _eval(self, s, j):
        sc = np.ndim(s) == 0
        out, _ = self.dev.eval(s)
        return _out(out[j], sc)

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

    def x_as_coeffs(self, s, lookahead, deg=4):
        if deg != 4:
            raise NotImplementedError("the device fit is the agent's quartic (POLY_DEG = 4, agent.py:140)")
        cx, _ = self.dev.polyfit([s], lookahead)
        return list(cx[:, 0].cpu().numpy())

    def y_as_coeffs(self, s, lookahead, deg=4):
        if deg != 4:
            raise NotImplementedError("the device fit is the agent's quartic (POLY_DEG = 4, agent.py:140)")
        _, cy = self.dev.polyfit([s], lookahead)
        return list(cy[:, 0].cpu().numpy())

    def projection(self, X, Y, bounds=None):
        if bounds is None or 5 < abs(bounds[1] - bounds[0]):
            return self.projection_global(X, Y)
        return self.projection_local(X, Y, bounds)

    def projection_local(self, X, Y, bounds=None, warn=True):
        if bounds is None:
            bounds = (0, self.length)
        s, d, _ = self.dev.projection([X], [Y], [bounds[0]], [bounds[1]])
        return float(s[0]), float(d[0])

    def projection_global(self, X, Y):
        lo = np.arange(0.0, self.length, 5.0)
        hi = np.minimum(lo + 5.0, self.length)
        n = len(lo)
        s, d, _ = self.dev.projection(np.full(n, X), np.full(n, Y), lo, hi)
        i = int(np.argmin(d.cpu().numpy()))
        return float(s[i]), float(d[i])

    def lookup_error(self, s, lookahead):
        err, _, _, _ = self.dev.lookup_error([s], lookahead)
        v = float(err[0])
        if v != v:
            raise KeyError(f"lane table has no row for the window of s={s} (reference: pandas KeyError)")
        return v

    def error_sign(self, X, Y, s):
        return int(self.dev.error_sign([X], [Y], [s])[0])

    def unit_tangent(self, s):
        out, _ = self.dev.eval([s])
        d = out[2:4, 0].cpu().numpy()
        return d / np.linalg.norm(d)

    def unit_tangent_yaw(self, s):
        return float(self.dev.frame([s])["yaw"][0])

    def curvature(self, s):
        return float(self.dev.frame([s])["curvature"][0])

    def mean_curvature(self, s, lookahead, N=10):
        if N != 10:
            raise NotImplementedError("mean_curvature uses N = 10 (the reference's default)")
        return float(self.dev.frame([s], mc_lookahead=lookahead)["mean_curvature"][0])

    def unit_principal_normal(self, s):
        f = self.dev.frame([s])
        return float(f["nx"][0]), float(f["ny"][0])
