"""Drop-in ``splines.TrackSegments`` (splines/TrackSegments.py:7-35), used by the GA
(GA/pdGA.py:3, GA/mpcGA.py:4) to split a lap into ``n_cp`` segments of equal model lap
time.  Same constructor and attributes (``line, n_cp, v_max, curve_c, lap_time, bounds``),
same quadrature (scipy ``quad``, limit 500) and root finder (``fsolve`` from the previous
bound), and the reference's curve radius kept as written,
``1 / |(G'x - G'y) G''y|``.

The integrand is evaluated on the host: ``centerline`` may be any object with
``dGy/dGx/ddGy`` and ``length`` (``mpcracing.track.Track``, or the drop-in
``splines.ParameterizedCenterline``, whose host spline is used instead of a device round
trip per quadrature node).  This is setup work outside the solve path.
"""
import math

from scipy import integrate, optimize


class TrackSegments:
    def __init__(self, centerline, n_cp, v_max, d_f, d_r, m):
        self.line = centerline
        self._geom = getattr(centerline, "host_track", None) or centerline
        self.n_cp = n_cp
        self.v_max = v_max
        self.curve_c = (2 * d_f + 2 * d_r) / m
        self.lap_time = self.segment_time(0, centerline.length)
        self.bounds = self.calculate_segment_bounds()

    def curve_radius(self, s):
        g = self._geom
        return 1 / abs((g.dGx(s) - g.dGy(s)) * g.ddGy(s))

    def curve_velocity(self, s):
        return min(self.v_max, math.sqrt(self.curve_radius(s) * self.curve_c))

    def segment_time(self, s_0, s_1):
        return integrate.quad(lambda x: 1 / self.curve_velocity(x), s_0, s_1, limit=500)[0]

    def calculate_segment_bounds(self):
        bounds = [0]
        for _ in range(self.n_cp):
            b = optimize.fsolve(lambda x: self.segment_time(bounds[-1], x) - (self.lap_time / self.n_cp), bounds[-1])[0]
            bounds.append(b)
        return bounds

    def get_bound(self, i):
        assert i >= 0
        assert i < self.n_cp
        return self.bounds[i]
