"""Track geometry on the host (spline construction + per-instance MPC inputs).

Mirrors ``splines/ParameterizedLine.py`` / ``splines/ParameterizedCenterline.py``
of the reference: the centerline is the scipy not-a-knot cubic B-spline of the
chord-length-parameterised waypoints (ParameterizedLine.from_waypoints
:162-178), closed with a midpoint at alpha = 0.9 when the loop is open
(ParameterizedCenterline.from_file :93-105); the lane tables keep the
reference's left/right file swap (:17-21).  Construction is a once-per-track
host step; per-instance queries used to build MPC inputs are vectorised numpy
here (the batched device versions are the prep kernels).
"""
import math
import os

import numpy as np
from scipy.interpolate import make_interp_spline

HERE = os.path.dirname(os.path.abspath(__file__))
TRACK_DIR = os.path.abspath(os.path.join(HERE, "..", "data", "tracks"))
TRACKS = ["shanghai_intl_circuit", "t1_triple", "t2_triple", "t3", "t4"]
CAR_WIDTH = 1.85  # VehicleParameters.car_width


def _euclidean(p1, p2):
    return math.sqrt((p1[0] - p2[0]) ** 2 + (p1[1] - p2[1]) ** 2)


def _midpoint(p1, p2, alpha=0.5):
    return (p2[0] - p1[0]) * alpha + p1[0], (p2[1] - p1[1]) * alpha + p1[1]


def spline_from_waypoints(xy):
    """ParameterizedLine.from_waypoints (:162-178): chord-length s accumulated with the reference's
    Python euclidean, scipy not-a-knot cubic interpolation.  Returns (spline_x, spline_y, length)."""
    ss = [0.0]
    cum = 0.0
    for i in range(len(xy) - 1):
        cum += _euclidean(xy[i], xy[i + 1])
        ss.append(cum)
    s = np.array(ss)
    xy = np.asarray(xy, dtype=np.float64)
    return make_interp_spline(s, xy[:, 0]), make_interp_spline(s, xy[:, 1]), ss[-1]


class Track:
    def __init__(self, name="shanghai_intl_circuit"):
        d = np.load(os.path.join(TRACK_DIR, f"{name}.npz"))
        self.name = name
        wps = [tuple(p) for p in d["waypoints"].tolist()]
        if _euclidean(wps[-1], wps[0]) > 0.1:
            wps.append(_midpoint(wps[-1], wps[0], alpha=0.9))
        ss = [0.0]
        cum = 0.0
        for i in range(len(wps) - 1):
            cum += _euclidean(wps[i], wps[i + 1])
            ss.append(cum)
        s = np.array(ss)
        self.spline_x = make_interp_spline(s, np.array([p[0] for p in wps]))
        self.spline_y = make_interp_spline(s, np.array([p[1] for p in wps]))
        self.length = ss[-1]
        self.dx = self.spline_x.derivative()
        self.dy = self.spline_y.derivative()
        self.ddx = self.dx.derivative()
        self.ddy = self.dy.derivative()
        self.err_ss = d["err_ss"]
        self.err_left = d["err_left"]
        self.err_right = d["err_right"]
        self._err = {float(a): (float(l), float(r)) for a, l, r in zip(self.err_ss, self.err_left, self.err_right)}
        # lane boundaries, swapped exactly as ParameterizedCenterline.py:17-21
        self.right_lane_xy = np.stack([d["left_csv_x"], d["left_csv_y"]], 1)
        self.left_lane_xy = np.stack([d["right_csv_x"], d["right_csv_y"]], 1)

    def lane_spline(self, side):
        """ParameterizedLane.from_file (ParameterizedLane.py:22-25) for self.right_lane / self.left_lane
        (the file swap kept): (spline_x, spline_y, length) of that lane boundary."""
        xy = self.right_lane_xy if side == "right" else self.left_lane_xy
        return spline_from_waypoints([tuple(p) for p in xy.tolist()])

    @property
    def knots(self):
        return np.asarray(self.spline_x.t)

    def _m(self, s):
        return np.mod(s, self.length)

    def Gx(self, s):
        return self.spline_x(self._m(s))

    def Gy(self, s):
        return self.spline_y(self._m(s))

    def dGx(self, s):
        return self.dx(self._m(s))

    def dGy(self, s):
        return self.dy(self._m(s))

    def ddGx(self, s):
        return self.ddx(self._m(s))

    def ddGy(self, s):
        return self.ddy(self._m(s))

    def xy_coeffs(self, s, lookahead, deg=4):
        """x_as_coeffs / y_as_coeffs (ParameterizedLine.py:43-64): 50 samples, np.polyfit in global s."""
        ss = np.linspace(0, lookahead, 50) + s
        return np.polyfit(ss, self.Gx(ss), deg=deg), np.polyfit(ss, self.Gy(ss), deg=deg)

    def unit_tangent(self, s):
        d = np.array([self.dGx(s), self.dGy(s)])
        return d / np.linalg.norm(d, axis=0)

    def unit_tangent_yaw(self, s):
        ut = self.unit_tangent(s)
        return np.arctan2(ut[1], ut[0])

    def unit_principal_normal(self, s):
        ux, uy = self.unit_tangent(s)
        return uy, -ux

    def lookup_error(self, s, lookahead):
        """ParameterizedCenterline.lookup_error (:61-80): Python round-half-even keys, window min."""
        def r2(x):
            return round(x * 2) / 2
        s_round = r2(s)
        la = r2(lookahead)
        left_min = right_min = 10000
        for q in np.arange(s_round, s + la, 0.5):
            left, right = self._err[r2(q % self.length)]
            left_min = left if left < left_min else left_min
            right_min = right if right < right_min else right_min
        return min(right_min, left_min)
