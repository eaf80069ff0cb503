"""Batched centerline geometry on the GPU (the agent's per-tick MPC inputs).

``DeviceTrack`` uploads a track's spline tables once (``mr_track_create``) and
answers batches of the queries the reference agent runs before every solve
(agent.py:156-168, 271-274) through the gfx950 kernels of ``csrc/mr_track.h``:

* ``eval``        -- Gx, Gy, dGx, dGy, ddGx, ddGy       splines/ParameterizedLine.py:19-41
* ``polyfit``     -- x_as_coeffs / y_as_coeffs (deg 4)   ParameterizedLine.py:43-64
* ``lookup_error``-- lane-table window min             splines/ParameterizedCenterline.py:61-80
* ``projection``  -- projection_local (bounded Brent)   ParameterizedLine.py:80-97
* ``frame``       -- unit_tangent yaw, curvature, mean_curvature, unit_principal_normal  :107-149
* ``error_sign``  -- ParameterizedCenterline.py:82-91
* ``prep``        -- projection -> coeffs -> max_error, fused (feeds ``BatchSolver`` inputs)
* ``lane_errors`` / ``lane_width_table`` -- the offline lane-width table build
  (script/make_lane_width_lookup_table.py, ParameterizedCenterline.get_errors :41-58)

The spline itself is constructed once on the host exactly as the reference does
(scipy ``make_interp_spline``, ``mpcracing.track.Track``).  There is no CPU
fallback: without a GPU the constructor raises.
"""
import ctypes

import numpy as np
import torch

from . import abi
from .track import Track, CAR_WIDTH


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def native_spline(lib, x, y, close_loop):
    """ParameterizedLine.from_waypoints (:162-178) in the library (mr_spline_from_waypoints, host code,
    no scipy): returns knots t, coefficients cx, cy and the length L."""
    n = len(x)
    x = np.ascontiguousarray(x, dtype=np.float64)
    y = np.ascontiguousarray(y, dtype=np.float64)
    t, cx, cy = np.zeros(n + 5), np.zeros(n + 1), np.zeros(n + 1)
    nt, L = ctypes.c_int32(), ctypes.c_double()
    P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))  # noqa: E731
    rc = lib.mr_spline_from_waypoints(P(x), P(y), n, int(close_loop), P(t), P(cx), P(cy), ctypes.byref(nt),
                                      ctypes.byref(L))
    if rc != 0:
        raise RuntimeError(f"mr_spline_from_waypoints: {lib.mr_last_error().decode()}")
    m = nt.value
    return t[:m].copy(), cx[:m - 4].copy(), cy[:m - 4].copy(), L.value


class DeviceTrack:
    def __init__(self, track="shanghai_intl_circuit", device=0, tables=None):
        """``track``: a track name or ``mpcracing.track.Track``; or ``tables`` = (t, cx, cy, L,
        err_left, err_right) for a spline built elsewhere (the drop-in ParameterizedLine's
        ``from_waypoints``; lane tables may be None)."""
        if not torch.cuda.is_available():
            raise RuntimeError("mpcracing.DeviceTrack needs a ROCm GPU")
        self.lib = abi.load_product()
        self.device = torch.device("cuda", int(device))
        if tables is None:
            tr = track if isinstance(track, Track) else Track(track)
            self.track = tr
            if not np.array_equal(tr.spline_y.t, tr.spline_x.t) or tr.spline_x.k != 3:
                raise ValueError("centerline splines must share cubic knots")
            ss = np.asarray(tr.err_ss, dtype=np.float64)
            if not np.array_equal(ss, 0.5 * np.arange(len(ss))):
                raise ValueError("lane table rows must be s = 0.5 * row (make_lane_width_lookup_table.py)")
            tables = (tr.spline_x.t, tr.spline_x.c, tr.spline_y.c, tr.length, tr.err_left, tr.err_right)
        else:
            self.track = None
        t, cx, cy, L, el, er = tables
        t = np.ascontiguousarray(t, dtype=np.float64)
        cx = np.ascontiguousarray(cx, dtype=np.float64)
        cy = np.ascontiguousarray(cy, dtype=np.float64)
        P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double)) if a is not None else None  # noqa: E731
        el = None if el is None else np.ascontiguousarray(el, dtype=np.float64)
        er = None if er is None else np.ascontiguousarray(er, dtype=np.float64)
        nr = 0 if el is None else len(el)
        h = ctypes.c_void_p()
        self._check(self.lib.mr_track_create(ctypes.byref(h), int(device), P(t), len(t), P(cx), P(cy), len(cx),
                                             float(L), P(el), P(er), nr))
        self.h = h
        self.length = float(L)

    def _check(self, rc):
        if rc != 0:
            raise RuntimeError(f"libmpcracing error {rc}: {self.lib.mr_last_error().decode()}")

    def __del__(self):
        self.close_lanes()
        h = getattr(self, "h", None)
        if h is not None and h.value:
            self.lib.mr_track_destroy(h)
            self.h = None

    def _d(self, a):
        return torch.as_tensor(np.asarray(a, dtype=np.float64) if not isinstance(a, torch.Tensor) else a,
                               dtype=torch.float64, device=self.device).reshape(-1).contiguous()

    def _f(self, *shape):
        return torch.empty(shape, dtype=torch.float64, device=self.device)

    def _i(self, n):
        return torch.empty(n, dtype=torch.int32, device=self.device)

    def _stream(self, stream):
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        return ctypes.c_void_p(st.cuda_stream)

    def eval(self, s, stream=None):
        """[6][n] = (Gx, Gy, dGx, dGy, ddGx, ddGy)(s mod L) and the knot span [n]."""
        s = self._d(s)
        n = s.numel()
        out, span = self._f(6, n), self._i(n)
        self._check(self.lib.mr_track_eval(self.h, n, _ptr(s), _ptr(out), _ptr(span), self._stream(stream)))
        return out, span

    def frame(self, s, mc_lookahead=45.0, stream=None):
        s = self._d(s)
        n = s.numel()
        yaw, kap, nx, ny, mk = (self._f(n) for _ in range(5))
        self._check(self.lib.mr_track_frame(self.h, n, _ptr(s), _ptr(yaw), _ptr(kap), _ptr(nx), _ptr(ny),
                                            float(mc_lookahead), _ptr(mk), self._stream(stream)))
        return dict(yaw=yaw, curvature=kap, nx=nx, ny=ny, mean_curvature=mk)

    def error_sign(self, X, Y, s, stream=None):
        X, Y, s = self._d(X), self._d(Y), self._d(s)
        sg = self._i(s.numel())
        self._check(self.lib.mr_track_error_sign(self.h, s.numel(), _ptr(X), _ptr(Y), _ptr(s), _ptr(sg),
                                                 self._stream(stream)))
        return sg

    def polyfit(self, s, lookahead, stream=None, deg=4):
        """x_as_coeffs / y_as_coeffs: cx, cy [deg+1][n], highest order first, global s (0 <= deg <= 10)."""
        s = self._d(s)
        la = self._d(np.broadcast_to(np.asarray(lookahead, dtype=np.float64), (s.numel(),)).copy()
                     if not isinstance(lookahead, torch.Tensor) else lookahead)
        n = s.numel()
        cx, cy = self._f(deg + 1, n), self._f(deg + 1, n)
        if deg == 4:
            self._check(self.lib.mr_track_polyfit(self.h, n, _ptr(s), _ptr(la), _ptr(cx), _ptr(cy),
                                                  self._stream(stream)))
        else:
            self._check(self.lib.mr_track_polyfit_deg(self.h, n, _ptr(s), _ptr(la), int(deg), _ptr(cx), _ptr(cy),
                                                      self._stream(stream)))
        return cx, cy

    def lookup_error(self, s, lookahead, stream=None):
        s = self._d(s)
        n = s.numel()
        la = self._d(np.broadcast_to(np.asarray(lookahead, dtype=np.float64), (n,)).copy()
                     if not isinstance(lookahead, torch.Tensor) else lookahead)
        err, lo, hi, arg = self._f(n), self._i(n), self._i(n), self._i(n)
        self._check(self.lib.mr_track_lookup_error(self.h, n, _ptr(s), _ptr(la), _ptr(err), _ptr(lo), _ptr(hi),
                                                   _ptr(arg), self._stream(stream)))
        return err, lo, hi, arg

    def projection(self, X, Y, lo, hi, stream=None):
        X, Y, lo, hi = self._d(X), self._d(Y), self._d(lo), self._d(hi)
        n = X.numel()
        s, dist, nfev = self._f(n), self._f(n), self._i(n)
        self._check(self.lib.mr_track_projection(self.h, n, _ptr(X), _ptr(Y), _ptr(lo), _ptr(hi), _ptr(s),
                                                 _ptr(dist), _ptr(nfev), self._stream(stream)))
        return s, dist, nfev

    def prep(self, X, Y, lo, hi, lookback=5.0, lookahead=45.0, err_offset=CAR_WIDTH / 2, stream=None):
        """agent.py tick prep: s, dist, cx, cy [5][n], max_error (lookup_error - car_width/2)."""
        X, Y, lo, hi = self._d(X), self._d(Y), self._d(lo), self._d(hi)
        n = X.numel()
        s, dist, merr = self._f(n), self._f(n), self._f(n)
        cx, cy = self._f(5, n), self._f(5, n)
        self._check(self.lib.mr_track_prep(self.h, n, _ptr(X), _ptr(Y), _ptr(lo), _ptr(hi), float(lookback),
                                           float(lookahead), float(err_offset), _ptr(s), _ptr(dist), _ptr(cx),
                                           _ptr(cy), _ptr(merr), self._stream(stream)))
        return dict(s=s, dist=dist, cx=cx, cy=cy, max_error=merr)

    # ---- lane-width table build ----
    def _lane(self, side):
        lanes = self.__dict__.setdefault("_lanes", {})
        if side not in lanes:
            if side not in ("right", "left"):
                raise ValueError("side is 'right' or 'left'")
            if self.track is None:
                raise ValueError("lane tables need a named track (mpcracing.track.Track)")
            xy = self.track.right_lane_xy if side == "right" else self.track.left_lane_xy
            t, cx, cy, L = native_spline(self.lib, xy[:, 0], xy[:, 1], close_loop=False)
            P = lambda a: a.ctypes.data_as(ctypes.POINTER(ctypes.c_double))  # noqa: E731
            h = ctypes.c_void_p()
            self._check(self.lib.mr_track_create(ctypes.byref(h), self.device.index, P(t), len(t), P(cx), P(cy),
                                                 len(cx), float(L), None, None, 0))
            lanes[side] = h
        return lanes[side]

    def lane_errors(self, side, s, stream=None):
        """ParameterizedCenterline.get_errors(lane, s_i, 0) for every s_i (ParameterizedCenterline.py:41-58):
        distance from G(s_i) to the `side` lane boundary (self.right_lane / self.left_lane of the
        reference, file swap kept), global over the lane.  Returns (dist [n], lane progress [n])."""
        s = self._d(s)
        n = s.numel()
        dist, u = self._f(n), self._f(n)
        self._check(self.lib.mr_track_lane_table(self.h, self._lane(side), n, _ptr(s), _ptr(dist), _ptr(u),
                                                 self._stream(stream)))
        return dist, u

    def lane_width_table(self, step=0.5, stream=None):
        """script/make_lane_width_lookup_table.py:52-66: ss = arange(0, L, step), right / left errors.
        Returns numpy (ss, right, left) -- the columns of lanes/<track>_max_error.csv."""
        ss = np.arange(0, self.length, step=step)
        right, _ = self.lane_errors("right", ss, stream)
        left, _ = self.lane_errors("left", ss, stream)
        return ss, right.cpu().numpy(), left.cpu().numpy()

    def close_lanes(self):
        for h in self.__dict__.get("_lanes", {}).values():
            if h.value:
                self.lib.mr_track_destroy(h)
        self.__dict__["_lanes"] = {}
