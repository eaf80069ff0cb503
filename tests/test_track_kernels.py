"""Centerline kernels (csrc/mr_track.h, host build) against the reference's golden vectors.

The golden vectors were produced by the reference's own splines/ package
(tests/golden/make_golden.py).  Integer outputs and everything computed by plain IEEE
arithmetic in the reference's order are checked bit for bit: spline values (G2), lane-table
window minima (G4), the bounded-Brent projection (G5), curvature / mean curvature / error sign
(G6).  Tolerances where the reference calls a library routine that is not reproduced
operation for operation: unit-tangent yaw and principal normal (numpy's norm / libm atan2)
to 4e-16, and the deg-4 fit (numpy's LAPACK SVD) on its VALUES over the fit window to 5e-7 m
(the fit itself misses the spline by ~7e-3 m).
"""
import json
import os

import numpy as np
import pytest

from track_twin import HostTrack

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "golden.npz"))
TRACKS = json.load(open(os.path.join(HERE, "golden", "golden.json")))["tracks"]


@pytest.fixture(scope="module", params=TRACKS)
def trk(request):
    return request.param, HostTrack(G, request.param)


def test_spline_eval_bitexact(trk):
    track, ht = trk
    p = track + "/"
    out, span = ht.eval(G[p + "g2_s"])
    assert np.array_equal(out.T, G[p + "g2_vals"])
    # knot span = scipy interval search (t[l] <= s mod L < t[l+1], clamped to [3, n-1])
    t = G[p + "t"]
    m = np.mod(G[p + "g2_s"], float(G[p + "L"]))
    ref = np.clip(np.searchsorted(t, m, side="right") - 1, 3, len(t) - 5)
    assert np.array_equal(span, ref)


def test_lookup_error_bitexact(trk):
    track, ht = trk
    p = track + "/"
    err, lo, hi, arg = ht.lookup(G[p + "g4_s"], G[p + "g4_la"])
    assert np.array_equal(err, G[p + "g4_err"])
    assert (lo >= 0).all() and (hi >= 0).all() and (arg >= 0).all()
    # the minimum is attained at the reported row, on the left or the right lane table
    assert np.array_equal(err, np.where(ht.el[arg] < ht.er[arg], ht.el[arg], ht.er[arg])) or \
        ((err == ht.el[arg]) | (err == ht.er[arg])).all()


def test_projection_bitexact(trk):
    track, ht = trk
    p = track + "/"
    xy = G[p + "g5_xy"]
    s, d, nfev = ht.projection(xy[:, 0], xy[:, 1], G[p + "g5_lo"], G[p + "g5_hi"])
    assert np.array_equal(np.stack([s, d], 1), G[p + "g5_res"])
    assert (nfev > 3).all() and (nfev < 500).all()


def test_frame_curvature_sign(trk):
    track, ht = trk
    p = track + "/"
    yaw, kap, nx, ny, mk = ht.frame(G[p + "g6_s"], 45.0)
    assert np.array_equal(kap, G[p + "g6_kappa"]) and np.array_equal(mk, G[p + "g6_meank"])
    assert np.abs(yaw - G[p + "g6_yaw"]).max() <= 4.5e-16
    assert np.abs(np.stack([nx, ny], 1) - G[p + "g6_upn"]).max() <= 4.5e-16
    sxy = G[p + "g6_sign_xy"]
    assert np.array_equal(ht.error_sign(sxy[:, 0], sxy[:, 1], G[p + "g6_sign_s"]), G[p + "g6_sign"])


def test_polyfit_values(trk):
    track, ht = trk
    p = track + "/"
    cx, cy = ht.polyfit(G[p + "g3_s"], G[p + "g3_la"])
    for i, (a, b) in enumerate(zip(G[p + "g3_s"], G[p + "g3_la"])):
        ss = np.linspace(0, b, 50) + a
        assert np.abs(np.polyval(cx[:, i], ss) - np.polyval(G[p + "g3_cx"][i], ss)).max() < 5e-7
        assert np.abs(np.polyval(cy[:, i], ss) - np.polyval(G[p + "g3_cy"][i], ss)).max() < 5e-7


def test_lookup_error_keyerror_is_nan():
    """A window key past the last table row is the reference's KeyError (pandas .loc): NaN, rows -1."""
    ht = HostTrack(G, "shanghai_intl_circuit", rows=100)  # a table truncated to s < 50 m
    err, lo, hi, arg = ht.lookup([60.0, 10.0], [5.0, 5.0])
    assert np.isnan(err[0]) and lo[0] == -1 and arg[0] == -1
    assert err[1] == min(ht.el[20:30].min(), ht.er[20:30].min())


@pytest.mark.parametrize("deg,tol", [(0, 1e-9), (1, 1e-9), (2, 1e-9), (3, 1e-8), (4, 5e-7), (5, 1e-4)])
def test_polyfit_any_degree(trk, deg, tol):
    """x_as_coeffs / y_as_coeffs with the reference's deg argument (ParameterizedLine.py:43-64,
    mr_track_polyfit_deg) against numpy.polyfit on the same spline samples, on the fitted VALUES over the
    window.  The tolerance grows with the degree because both sides evaluate monomials in global s
    (s up to 1 900 m here): from deg 6 on numpy itself warns that the fit is poorly conditioned and the
    two differ by centimetres and more -- the reference's "please don't make this too high"."""
    track, ht = trk
    p = track + "/"
    s, la = G[p + "g3_s"], G[p + "g3_la"]
    cx, cy = ht.polyfit_deg(s, la, deg)
    assert cx.shape == (deg + 1, len(s))
    for i in range(len(s)):
        ss = np.linspace(0, la[i], 50) + s[i]
        g = ht.eval(ss)[0]
        for c, y in ((cx, g[0]), (cy, g[1])):
            ref = np.polyfit(ss, y, deg)
            assert np.abs(np.polyval(c[:, i], ss) - np.polyval(ref, ss)).max() < tol
    if deg == 4:  # the general path reproduces the agent's quartic bit for bit
        qx, qy = ht.polyfit(s, la)
        assert np.array_equal(qx, cx) and np.array_equal(qy, cy)
