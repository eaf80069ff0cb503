"""GPU parity of the centerline kernels (libmpcracing.so, gfx950) against the reference's golden
vectors -- same bars as tests/test_track_kernels.py (host build): bit-exact spline values, knot
spans, lane-table minima and rows, Brent projections, curvature, mean curvature and error signs;
yaw / normal to 2e-15 (device libm atan2); quartic-fit values to 5e-7 m of numpy's polyfit."""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu

from mpcracing import workload as wl  # noqa: E402
from mpcracing.track import Track  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "golden.npz"))
TRACKS = json.load(open(os.path.join(HERE, "golden", "golden.json")))["tracks"]


def _np(t):
    return t.cpu().numpy()


@pytest.fixture(scope="module", params=TRACKS)
def dev(request):
    from mpcracing.geometry import DeviceTrack
    tr = Track(request.param)
    p = request.param + "/"
    # the host-built spline equals the reference's (G1) bit for bit, so the device tables do too
    assert np.array_equal(tr.spline_x.t, G[p + "t"]) and np.array_equal(tr.spline_x.c, G[p + "cx"])
    return request.param, DeviceTrack(tr)


def test_eval_span_lookup_projection_bitexact(dev):
    track, d = dev
    p = track + "/"
    out, span = d.eval(G[p + "g2_s"])
    assert np.array_equal(_np(out).T, G[p + "g2_vals"])
    t = G[p + "t"]
    m = np.mod(G[p + "g2_s"], float(G[p + "L"]))
    assert np.array_equal(_np(span), np.clip(np.searchsorted(t, m, side="right") - 1, 3, len(t) - 5))
    err, lo, hi, arg = d.lookup_error(G[p + "g4_s"], G[p + "g4_la"])
    assert np.array_equal(_np(err), G[p + "g4_err"])
    assert (_np(lo) >= 0).all() and (_np(arg) >= 0).all()
    xy = G[p + "g5_xy"]
    s, dist, nfev = d.projection(xy[:, 0], xy[:, 1], G[p + "g5_lo"], G[p + "g5_hi"])
    assert np.array_equal(np.stack([_np(s), _np(dist)], 1), G[p + "g5_res"])


def test_frame_sign_polyfit(dev):
    track, d = dev
    p = track + "/"
    f = d.frame(G[p + "g6_s"], 45.0)
    assert np.array_equal(_np(f["curvature"]), G[p + "g6_kappa"])
    assert np.array_equal(_np(f["mean_curvature"]), G[p + "g6_meank"])
    assert np.abs(_np(f["yaw"]) - G[p + "g6_yaw"]).max() <= 2e-15
    assert np.abs(np.stack([_np(f["nx"]), _np(f["ny"])], 1) - G[p + "g6_upn"]).max() <= 2e-15
    sxy = G[p + "g6_sign_xy"]
    assert np.array_equal(_np(d.error_sign(sxy[:, 0], sxy[:, 1], G[p + "g6_sign_s"])), G[p + "g6_sign"])
    cx, cy = d.polyfit(G[p + "g3_s"], torch.tensor(G[p + "g3_la"]))
    cx, cy = _np(cx), _np(cy)
    for i, (a, b) in enumerate(zip(G[p + "g3_s"], G[p + "g3_la"])):
        ss = np.linspace(0, b, 50) + a
        assert np.abs(np.polyval(cx[:, i], ss) - np.polyval(G[p + "g3_cx"][i], ss)).max() < 5e-7
        assert np.abs(np.polyval(cy[:, i], ss) - np.polyval(G[p + "g3_cy"][i], ss)).max() < 5e-7


def test_prep_feeds_the_solver():
    """agent.py tick on the device: projection -> quartic fit -> lane bound -> batched solve, compared with
    the same inputs prepared on the host (mpcracing.track, numpy/scipy) and solved on the device."""
    from mpcracing.batch import solver_for_config
    from mpcracing.geometry import DeviceTrack
    name = "C4"
    cfg = wl.CONFIGS[name]
    b = wl.make_batch(name, limit=256)
    tr = wl.track(cfg["track"])
    d = DeviceTrack(tr)
    X, Y, s0 = b["state0"][0], b["state0"][1], b["s0"]
    la = cfg["N"] * cfg["Ts"] * wl.V_MAX + 25.0
    pr = d.prep(X, Y, s0 - 2.0, s0 + 2.0, lookback=5.0, lookahead=la)
    s = _np(pr["s"])
    # host reference of the same chain on the device's progress
    for i in range(0, 256, 37):
        hx, hy = tr.xy_coeffs(s[i] - 5.0, la)
        ss = np.linspace(0, la, 50) + s[i] - 5.0
        assert np.abs(np.polyval(_np(pr["cx"])[:, i], ss) - np.polyval(hx, ss)).max() < 5e-7
        assert np.abs(np.polyval(_np(pr["cy"])[:, i], ss) - np.polyval(hy, ss)).max() < 5e-7
        assert _np(pr["max_error"])[i] == tr.lookup_error(s[i], la) - 1.85 / 2
    # solve from device-prepared inputs
    bb = dict(b)
    bb["s0"] = s
    bb["cx"], bb["cy"] = _np(pr["cx"]), _np(pr["cy"])
    bb["max_error"] = _np(pr["max_error"])
    sol = solver_for_config(name, 256)
    o = {k: v.cpu().numpy() for k, v in sol.solve(bb).items()}
    # IPOPT's outcomes at the reference's options: solved / acceptable, or stopped at an almost-feasible
    # point when the objective scaling makes the unscaled tests unreachable -- never
    # infeasible, max_iter a small minority
    st = np.bincount(o["status"], minlength=5)
    assert st[4] == 0 and st[2] <= 0.02 * 256, st


def test_lane_table_rows_golden():
    """Lane-table rows read by the reference's lookup_error (first, last, window arg-min; fixture from the
    reference's own loop, tests/golden/make_caller_golden.py) -- bit-exact on the device."""
    from mpcracing.geometry import DeviceTrack
    cg = json.load(open(os.path.join(HERE, "golden", "callers_golden.json")))
    for track, rows in cg["G4r"].items():
        d = DeviceTrack(Track(track))
        s = np.array([r["s"] for r in rows])
        la = torch.tensor([r["la"] for r in rows], dtype=torch.float64)
        err, lo, hi, arg = (_np(v) for v in d.lookup_error(s, la))
        assert np.array_equal(lo, [r["row_lo"] for r in rows]) and np.array_equal(hi, [r["row_hi"] for r in rows])
        assert np.array_equal(arg, [r["row_arg"] for r in rows])
        ok = np.array([r["err"] is not None for r in rows])
        assert np.array_equal(err[ok], [r["err"] for r in rows if r["err"] is not None])


def test_dropin_line_from_waypoints():
    """splines.ParameterizedLine.from_waypoints (library host code) -> device queries; the spline equals the
    reference's (G1 knots) and its values match the host scipy view of the same tables."""
    from splines.ParameterizedLane import ParameterizedLane
    from splines.ParameterizedCenterline import ParameterizedCenterline
    cl = ParameterizedCenterline("t4")
    p = "t4/"
    assert np.array_equal(cl.spline_x.t, G[p + "t"])
    s = np.linspace(-10, cl.length + 10, 97)
    h = cl.host_track
    np.testing.assert_allclose(cl.Gx(s), h.Gx(s), rtol=0, atol=1e-12)
    np.testing.assert_allclose(cl.dGy(s), h.dGy(s), rtol=0, atol=1e-12)
    lane = cl.right_lane
    assert isinstance(lane, ParameterizedLane) and lane.length > 0
    s0 = 100.0
    ps, dist = lane.projection(cl.Gx(s0), cl.Gy(s0), bounds=None)
    assert lane.last_progress == ps and dist > 0
    assert cl.lookup_error(s0, 45.0) == wl.track("t4").lookup_error(s0, 45.0)


def test_polyfit_any_degree_matches_host_build(dev):
    """mr_track_polyfit_deg (the reference's deg argument, ParameterizedLine.py:43-64) on the device is
    bit-exact against the host build of the same source for every supported degree (0..10; the CPU suite
    checks those against numpy.polyfit), deg 4 equals mr_track_polyfit, and deg 11 is an argument error."""
    from track_twin import HostTrack
    track, d = dev
    p = track + "/"
    ht = HostTrack(G, track)
    s, la = G[p + "g3_s"], G[p + "g3_la"]
    for deg in range(0, 11):
        cx, cy = d.polyfit(s, torch.tensor(la), deg=deg)
        hx, hy = ht.polyfit_deg(s, la, deg)
        assert np.array_equal(_np(cx), hx) and np.array_equal(_np(cy), hy), deg
    q4 = d.polyfit(s, torch.tensor(la))
    assert np.array_equal(_np(q4[0]), ht.polyfit_deg(s, la, 4)[0])
    with pytest.raises(RuntimeError):
        d.polyfit(s, torch.tensor(la), deg=11)
