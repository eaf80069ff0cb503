"""Edge cases of the C ABI: configuration limits (no GPU needed: mr_create validates before any
HIP call), empty batches, the horizon extremes of the lane-per-stage mapping (N = 1, 2 and the
maximum 63, where every lane of the wavefront owns a stage), ragged batches."""
import ctypes
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

from mpcracing import abi  # noqa: E402
from mpcracing import workload as wl  # noqa: E402


def _cfg(**kw):
    lib = abi.load_product()
    c = abi.MRConfig()
    assert lib.mr_config_default(ctypes.byref(c)) == 0
    for k, v in kw.items():
        setattr(c, k, v)
    return lib, c


@pytest.mark.parametrize("field,value", [("N", 0), ("N", 64), ("model", 7), ("precision", 5), ("max_batch", 0),
                                         ("Ts", 0.0)])
def test_create_rejects_bad_config(field, value):
    lib, c = _cfg(**{field: value})
    h = ctypes.c_void_p()
    assert lib.mr_create(ctypes.byref(h), ctypes.byref(c)) == -1  # MR_ERR_ARG, before any device call
    assert lib.mr_last_error() and not h.value


def test_track_entry_points_reject_bad_arguments():
    lib = abi.load_product()
    P = ctypes.POINTER(ctypes.c_double)
    x = np.arange(3, dtype=np.float64)
    t = np.zeros(16)
    nt, L = ctypes.c_int32(), ctypes.c_double()
    pp = lambda a: a.ctypes.data_as(P)  # noqa: E731
    assert lib.mr_spline_from_waypoints(pp(x), pp(x), 3, 0, pp(t), pp(t), pp(t), ctypes.byref(nt),
                                        ctypes.byref(L)) == -1  # fewer than 4 waypoints
    assert lib.mr_track_lane_table(None, None, 4, None, None, None, None) == -1
    h = ctypes.c_void_p()
    assert lib.mr_track_create(ctypes.byref(h), 0, pp(t), 16, pp(t), pp(t), 12, 1.0, None, None, 5) == -1  # rows, no table


def _slice(b, n):
    return {k: (v[..., :n].copy() if v is not None else None) for k, v in b.items()}


@pytest.mark.gpu
def test_empty_batch():
    pytest.importorskip("torch")
    from mpcracing.batch import BatchSolver
    s = BatchSolver(20, "kin", "fp64", max_batch=4)
    out = s.solve(_slice(wl.make_batch("C2", limit=1), 0))
    assert out["status"].numel() == 0


@pytest.mark.gpu
@pytest.mark.parametrize("N", [1, 2, 63])
def test_horizon_extremes_match_host_build(N):
    """Same solver source on the GPU and on the host at the smallest horizons and at N = 63."""
    pytest.importorskip("torch")
    import host_twin as ht
    from mpcracing.batch import BatchSolver
    b = wl.make_batch("C2", limit=3)  # ragged: 3 instances
    # the same options on both builds (acceptable_iter 15): at N = 63 the unscaled tests are out of reach,
    # and with acceptable_iter 0 whether a line search fails at the mu floor (acceptable exit) or the
    # solve runs to max_iter is decided by rounding, which the two builds do differently (FMA)
    s = BatchSolver(N, "kin", "fp64", max_batch=5, tol=1e-10, acceptable_iter=15)
    o = {k: v.cpu().numpy() for k, v in s.solve(b).items()}
    h = ht.solve(ht.config(N, "kin", "fp64", tol=1e-10, acceptable_iter=15), b, nthreads=4)
    assert (o["status"] == h["status"]).all(), (o["status"], h["status"])
    # at N = 63 the objective scaling is small enough that IPOPT's unscaled complementarity test fails at
    # the mu floor: the solves end "acceptable" (status 1) at the same point on both builds
    ok = o["status"] <= 1
    assert ok.all()
    dU = np.abs(o["U"] - h["U"])[:, :, ok]
    dU[0, -1, :] = 0.0  # last throttle: fixed by the barrier only
    assert dU.max() < 1e-6 and np.abs(o["S"] - h["S"])[:, ok].max() < 1e-6
