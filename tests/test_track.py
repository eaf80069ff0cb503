"""Host-side track construction of the product (mpcracing.track) against the reference's
own spline tables and queries (golden G1-G4)."""
import json
import os

import numpy as np
import pytest

from mpcracing.track import Track

HERE = os.path.dirname(os.path.abspath(__file__))
G = np.load(os.path.join(HERE, "golden", "golden.npz"))
TRACKS = json.load(open(os.path.join(HERE, "golden", "golden.json")))["tracks"]


@pytest.mark.parametrize("track", TRACKS)
def test_spline_table_identical(track):
    t = Track(track)
    p = track + "/"
    assert np.array_equal(t.spline_x.t, G[p + "t"])
    assert np.array_equal(t.spline_x.c, G[p + "cx"]) and np.array_equal(t.spline_y.c, G[p + "cy"])
    assert t.length == float(G[p + "L"])


@pytest.mark.parametrize("track", TRACKS)
def test_queries(track):
    t = Track(track)
    p = track + "/"
    s = G[p + "g2_s"]
    mine = np.stack([t.Gx(s), t.Gy(s), t.dGx(s), t.dGy(s), t.ddGx(s), t.ddGy(s)], 1)
    assert np.array_equal(mine, G[p + "g2_vals"])
    for a, b, rx, ry in zip(G[p + "g3_s"], G[p + "g3_la"], G[p + "g3_cx"], G[p + "g3_cy"]):
        cx, cy = t.xy_coeffs(a, b)
        assert np.array_equal(cx, rx) and np.array_equal(cy, ry)
    e = [t.lookup_error(a, b) for a, b in zip(G[p + "g4_s"], G[p + "g4_la"])]
    assert np.array_equal(e, G[p + "g4_err"])


def test_workload_shards_partition_the_batch():
    from mpcracing import workload as wl
    full = wl.make_batch("C2", rank=0, world=1, per_gpu=256)
    parts = [wl.make_batch("C2", rank=r, world=4, per_gpu=64) for r in range(4)]
    for k in ("state0", "s0", "cx", "cy", "max_error"):
        assert np.array_equal(np.concatenate([p[k] for p in parts], axis=-1), full[k])
