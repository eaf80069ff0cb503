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
    """The n_shards strided shards of a config are disjoint and union to its global batch (C4 at 1 024 per
    shard: 64 shards of 8 segments; the full batch = all 512 segments in lap order)."""
    from mpcracing import workload as wl
    full = wl.make_batch("C4", rank=0, world=1, per_gpu=65536, limit=None)
    M = wl.CONFIGS["C4"]["M"]
    n = 8
    for r in range(n):
        part = wl.make_batch("C4", rank=r, world=n, per_gpu=8192)
        segs, K, n_shards = wl.shard_segments("C4", r, n, 8192)
        assert K == 512 and n_shards == 8 and segs == list(range(r, 512, 8))
        cols = np.concatenate([np.arange(k * M, (k + 1) * M) for k in segs])
        for k in ("state0", "s0", "cx", "cy", "max_error"):
            assert np.array_equal(part[k], full[k][..., cols])
