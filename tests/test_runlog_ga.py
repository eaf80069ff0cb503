"""Host-side pieces of the closed loop: the reference Logger format and the GA scoring."""
import csv
import os
import pickle
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "mpc-racing_amd"))
from mpcracing import ga, runlog  # noqa: E402


def _records(T=4, B=2, N=5, start=2):
    rng = np.random.default_rng(0)
    recs = []
    for k in range(T):
        ctl = k >= start
        r = {key: rng.normal(size=B) for key in ("X", "Y", "yaw", "vx", "vy", "progress", "error", "cmd_throttle",
                                                 "cmd_steer", "cmd_brake")}
        r["yawdot"] = np.full(B, np.nan) if k == 0 else rng.normal(size=B)
        r.update(step=k, controlled=ctl)
        if ctl:
            r.update(predicted_states=rng.normal(size=(6, N + 1, B)), controls=rng.normal(size=(2, N, B)),
                     s_hat=rng.normal(size=(N + 1, B)), e_hat_c=rng.normal(size=(N, B)),
                     e_hat_l=rng.normal(size=(N, B)))
        else:
            r.update(predicted_states=None, controls=None, s_hat=None, e_hat_c=None, e_hat_l=None)
        recs.append(r)
    return recs


def test_logger_format(tmp_path):
    recs = _records()
    runlog.write_run(recs, str(tmp_path), vehicle=1, dt=0.05)
    rows = list(csv.reader(open(tmp_path / "steps.csv")))
    assert rows[0] == runlog.MEMBER_NAMES  # Logger.py:5-8
    assert len(rows) == len(recs) + 1
    assert rows[1][runlog.MEMBER_NAMES.index("yawdot")] == "None"
    assert float(rows[2][1]) == recs[1]["X"][1]
    assert rows[3][runlog.MEMBER_NAMES.index("next_left_lane_point_x")] == "None"
    d0 = pickle.load(open(tmp_path / "mpc" / "0", "rb"))  # written by this test
    assert set(d0) == {"controlled", "step", "predicted_states", "controls", "mean_ts", "time", "s_hat", "e_hat_c",
                       "e_hat_l"}
    assert d0["controlled"] is False and d0["predicted_states"] is None
    d3 = pickle.load(open(tmp_path / "mpc" / "3", "rb"))
    assert d3["controlled"] is True and len(d3["predicted_states"]) == 6 and len(d3["controls"]) == 5
    assert d3["predicted_states"][2].x == recs[3]["predicted_states"][0, 2, 1]
    assert d3["controls"][0] == (recs[3]["controls"][0, 0, 1], recs[3]["controls"][1, 0, 1])
    # mean_ts as agent.py:285 from 0.3
    m = 0.3
    for k in range(4):
        m = m + ((0.05 - m) / (k + 1))
    assert abs(d3["mean_ts"] - m) < 1e-15


def test_ga_reward_and_average():
    t = np.array([[1.0, 2.0], [1.5, 2.5]])
    r, avg = ga.rewards(t, [1.2, 2.2])
    a0 = 0.3 * 1.0 + 0.7 * 1.2
    assert abs(avg[0] - (0.3 * 1.5 + 0.7 * a0)) < 1e-15
    assert abs(r[0] - (np.exp(-4 * (1.0 - 1.2)) + np.exp(-4 * (2.0 - 2.2)))) < 1e-12


def test_segment_times_interpolation():
    class R:
        def __init__(self, p):
            import torch
            self.d = {"progress": torch.tensor(p, dtype=torch.float64)}

        def __getitem__(self, k):
            return self.d[k]
    recs = [R([10.0, 990.0]), R([11.0, 999.0]), R([12.0, 1.0]), R([13.0, 3.0])]
    t = ga.segment_times(recs, np.array([10.0, 990.0]), np.array([12.5, 2.0]), 1000.0, 0.05)
    assert abs(t[0] - 0.05 * 2.5) < 1e-12
    assert abs(t[1] - 0.05 * 2.5) < 1e-12
