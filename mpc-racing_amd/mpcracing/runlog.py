"""Run logs of the batched closed loop in the reference's Logger format (Logger.py:5-50).

``write_run(records, run_dir, vehicle)`` writes one vehicle's run as the reference agent would:

* ``<run_dir>/steps.csv`` -- header ``Logger.member_names``, one row per tick, each value as
  ``str()`` of the agent attribute (``None`` where the agent has none: the yaw rate of the first
  tick and the CARLA lane-boundary points, which a models/ plant does not produce);
* ``<run_dir>/mpc/<step>`` -- the per-tick pickle of ``Logger.pickle_mpc_res``: ``controlled,
  step, predicted_states`` (list of ``models.State.State``), ``controls`` (list of (throttle,
  steer)), ``mean_ts, time, s_hat, e_hat_c, e_hat_l``.

so replay tooling written against the reference's runs (script/replay_mpc.py,
script/test_model_error.py) reads batched results unchanged.  Host-side I/O only.
"""
import math
import os
import pickle

import numpy as np

MEMBER_NAMES = ['steps', 'X', 'Y', 'yaw', 'vx', 'vy', 'yawdot',
                'progress', 'error', 'cmd_throttle', 'cmd_steer', 'cmd_brake',
                'next_left_lane_point_x', 'next_left_lane_point_y', 'next_right_lane_point_x',
                'next_right_lane_point_y', 'last_ts', 'mpc_time']


def _host(v, i):
    if v is None:
        return None
    a = v.detach().cpu().numpy() if hasattr(v, "detach") else np.asarray(v)
    return a[..., i]


def _val(x):
    if x is None:
        return None
    x = float(x)
    return None if math.isnan(x) else x


def write_run(records, run_dir, vehicle=0, dt=0.05, mpc_times=None):
    """records: ``mpcracing.ClosedLoop.run`` output; one vehicle's run into ``run_dir``."""
    from models.State import State
    os.makedirs(os.path.join(run_dir, "mpc"), exist_ok=True)
    i = vehicle
    mean_ts = 0.3  # agent.py:71, updated as agent.py:285
    predicted, controls, s_hat, e_c, e_l = None, None, None, None, None
    with open(os.path.join(run_dir, "steps.csv"), "w") as f:
        f.write(",".join(MEMBER_NAMES) + "\n")
        for r in records:
            step = int(r["step"])
            mean_ts = mean_ts + ((dt - mean_ts) / (step + 1))
            mpc_time = 0 if mpc_times is None else mpc_times[step]
            row = dict(steps=step, X=_val(_host(r["X"], i)), Y=_val(_host(r["Y"], i)),
                       yaw=_val(_host(r["yaw"], i)), vx=_val(_host(r["vx"], i)), vy=_val(_host(r["vy"], i)),
                       yawdot=_val(_host(r["yawdot"], i)), progress=_val(_host(r["progress"], i)),
                       error=_val(_host(r["error"], i)), cmd_throttle=_val(_host(r["cmd_throttle"], i)),
                       cmd_steer=_val(_host(r["cmd_steer"], i)), cmd_brake=_val(_host(r["cmd_brake"], i)),
                       next_left_lane_point_x=None, next_left_lane_point_y=None, next_right_lane_point_x=None,
                       next_right_lane_point_y=None, last_ts=dt, mpc_time=mpc_time)
            f.write(",".join(str(row[k]) for k in MEMBER_NAMES) + "\n")
            if r["controlled"]:
                X = _host(r["predicted_states"], i)   # [6][N+1]
                U = _host(r["controls"], i)           # [2][N]
                predicted = [State(x=float(t[0]), y=float(t[1]), yaw=float(t[2]), v_x=float(t[3]), v_y=float(t[4]),
                                   yaw_dot=float(t[5])) for t in X.T]
                controls = [(float(a), float(b)) for a, b in U.T]
                s_hat = _host(r["s_hat"], i).copy()
                e_c = [float(v) for v in _host(r["e_hat_c"], i)]
                e_l = [float(v) for v in _host(r["e_hat_l"], i)]
            data = {"controlled": bool(r["controlled"]), "step": step, "predicted_states": predicted,
                    "controls": controls, "mean_ts": mean_ts, "time": mpc_time, "s_hat": s_hat,
                    "e_hat_c": e_c, "e_hat_l": e_l}
            with open(os.path.join(run_dir, "mpc", str(step)), "wb") as g:
                pickle.dump(data, g, protocol=pickle.HIGHEST_PROTOCOL)
