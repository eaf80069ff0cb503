"""Test helper: the reference agent's closed loop on the CPU (TEST-ONLY checker).

agent.run_step / run_mpc (agent.py:138-314) per vehicle, with
* sensing from the oracle (oracle.plant.agent_sense on oracle.splines.Centerline),
* the plant from the oracle (oracle.plant, pinned to the reference's models/ rollouts),
* the MPC from the host build of the solver source (libmpcracing_host.so, host_twin) -- the
  oracle's dense IPM would take minutes per solve.
Same conventions as mpcracing.closed_loop: yaw rate by finite differences (agent.py:240-249),
negative throttle applied as brake and fed back (agent.py:149, 289-306), shifted warm start.
"""
import math

import numpy as np

import host_twin as ht
from oracle import plant


def run(cl, state0, ticks, N=15, model="blend", start_control_at=2, dt=0.05, Ts=0.05, lookback=5.0,
        lookahead=45.0, runtime=(1000.0, 0.85, 50.0, 2.0, 5000.0), solver_cfg=None):
    state = np.array(state0, dtype=np.float64)
    B = state.shape[1]
    prev = [None] * B
    old_yaw = [None] * B
    cmd_thr, cmd_brake, cmd_steer = np.zeros(B), np.zeros(B), np.zeros(B)
    last_controls = None
    rt = np.asarray(runtime, dtype=np.float64)  # shared (5,) or per vehicle [5][B] (a GA population)
    rt = np.tile(rt.reshape(5, 1), (1, B)) if rt.size == 5 else rt.reshape(5, B).copy()
    cfg = solver_cfg if solver_cfg is not None else ht.config(N, "dyn", "fp64", False, Ts)
    recs = []
    for step in range(ticks):
        X, Y, yaw, vx, vy = (state[j].copy() for j in range(5))
        yawdot = np.full(B, math.nan)
        for i in range(B):
            if old_yaw[i] is not None:
                d = yaw[i] - old_yaw[i]
                if d > 3:
                    d = yaw[i] - (old_yaw[i] + np.pi * 2)
                elif d < -3:
                    d = yaw[i] - (old_yaw[i] - np.pi * 2)
                yawdot[i] = d / dt
        sense = [plant.agent_sense(cl, float(X[i]), float(Y[i]), prev[i], lookback, lookahead) for i in range(B)]
        prog = np.array([r[0] for r in sense])
        err = np.array([r[1] for r in sense])
        rec = dict(step=step, X=X, Y=Y, yaw=yaw, vx=vx, vy=vy, yawdot=yawdot, progress=prog, error=err)
        if step >= start_control_at:
            thr0 = np.where(cmd_brake == 0, cmd_thr, -cmd_brake)
            batch = dict(state0=np.stack([X, Y, yaw, vx, vy, yawdot, thr0, cmd_steer]), s0=prog,
                         cx=np.array([r[2] for r in sense]).T, cy=np.array([r[3] for r in sense]).T,
                         max_error=np.array([r[4] for r in sense]),
                         runtime=rt,
                         u_init=None if last_controls is None else
                         np.concatenate([last_controls[:, 1:], last_controls[:, -1:]], axis=1))
            out = ht.solve(cfg, batch)
            last_controls = out["U"].copy()
            throttle, steer = out["U"][0, 0].copy(), out["U"][1, 0].copy()
            rec.update(status=out["status"].copy(), iters=out["iters"].copy(), U=out["U"].copy())
        else:
            throttle, steer = np.full(B, 0.5), np.zeros(B)
        cmd_brake = np.where(throttle < 0, -throttle, 0.0)
        cmd_thr = np.where(throttle < 0, 0.0, throttle)
        cmd_steer = steer.copy()
        rec.update(cmd_throttle=cmd_thr.copy(), cmd_brake=cmd_brake.copy(), cmd_steer=cmd_steer.copy())
        state = np.array([plant.STEP[model](list(state[:, i]), float(cmd_thr[i] - cmd_brake[i]), float(cmd_steer[i]),
                                            dt) for i in range(B)]).T
        old_yaw = list(yaw)
        prev = list(prog)
        recs.append(rec)
    return recs, state
