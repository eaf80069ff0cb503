"""Batched closed loop on the GPU: the reference agent's control tick for B vehicles at once.

The reference drives one car in CARLA; each tick (``agent.run_step``, agent.py:207-314) it
senses (projection onto the centerline with the previous progress as bounds, signed error,
agent.py:237-274), and from step ``start_control_at`` = 50 on solves the MPC (``run_mpc``,
agent.py:138-205: N = 15, Ts = 0.05, quartic fit over [progress - 5, progress + 40], max_error =
lookup_error(progress, 45) - car_width / 2, warm start = the previous controls) and applies the
first control; before that it applies (0.5, 0.0).  SURVEY §8(f) rank 1: the same loop with a
``models/`` plant in place of the simulator (the reference's own stand-in, script/verify_*.py).

Here every tick is four device steps on one stream, with no host synchronisation:

1. ``mr_agent_sense``  (csrc/mr_agent.h)  progress, error, cx, cy, max_error for all vehicles;
2. input glue (torch ops on the device): state0 rows, shifted warm start (MPC.py:120-121);
3. ``mr_solve_batch``  (csrc/mr_wave.h)   the B MPC solves, one wavefront each;
4. ``mr_plant_step``   (csrc/mr_plant.h)  one plant step per vehicle with the applied command.

Measurement model: the plant state is the simulator truth; the agent's own derivations are kept
-- yaw rate by finite differences of the (wrapped) yaw over the tick (agent.py:240-249), the
commanded throttle fed back as ``cmd_throttle`` / ``cmd_brake`` (agent.py:289-306).  The plant's
body-frame velocities stand for the agent's rotation of the simulator's world velocity
(agent.py:252-253).  No CPU fallback: the constructor raises without a GPU.
"""
import math

import numpy as np
import torch

from .batch import BatchSolver
from .geometry import DeviceTrack, _ptr
from .track import CAR_WIDTH

PLANT = {"kin": 0, "dyn": 1, "blend": 2}
LOG_KEYS = ("X", "Y", "yaw", "vx", "vy", "yawdot", "progress", "error", "cmd_throttle", "cmd_steer", "cmd_brake",
            "status", "iters")


class ClosedLoop:
    def __init__(self, track="shanghai_intl_circuit", B=1, N=15, plant="blend", mpc_model="dyn",
                 precision="fp64", Ts=0.05, dt=0.05, start_control_at=50, lookback=5.0, lookahead=45.0,
                 runtime=(1000.0, 0.85, 50.0, 2.0, 5000.0), device=0, **solver_kw):
        if start_control_at < 1:
            raise ValueError("start_control_at >= 1: the MPC's yaw rate is a finite difference over one tick")
        self.track = track if isinstance(track, DeviceTrack) else DeviceTrack(track, device=device)
        self.lib = self.track.lib
        self.dev = self.track.device
        self.B, self.N = int(B), int(N)
        self.plant = PLANT[plant]
        self.dt, self.start_control_at = float(dt), int(start_control_at)
        self.lookback, self.lookahead = float(lookback), float(lookahead)
        # dispatch: longest-expected-first by the previous tick's iteration counts of the same vehicles
        # (mr_config.dispatch_order 2, LPT with a distribution-agnostic estimate); results do not depend on it
        solver_kw.setdefault("dispatch_order", 2)
        self.solver = BatchSolver(N, mpc_model, precision, False, Ts, max_batch=self.B, device=device, **solver_kw)
        f = dict(dtype=torch.float64, device=self.dev)
        # RuntimeControllerParameters (control/ControllerParameters.py:26-32) as (alpha_c, d_max, q_v_y, n,
        # beta_delta), shared (5 values) or per vehicle ([5][B], e.g. a GA population); the reference's
        # NLP reads the class attribute d_max (MPC.py:50), which callers reproduce by passing 0.85
        rt = torch.as_tensor(np.asarray(runtime, dtype=np.float64), **f)
        self.runtime = (rt.reshape(5, 1).expand(5, self.B) if rt.numel() == 5 else rt.reshape(5, self.B)).contiguous()
        self.sol = self.solver.alloc_outputs(self.B)
        self.progress = torch.empty(self.B, **f)
        self.error = torch.empty(self.B, **f)
        self.cx = torch.empty((5, self.B), **f)
        self.cy = torch.empty((5, self.B), **f)
        self.max_error = torch.empty(self.B, **f)
        self.cmd = torch.empty((2, self.B), **f)
        self.state_next = torch.empty((6, self.B), **f)

    # ------------------------------------------------------------------ state
    def reset(self, state):
        """state [6][B] = (x, y, yaw, v_x, v_y, yaw_dot) of every vehicle (host or device)."""
        f = dict(dtype=torch.float64, device=self.dev)
        self.state = torch.as_tensor(np.asarray(state, dtype=np.float64) if not isinstance(state, torch.Tensor)
                                     else state, **f).reshape(6, self.B).contiguous().clone()
        nan = torch.full((self.B,), math.nan, **f)
        self.prev_progress = nan.clone()   # agent.progress = None: first projection is global
        self.old_yaw = nan.clone()
        self.cmd_throttle = torch.zeros(self.B, **f)  # agent.py:53-55
        self.cmd_steer = torch.zeros(self.B, **f)
        self.cmd_brake = torch.zeros(self.B, **f)
        self.last_controls = None
        self.steps = 0

    @staticmethod
    def start_states(track, s0, v0=10.0, offset=0.0):
        """Vehicles on the centerline tangent at progress s0 [B] (lateral offset along the normal)."""
        s0 = np.atleast_1d(np.asarray(s0, dtype=np.float64))
        g, _ = track.eval(s0)
        fr = track.frame(s0)
        g = g.cpu().numpy()
        yaw, nx, ny = (fr[k].cpu().numpy() for k in ("yaw", "nx", "ny"))
        B = len(s0)
        return np.stack([g[0] + offset * nx, g[1] + offset * ny, yaw, np.full(B, float(v0)), np.zeros(B),
                         np.zeros(B)])

    # ------------------------------------------------------------------ one tick
    def tick(self, stream=None):
        """agent.run_step for every vehicle; returns this tick's record (device tensors, no sync).
        Everything -- the library launches and the torch glue between them -- is ordered on ``stream``
        (torch's current stream by default), so the caching allocator and the clones see the kernels'
        order."""
        st = stream if stream is not None else torch.cuda.current_stream(self.dev)
        with torch.cuda.stream(st):
            return self._tick(st)

    def _tick(self, st):
        sp = ctypes_stream(st)
        B, s = self.B, self.state
        X, Y, yaw, vx, vy = s[0], s[1], s[2], s[3], s[4]
        # yaw rate by finite differences of the wrapped yaw (agent.py:240-249)
        d = yaw - self.old_yaw
        d = torch.where(d > 3, yaw - (self.old_yaw + np.pi * 2), torch.where(d < -3, yaw - (self.old_yaw - np.pi * 2), d))
        yawdot = d / self.dt
        # sensing + MPC inputs (agent.py:156-168, 271-274)
        self._check(self.lib.mr_agent_sense(self.track.h, B, _ptr(X.contiguous()), _ptr(Y.contiguous()),
                                            _ptr(self.prev_progress), self.lookback, self.lookahead, CAR_WIDTH / 2,
                                            _ptr(self.progress), _ptr(self.error), _ptr(self.cx), _ptr(self.cy),
                                            _ptr(self.max_error), sp))
        controlled = self.steps >= self.start_control_at
        if controlled:
            thr0 = torch.where(self.cmd_brake == 0, self.cmd_throttle, -self.cmd_brake)   # agent.py:149
            state0 = torch.stack([X, Y, yaw, vx, vy, yawdot, thr0, self.cmd_steer]).contiguous()
            u_init = None
            if self.last_controls is not None:  # shifted warm start (MPC.py:120-121)
                lc = self.last_controls
                u_init = torch.cat([lc[:, 1:], lc[:, -1:]], dim=1).contiguous()
            dev_in = dict(state0=state0, s0=self.progress, cx=self.cx, cy=self.cy, max_error=self.max_error,
                          runtime=self.runtime, u_init=u_init,
                          # the previous tick's iters, read by the order kernel before this solve writes them
                          order_hint=self.sol["iters"] if self.last_controls is not None else None)
            self.solver.launch(dev_in, self.sol, stream=st)
            U = self.sol["U"]
            self.last_controls = U.clone()
            throttle, steer = U[0, 0], U[1, 0]
        else:
            throttle = torch.full((B,), 0.5, dtype=torch.float64, device=self.dev)
            steer = torch.zeros(B, dtype=torch.float64, device=self.dev)
        # carla.VehicleControl: negative throttle is brake (agent.py:289-306)
        self.cmd_brake = torch.where(throttle < 0, -throttle, torch.zeros_like(throttle))
        self.cmd_throttle = torch.where(throttle < 0, torch.zeros_like(throttle), throttle)
        self.cmd_steer = steer.clone()
        rec = dict(step=self.steps, X=X.clone(), Y=Y.clone(), yaw=yaw.clone(), vx=vx.clone(), vy=vy.clone(),
                   yawdot=yawdot, progress=self.progress.clone(), error=self.error.clone(),
                   cmd_throttle=self.cmd_throttle, cmd_steer=self.cmd_steer, cmd_brake=self.cmd_brake,
                   controlled=controlled,
                   status=self.sol["status"].clone() if controlled else None,
                   iters=self.sol["iters"].clone() if controlled else None,
                   predicted_states=self.sol["X"].clone() if controlled else None,
                   controls=self.last_controls if controlled else None,
                   s_hat=self.sol["S"].clone() if controlled else None,
                   e_hat_c=self.sol["eC"].clone() if controlled else None,
                   e_hat_l=self.sol["eL"].clone() if controlled else None)
        # plant step with the simulator's command throttle - brake (models/Model.py:83-88)
        self.cmd[0] = self.cmd_throttle - self.cmd_brake
        self.cmd[1] = self.cmd_steer
        self._check(self.lib.mr_plant_step(self.plant, B, _ptr(self.state), _ptr(self.cmd), self.dt,
                                           _ptr(self.state_next), sp))
        self.state, self.state_next = self.state_next, self.state
        self.old_yaw = yaw.clone()
        self.prev_progress = self.progress.clone()
        self.steps += 1
        return rec

    def run(self, ticks, stream=None):
        """``ticks`` agent steps; returns the list of per-tick records (device tensors)."""
        return [self.tick(stream) for _ in range(int(ticks))]

    def _check(self, rc):
        if rc != 0:
            raise RuntimeError(f"libmpcracing error {rc}: {self.lib.mr_last_error().decode()}")


def ctypes_stream(st):
    import ctypes
    return ctypes.c_void_p(st.cuda_stream)
