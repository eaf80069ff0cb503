"""The drop-in ``control.MPC.MPC`` (CPU: the GPU solver replaced by a recording stand-in).

Checks the host logic around the solve, not the solve itself (tests/test_gpu.py::test_dropin_mpc_class
runs it on the GPU): the configuration the class hands to the solver -- the reference's IPOPT options
(control/MPC.py:152-161: tol 1e-4, acceptable_tol 1e-2, IPOPT's acceptable_iter 15, max_iter
FixedControllerParameters.max_iter = 500) and the reference's constants -- the warm-start initial guess
(MPC.py:120-121), and the result handling of the reference's try / except (MPC.py:164-181): ``sol`` and
``dual`` None unless IPOPT's status is solved / acceptable, ``ret`` always the last iterate."""
import math

import numpy as np
import pytest
import torch

from control import MPC as mpc_mod
from control.ControllerParameters import FixedControllerParameters, RuntimeControllerParameters
from models.State import State
from mpcracing import batch as batch_mod


class _FakeSolver:
    instances = []

    def __init__(self, N, model, precision, lane, Ts, max_batch=1, device=0, tyres=None, **kw):
        self.args = dict(N=N, model=model, precision=precision, lane=lane, Ts=Ts, max_batch=max_batch, **kw)
        self.status = 0
        self.batches = []
        _FakeSolver.instances.append(self)

    def solve(self, b, duals=False):
        self.batches.append(b)
        N = self.args["N"]
        out = dict(X=np.ones((6, N + 1, 1)), U=np.zeros((2, N, 1)), S=np.arange(N + 1.0)[:, None],
                   eC=np.zeros((N, 1)), eL=np.zeros((N, 1)), status=np.array([self.status], np.int32),
                   iters=np.array([7], np.int32), obj=np.array([1.5]), kkt=np.array([1e-9]),
                   lam_g=np.arange(13 * N + 9, dtype=np.float64)[:, None])
        return {k: torch.from_numpy(v) for k, v in out.items()}


@pytest.fixture
def fake(monkeypatch):
    _FakeSolver.instances.clear()
    monkeypatch.setattr(batch_mod, "BatchSolver", _FakeSolver)
    monkeypatch.setattr(mpc_mod, "_solvers", {})
    return _FakeSolver


def _args(throttle=0.19, steer=0.63):
    st = State(x=171, y=91.8, yaw=-0.219, v_x=20, v_y=0.48, yaw_dot=-0.059, throttle=throttle, steer=steer)
    return (st, 69.6, [0.0, 1.0, 0.0, 0.0, 0.0], [0.0, 0.0, 0.0, 0.0, 0.0], 3.0, RuntimeControllerParameters())


def test_reference_ipopt_options(fake):
    mpc_mod.MPC(*_args(), Ts=0.1, N=20)
    a = fake.instances[-1].args
    assert a["tol"] == 1e-4 and a["acceptable_tol"] == 1e-2 and a["acceptable_iter"] == 15
    assert a["max_iter"] == FixedControllerParameters.max_iter == 500
    fp = FixedControllerParameters()
    assert a["lambda_s"] == fp.lambda_s and a["q_v_max"] == fp.q_v_max and a["v_max"] == fp.v_max
    assert a["N"] == 20 and a["Ts"] == 0.1 and a["model"] == "dyn" and a["precision"] == "fp64"
    # overriding the options gives a separate cached handle
    mpc_mod.MPC(*_args(), Ts=0.1, N=20, tol=1e-8, acceptable_iter=0)
    assert len(fake.instances) == 2 and fake.instances[-1].args["tol"] == 1e-8
    mpc_mod.MPC(*_args(), Ts=0.1, N=20)
    assert len(fake.instances) == 2  # the default handle is reused


@pytest.mark.parametrize("status,ok", [(0, True), (1, True), (2, False), (3, False), (4, False)])
def test_failure_semantics(fake, status, ok):
    mpc_mod.MPC(*_args(), Ts=0.1, N=20)  # create the handle
    fake.instances[-1].status = status
    m = mpc_mod.MPC(*_args(), Ts=0.1, N=20)
    sol, ret, dual = m.solution()
    assert bool(sol) == ok and (dual is not None) == ok
    States, U, S_hat, eC, eL = ret  # the last iterate either way (opti.debug.value on failure)
    assert States.shape == (6, 21) and U.shape == (2, 20) and S_hat.shape == (21,) and len(eC) == 20
    if ok:
        assert dual.shape == (13 * 20 + 9,)


def test_state0_rows_and_warm_start(fake):
    m = mpc_mod.MPC(*_args(throttle=None, steer=0.1), last_controls=[(0.1 * i, -0.01 * i) for i in range(20)],
                    Ts=0.1, N=20)
    b = fake.instances[-1].batches[-1]
    assert math.isnan(b["state0"][6, 0]) and b["state0"][7, 0] == 0.1
    u = b["u_init"][:, :, 0]
    assert np.allclose(u[0, :19], 0.1 * np.arange(1, 20)) and u[0, 19] == u[0, 18]  # shifted, last repeated
    assert m.solution()[2].shape == (13 * 20 + 8,)  # the throttle rate row of state0 is absent
    with pytest.raises(ValueError):
        mpc_mod.MPC(*_args(throttle=None), Ts=0.1, N=20)  # no initial guess for the controls
