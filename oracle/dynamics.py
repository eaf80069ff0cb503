"""Oracle restatement of the MPC vehicle dynamics (test infrastructure only).

Line-by-line restatements of the reference's symbolic dynamics, written against
a math namespace ``M`` so the same code runs on python floats / numpy (``NP``)
and on torch tensors (``TORCH``, used by ``oracle.nlp`` for exact autograd
derivatives):

* ``Fx``                  control/MPC.py:273-283  (C_wheel = 2*3.14*r_wheel, VehicleParameters.py:16)
* ``steer_cmd_to_angle``  control/MPC.py:262-271, control/util.py:10-11 (pi ~ 3.14)
* ``f_vehicle``           control/MPC.py:186-229  (dynamic bicycle, linear tyres, vx + 0.1)
* ``f_vehicle_kinematic`` control/MPC.py:231-260  (the unused kinematic form; A3 quirks kept)
* ``blend_lambda``        models/BlendedBicycleModel.py:22-26 (+ VehicleParameters.py:37-38)
* ``pacejka_naive``       learning/vehicle.py:79-92 (the magic formula exactly as written)

Constants are models/VehicleParameters.py:3-41.
"""
import math

import numpy as np


class VP:
    m = 1845.0
    max_steer = 70.0
    T_max = 743.0
    r_wheel = 0.37
    C_wheel = 2 * 3.14 * 0.37
    R = 9.0
    rho = 1.225
    C_d = 0.23
    A_f = 2.2
    C_roll = 0.012
    Iz = 3960.0
    lf = 0.8
    lr = 2.0
    Cf = 65000.0
    Cr = 65000.0
    g = 9.81
    Vblendmin = 2.0
    Vblendmax = 15.0
    car_width = 1.85


class _NP:
    atan2 = staticmethod(np.arctan2)
    sin = staticmethod(np.sin)
    cos = staticmethod(np.cos)
    tan = staticmethod(np.tan)
    sqrt = staticmethod(np.sqrt)
    atan = staticmethod(np.arctan)
    exp = staticmethod(np.exp)

    @staticmethod
    def stack(xs):
        return np.array(xs)


NP = _NP()


def _torch_ns():
    import torch

    class _T:
        atan2 = staticmethod(torch.atan2)
        sin = staticmethod(torch.sin)
        cos = staticmethod(torch.cos)
        tan = staticmethod(torch.tan)
        sqrt = staticmethod(torch.sqrt)
        atan = staticmethod(torch.atan)
        exp = staticmethod(torch.exp)

        @staticmethod
        def stack(xs):
            return torch.stack(xs)
    return _T()


def deg2rad(z):
    return (z / 360) * 2 * 3.14


def Fx(throttle, v_x):
    wheel_rpm = (v_x / VP.C_wheel) * 60
    rpm = wheel_rpm * VP.R * 4.5
    eta = -0.00004428225806 * rpm + 1.282413306
    wheel_force = throttle * eta * VP.T_max * VP.R / VP.r_wheel
    drag_force = 0.5 * VP.rho * VP.C_d * VP.A_f * (v_x ** 2)
    rolling_resistance = VP.C_roll * VP.m * VP.g
    return wheel_force - drag_force - rolling_resistance


def steer_cmd_to_angle(steer_cmd, v_x, v_y, M=NP):
    vel = M.sqrt(v_x ** 2 + v_y ** 2) * 3.6
    gain = -0.001971664699 * vel + 0.986547
    return deg2rad(steer_cmd * gain * VP.max_steer)


def lateral_forces_linear(alpha_f, alpha_r, Cf=VP.Cf, Cr=VP.Cr):
    return Cf * alpha_f, Cr * alpha_r


def f_vehicle(x, u, Ts, M=NP, tyres=None):
    """Dynamic bicycle (MPC.py:186-229). ``tyres`` optionally replaces the
    linear tyres Cf*(delta-theta_f), Cr*(-theta_r) by callables of the slip
    angle (learning/vehicle.py:155-160 substitution, config 5)."""
    X, Y, yaw, v_x, v_y, yaw_dot = x[0], x[1], x[2], x[3], x[4], x[5]
    F = Fx(u[0], v_x)
    delta = steer_cmd_to_angle(u[1], v_x, v_y, M)
    theta_Vf = M.atan2(v_y + VP.lf * yaw_dot, v_x + 0.1)
    theta_Vr = M.atan2(v_y - VP.lr * yaw_dot, v_x + 0.1)
    if tyres is None:
        Fyf = VP.Cf * (delta - theta_Vf)
        Fyr = VP.Cr * (-theta_Vr)
    else:
        Fyf = tyres[0](delta - theta_Vf)
        Fyr = tyres[1](-theta_Vr)
    v_x_dot = ((F - Fyf * M.sin(delta)) / VP.m) + (v_y * yaw_dot)
    v_y_dot = ((Fyf * M.cos(delta) + Fyr) / VP.m) - (v_x * yaw_dot)
    yaw_dot_dot = ((Fyf * M.cos(delta) * VP.lf) - (Fyr * VP.lr)) / VP.Iz
    return M.stack([
        X + (v_x * M.cos(yaw) - v_y * M.sin(yaw)) * Ts,
        Y + (v_x * M.sin(yaw) + v_y * M.cos(yaw)) * Ts,
        yaw + yaw_dot * Ts,
        v_x + v_x_dot * Ts,
        v_y + v_y_dot * Ts,
        yaw_dot + yaw_dot_dot * Ts,
    ])


def f_vehicle_kinematic(x, u, Ts, M=NP):
    """Kinematic form of MPC.py:231-260 (psi+ uses the old r, vy+ = r*lr,
    r+ = vx/(lr+lf)*tan(delta) algebraic)."""
    X, Y, yaw, v_x, v_y, yaw_dot = x[0], x[1], x[2], x[3], x[4], x[5]
    F = Fx(u[0], v_x)
    delta = steer_cmd_to_angle(u[1], v_x, v_y, M)
    return M.stack([
        X + (v_x * M.cos(yaw) - v_y * M.sin(yaw)) * Ts,
        Y + (v_x * M.sin(yaw) + v_y * M.cos(yaw)) * Ts,
        yaw + yaw_dot * Ts,
        v_x + (F / VP.m) * Ts,
        yaw_dot * VP.lr,
        (v_x / (VP.lr + VP.lf)) * M.tan(delta),
    ])


def blend_lambda(v_x, v_y):
    """models/BlendedBicycleModel.py:22-26: clip((hypot - Vmin)/(Vmax - Vmin), 0, 1)."""
    vel = math.hypot(float(v_x), float(v_y))
    return min(max((vel - VP.Vblendmin) / (VP.Vblendmax - VP.Vblendmin), 0.0), 1.0)


def f_blend(x, u, Ts, M=NP, tyres=None):
    """Build-defined Blended NLP dynamics: lambda*f_dyn + (1-lambda)*f_kin
    with the smooth MPC forms.  The region (lambda in (0,1) vs clipped) is chosen by
    the current speed; inside, lambda is the differentiable hypot law."""
    v_x, v_y = x[3], x[4]
    vel_f = math.hypot(float(v_x), float(v_y))
    fd = f_vehicle(x, u, Ts, M, tyres)
    fk = f_vehicle_kinematic(x, u, Ts, M)
    if vel_f <= VP.Vblendmin:
        return fk
    if vel_f >= VP.Vblendmax:
        return fd
    lam = (M.sqrt(v_x ** 2 + v_y ** 2) - VP.Vblendmin) / (VP.Vblendmax - VP.Vblendmin)
    return lam * fd + (1 - lam) * fk


def pacejka_naive(alpha, a, Fz, M=NP):
    """learning/vehicle.py:79-92 verbatim math (Sh = Sv = 0)."""
    C = a[0]
    D = (a[1] * Fz + a[2]) * Fz
    BCD = a[3] * math.sin(a[4] * math.atan(a[5] * Fz))
    B = BCD / (C * D)
    E = a[6] * Fz ** 2 + a[7] * Fz + a[8]
    phi = (1 - E) * alpha + (E / B) * M.atan(B * alpha)
    return D * M.sin(C * M.atan(B * phi))


def pacejka_mp(alpha, a, Fz, dps=60):
    """The same formula in mpmath at ``dps`` digits: the exact value of the
    reference's expression, free of its fp64 cancellation (|E| ~ 1e10)."""
    import mpmath as mp
    with mp.workdps(dps):
        a = [mp.mpf(v) for v in a]
        Fz = mp.mpf(Fz)
        al = mp.mpf(alpha)
        C = a[0]
        D = (a[1] * Fz + a[2]) * Fz
        BCD = a[3] * mp.sin(a[4] * mp.atan(a[5] * Fz))
        B = BCD / (C * D)
        E = a[6] * Fz ** 2 + a[7] * Fz + a[8]
        phi = (1 - E) * al + (E / B) * mp.atan(B * al)
        return float(D * mp.sin(C * mp.atan(B * phi)))


MODELS = {"kin": "kinematic", "dyn": "dynamic", "blend": "blended",
          "blend_pacejka": "blended + pacejka", "dyn_pacejka": "dynamic + pacejka"}


def model_fn(model, tyres=None):
    if model == "kin":
        return lambda x, u, Ts, M=NP: f_vehicle_kinematic(x, u, Ts, M)
    if model == "dyn":
        return lambda x, u, Ts, M=NP: f_vehicle(x, u, Ts, M)
    if model == "dyn_pacejka":
        return lambda x, u, Ts, M=NP: f_vehicle(x, u, Ts, M, tyres)
    if model == "blend":
        return lambda x, u, Ts, M=NP: f_blend(x, u, Ts, M)
    if model == "blend_pacejka":
        return lambda x, u, Ts, M=NP: f_blend(x, u, Ts, M, tyres)
    raise ValueError(model)
