"""Vehicle constants of the reference (models/VehicleParameters.py:3-41).

They parameterise the generated dynamics (csrc/gen_dynamics.h) through the
mr_config vehicle fields; changing a class attribute here changes the NLP the
next solver handle is built for, like editing the reference's class would.
"""
from dataclasses import dataclass


@dataclass
class VehicleParameters:
    m: float = 1845.0                  # mass (kg)
    max_steer = 70.0                   # wheel angle at full steer command (deg)
    min_steer = -70.0
    eta_motor = 0.9
    T_max = 743.0                      # peak motor torque (N m)
    r_wheel = 0.37                     # wheel radius (m)
    C_wheel = 2 * 3.14 * r_wheel       # circumference with pi ~ 3.14 (quirk)
    R = 9.0                            # gear ratio
    rho = 1.225                        # air density
    C_d = 0.23                         # drag coefficient
    A_f = 2.2                          # frontal area (m^2)
    C_roll = 0.012                     # rolling resistance coefficient
    max_rpm = 15000
    regen_brake_accel = 0.2
    Iz: float = 3960.0                 # yaw inertia (kg m^2)
    lf: float = 0.8                    # CoM to front axle (m)
    lr: float = 2                      # CoM to rear axle (m)
    Cf: float = 65_000                 # front cornering stiffness
    Cr: float = 65_000                 # rear cornering stiffness
    g: float = 9.81
    Vblendmin: float = 2               # kinematic below this speed (blended model)
    Vblendmax: float = 15              # dynamic above this speed
    Ts: int = 0.05
    car_width = 1.85


def config_fields():
    """mr_config vehicle fields from the (possibly modified) class attributes."""
    V = VehicleParameters
    return dict(m=V.m, Iz=V.Iz, lf=V.lf, lr=V.lr, Cf=V.Cf, Cr=V.Cr, T_max=V.T_max, r_wheel=V.r_wheel,
                C_wheel=V.C_wheel, R=V.R, rho=V.rho, C_d=V.C_d, A_f=V.A_f, C_roll=V.C_roll, g=V.g,
                max_steer_deg=V.max_steer, Vblendmin=V.Vblendmin, Vblendmax=V.Vblendmax)
