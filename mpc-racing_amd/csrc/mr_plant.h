// Plant models of the reference's closed loop (models/*.py), fp64, one lane per vehicle.
//
// These are the numpy "simulator-side" models the reference uses to stand in for CARLA
// (script/verify_*.py) -- NOT the MPC's internal dynamics (control/MPC.py:186-260), from which
// they differ: piecewise engine efficiency and steer gain, regenerative brake
// at throttle == 0, the Gaussian "carla_penalty", slip angles over vx (no +0.1), yaw wrapped by
// atan2(sin, cos), the kinematic yaw integrated with the new tan(delta) rate, and the true pi in
// deg2rad.  Evaluation order follows the Python expressions term by term.
#pragma once
#include "mr_common.h"

namespace mr {

enum PlantModel { PLANT_KIN = 0, PLANT_DYN = 1, PLANT_BLEND = 2 };

// models/VehicleParameters.py:3-41 (the plant reads the class defaults)
struct PlantConst {
  static constexpr double m = 1845.0, max_steer = 70.0, T_max = 743.0, r_wheel = 0.37;
  static constexpr double C_wheel = 2 * 3.14 * 0.37, R = 9.0, rho = 1.225, C_d = 0.23, A_f = 2.2;
  static constexpr double C_roll = 0.012, regen_brake_accel = 0.2, Iz = 3960.0, lf = 0.8, lr = 2.0;
  static constexpr double Cf = 65000.0, Cr = 65000.0, g = 9.81, Vblendmin = 2.0, Vblendmax = 15.0;
};

// Model.Fx (models/Model.py:15-64); v_x of the current state
MR_HD double plant_fx(double throttle, double v_x) {
  typedef PlantConst C;
  const double regen_brake_force = throttle == 0.0 ? C::regen_brake_accel * 9.81 * C::m : 0.0;
  const double wheel_rpm = (v_x / C::C_wheel) * 60;
  const double rpm = wheel_rpm * C::R * 4.5;
  const double eta = rpm < 9000 ? 1.0 : (rpm < 9500 ? 0.88 : (rpm < 10400 ? 0.81 : (rpm < 12500 ? 0.71 : 0.675)));
  // scipy.stats.norm.pdf(throttle, loc=0.5, scale=0.0775): exp(-z**2/2) / sqrt(2 pi) / scale
  const double z = (throttle - 0.5) / 0.0775;
  const double carla_penalty = exp(-(z * z) / 2.0) / 2.5066282746310002 / 0.0775 * C::m;
  const double wheel_force = throttle * eta * C::T_max * C::R / C::r_wheel;
  const double drag_force = 0.5 * C::rho * C::C_d * C::A_f * (v_x * v_x);
  const double rolling_resistance = C::C_roll * C::m * C::g;
  return wheel_force - drag_force - rolling_resistance - regen_brake_force - carla_penalty;
}

// Model.steer_cmd_to_angle (models/Model.py:66-81): piecewise gain, numpy deg2rad = x * (pi/180)
MR_HD double plant_steer_angle(double steer_cmd, double v_x, double v_y) {
  const double vel = sqrt(v_x * v_x + v_y * v_y) * 3.6;
  const double gain = vel < 20.0 ? 1.0 : (vel < 60.0 ? 0.9 : (vel < 120.0 ? 0.8 : 0.7));
  return steer_cmd * PlantConst::max_steer * gain * (3.141592653589793 / 180.0);
}

// KinematicBicycleModel.step (models/KinematicBicycleModel.py:11-48); x = (x, y, yaw, vx, vy, r)
MR_HD void plant_kin(const double* x, double thr, double steer, double Ts, double* o) {
  typedef PlantConst C;
  const double delta = plant_steer_angle(steer, x[3], x[4]);
  const double Fx = plant_fx(thr, x[3]);
  const double cy = cos(x[2]), sy = sin(x[2]);
  o[0] = x[0] + (x[3] * cy - x[4] * sy) * Ts;
  o[1] = x[1] + (x[3] * sy + x[4] * cy) * Ts;
  const double yaw_new = x[2] + ((x[3] / (C::lr + C::lf)) * tan(delta)) * Ts;
  o[3] = x[3] + (Fx / C::m) * Ts;
  o[5] = (x[3] / (C::lr + C::lf)) * tan(delta);
  o[4] = x[5] * C::lr;
  o[2] = atan2(sin(yaw_new), cos(yaw_new));
}

// DynamicBicycleModel.step (models/DynamicBicycleModel.py:16-78), linear tyres
MR_HD void plant_dyn(const double* x, double thr, double steer, double Ts, double* o) {
  typedef PlantConst C;
  const double Fx = plant_fx(thr, x[3]);
  const double delta = plant_steer_angle(steer, x[3], x[4]);
  const double theta_Vf = atan2(x[4] + C::lf * x[5], x[3]);
  const double theta_Vr = atan2(x[4] - C::lr * x[5], x[3]);
  const double Fyf = C::Cf * (delta - theta_Vf);
  const double Fyr = C::Cr * (-theta_Vr);
  const double sd = sin(delta), cd = cos(delta);
  const double v_x_dot = ((Fx - Fyf * sd) / C::m) + (x[4] * x[5]);
  const double v_y_dot = ((Fyf * cd + Fyr) / C::m) - (x[3] * x[5]);
  const double yaw_dot_dot = ((Fyf * cd * C::lf) - (Fyr * C::lr)) / C::Iz;
  const double cy = cos(x[2]), sy = sin(x[2]);
  o[0] = x[0] + (x[3] * cy - x[4] * sy) * Ts;
  o[1] = x[1] + (x[3] * sy + x[4] * cy) * Ts;
  const double yaw_new = x[2] + x[5] * Ts;
  o[3] = x[3] + v_x_dot * Ts;
  o[4] = x[4] + v_y_dot * Ts;
  o[5] = x[5] + yaw_dot_dot * Ts;
  o[2] = atan2(sin(yaw_new), cos(yaw_new));
}

// BlendedBicycleModel.step (models/BlendedBicycleModel.py:18-58): both models from the same
// state, lambda = clip((hypot(vx, vy) - 2) / (15 - 2), 0, 1), elementwise blend (wrapped yaws)
MR_HD void plant_step(int model, const double* x, double thr, double steer, double Ts, double* o) {
  if (model == PLANT_KIN) { plant_kin(x, thr, steer, Ts, o); return; }
  if (model == PLANT_DYN) { plant_dyn(x, thr, steer, Ts, o); return; }
  double k[6], d[6];
  plant_kin(x, thr, steer, Ts, k);
  plant_dyn(x, thr, steer, Ts, d);
  const double vel = hypot(x[3], x[4]);
  double lam = (vel - PlantConst::Vblendmin) / (PlantConst::Vblendmax - PlantConst::Vblendmin);
  lam = lam < 0.0 ? 0.0 : (lam > 1.0 ? 1.0 : lam);
  for (int j = 0; j < 6; ++j) o[j] = lam * d[j] + (1 - lam) * k[j];
}

}  // namespace mr
