// Per-instance driver shared by the gfx950 kernel and the host test build:
// reads instance i of the SoA batch inputs, solves, writes its outputs.
#pragma once
#include "../../include/mpcracing.h"
#include "mr_solver.h"

namespace mr {

template <typename T>
MR_HD void fill_params(const mr_config& c, const TyreCoef<double>& tf, const TyreCoef<double>& tr, ProbParams<T>& P) {
  P.N = c.N;
  P.model = c.model;
  P.lane = c.lane_bounds;
  P.Ts = T(c.Ts);
  P.lambda_s = T(c.lambda_s); P.alpha_L = T(c.alpha_L);
  P.min_steer = T(c.min_steer); P.max_steer = T(c.max_steer); P.min_thr = T(c.min_throttle);
  P.max_dsteer = T(c.max_steer_delta); P.min_dsteer = T(c.min_steer_delta);
  P.max_dthr = T(c.max_throttle_delta); P.min_dthr = T(c.min_throttle_delta);
  P.q_vmax = T(c.q_v_max); P.v_max = T(c.v_max); P.min_ds = T(c.min_s_delta);
  VehParams<T>& V = P.veh;
  V.m = T(c.m); V.Iz = T(c.Iz); V.lf = T(c.lf); V.lr = T(c.lr); V.Cf = T(c.Cf); V.Cr = T(c.Cr);
  V.T_max = T(c.T_max); V.r_wheel = T(c.r_wheel); V.C_wheel = T(c.C_wheel); V.R = T(c.R); V.rho = T(c.rho);
  V.C_d = T(c.C_d); V.A_f = T(c.A_f); V.C_roll = T(c.C_roll); V.g = T(c.g); V.max_steer = T(c.max_steer_deg);
  V.Vblendmin = T(c.Vblendmin); V.Vblendmax = T(c.Vblendmax);
  P.tf = {T(tf.B), T(tf.C), T(tf.E), T(tf.BCD), T(tf.K2)};
  P.tr = {T(tr.B), T(tr.C), T(tr.E), T(tr.BCD), T(tr.K2)};
  P.tol = T(c.tol);
  P.acc_tol = T(c.acceptable_tol);
  P.acc_iter = c.acceptable_iter;
  P.max_iter = c.max_iter;
}

// Taylor shift of a highest-first global-s polynomial to ascending powers of sigma = s - s0.
MR_HD void taylor_shift4(const double* c_desc, double s0, double* a) {
  double c[5];
  for (int j = 0; j < 5; ++j) c[j] = c_desc[4 - j];  // ascending
  // repeated synthetic division by (s - s0)
  for (int i = 0; i < 5; ++i)
    for (int j = 3; j >= i; --j) c[j] += s0 * c[j + 1];
  for (int j = 0; j < 5; ++j) a[j] = c[j];
}

template <typename T, int MODEL>
MR_HD SolveOut solve_instance(const ProbParams<T>& P, const mr_inputs& in, const mr_outputs& out, int64_t B,
                              int64_t i, WS<T> W) {
  const int N = P.N;
  Inst<T> I;
  const double X0 = in.state0[0 * B + i], Y0 = in.state0[1 * B + i];
  const double s0 = in.s0[i];
  I.x0[0] = T(0);
  I.x0[1] = T(0);
  for (int j = 2; j < 6; ++j) I.x0[j] = T(in.state0[j * B + i]);
  double thr0 = in.state0[6 * B + i], st0 = in.state0[7 * B + i];
  I.has_thr0 = (thr0 == thr0);
  I.has_steer0 = (st0 == st0);
  I.thr0 = I.has_thr0 ? T(thr0) : T(0);
  I.steer0 = I.has_steer0 ? T(st0) : T(0);
  double cxd[5], cyd[5], ax[5], ay[5];
  for (int j = 0; j < 5; ++j) { cxd[j] = in.cx[j * B + i]; cyd[j] = in.cy[j * B + i]; }
  taylor_shift4(cxd, s0, ax);
  taylor_shift4(cyd, s0, ay);
  ax[0] -= X0;
  ay[0] -= Y0;
  for (int j = 0; j < 5; ++j) { I.ax[j] = T(ax[j]); I.ay[j] = T(ay[j]); }
  I.max_err = T(in.max_error[i]);
  I.alpha_c = T(in.runtime[0 * B + i]);
  I.d_max = T(in.runtime[1 * B + i]);
  I.q_vy = T(in.runtime[2 * B + i]);
  I.n = (int)in.runtime[3 * B + i];
  if (I.n < 1) I.n = 1;
  I.beta = T(in.runtime[4 * B + i]);
  I.org[0] = T(X0);
  I.org[1] = T(Y0);
  I.org[2] = T(s0);
  Solver<T, MODEL> S(P, I, W);
  if (out.trace && out.trace_instance == i) { S.trace = out.trace; S.trace_cap = out.trace_cap; }
  S.init(in.u_init ? in.u_init + i : nullptr, B);
  SolveOut r = S.solve();
  // outputs (the ret tuple of control/MPC.py:166-171), back in global coordinates
  const int b = S.cur;
  for (int k = 0; k <= N; ++k) {
    T z[NZS];
    S.load_z(k, b, z);
    out.X[(0 * (N + 1) + k) * B + i] = (double)z[0] + X0;
    out.X[(1 * (N + 1) + k) * B + i] = (double)z[1] + Y0;
    for (int j = 2; j < 6; ++j) out.X[(j * (N + 1) + k) * B + i] = (double)z[j];
    out.S[k * B + i] = (double)z[6] + s0;
    if (k < N) {
      out.U[(0 * N + k) * B + i] = (double)z[11];
      out.U[(1 * N + k) * B + i] = (double)z[12];
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      out.eC[k * B + i] = (double)e.eC;
      out.eL[k * B + i] = (double)e.eL;
    }
  }
  out.status[i] = r.status;
  out.iters[i] = r.iters;
  if (out.obj) out.obj[i] = r.obj - (double)P.lambda_s * s0;  // -lambda_s * S_N in global s
  if (out.kkt) out.kkt[i] = r.kkt;
  if (out.constr_viol) out.constr_viol[i] = r.viol;
  return r;
}

// Cancellation-free Pacejka constants (fp64, host).
inline TyreCoef<double> pacejka_coef(const double* a, double Fz) {
  TyreCoef<double> c;
  c.C = a[0];
  double D = (a[1] * Fz + a[2]) * Fz;
  c.BCD = a[3] * sin(a[4] * atan(a[5] * Fz));
  c.B = c.BCD / (c.C * D);
  c.E = a[6] * Fz * Fz + a[7] * Fz + a[8];
  c.K2 = c.E * c.B * c.B;
  return c;
}

}  // namespace mr

namespace mr {
// Reference defaults: control/ControllerParameters.py:3-32, models/VehicleParameters.py:3-41,
// IPOPT options of control/MPC.py:151-161 (tol tightened to 1e-8: see DESIGN.md §Parity).
inline void fill_default_config(mr_config* c) {
  c->N = 30;
  c->model = MR_MODEL_DYNAMIC;
  c->precision = MR_PREC_FP64;
  c->lane_bounds = 0;
  c->max_batch = 1;
  c->device = 0;
  c->max_iter = 500;
  c->acceptable_iter = 15;
  c->Ts = 0.05;
  c->tol = 1e-8;
  c->acceptable_tol = 1e-6;
  c->lambda_s = 300; c->alpha_L = 500;
  c->min_steer = -0.9; c->max_steer = 0.9; c->min_throttle = -1.0;
  c->max_steer_delta = 0.2; c->min_steer_delta = -0.2;
  c->max_throttle_delta = 2.0; c->min_throttle_delta = -0.4;
  c->q_v_max = 2; c->v_max = 50; c->min_s_delta = 0.1;
  c->m = 1845.0; c->Iz = 3960.0; c->lf = 0.8; c->lr = 2.0; c->Cf = 65000.0; c->Cr = 65000.0;
  c->T_max = 743.0; c->r_wheel = 0.37; c->C_wheel = 2 * 3.14 * 0.37; c->R = 9.0; c->rho = 1.225;
  c->C_d = 0.23; c->A_f = 2.2; c->C_roll = 0.012; c->g = 9.81; c->max_steer_deg = 70.0;
  c->Vblendmin = 2.0; c->Vblendmax = 15.0;
  c->dispatch_order = 1;
}
}  // namespace mr
