// Per-instance primal-dual interior-point solver of the racing-MPC NLP.
//
// Replaces the CasADi Opti + IPOPT solve of control/MPC.py:30-181 (one
// instance per call) by one thread per instance running the whole solve.
//
// Formulation (equivalent reformulation of MPC.py's NLP):
//   stage state  x_k = [X, Y, psi, vx, vy, r, S, p_thr, p_steer, w_thr, w_steer]   (NX = 11)
//   stage input  u_k = [thr, steer, dS]                                              (NU = 3)
//   x_{k+1} = F(x_k, u_k):  vehicle block by the generated model (MPC.py:186-260),
//     S+ = S + dS (S_hat differences, MPC.py:134), p+ = (thr, steer) (previous control,
//     for the rate rows MPC.py:142-143 and the beta_delta term MPC.py:97),
//     w+ = (k == 0 ? (thr, steer) : w) (frozen U[:,0] for the wrap-around row at i = 0,
//     which reads U[:, -1] = U[:, N-1], MPC.py:142-143).
//   x_0 fixed: X_0 = state0, S_0 = s0 (MPC.py:101-107), p_0 = (throttle0, steer0) so the
//   stage-0 rate rows are the state0 rows of MPC.py:145-149.
//   Positions and progress are kept relative to (state0.x, state0.y, s0); the global-s
//   centerline polynomials (util.make_poly, highest order first) are Taylor-shifted to
//   sigma = s - s0 in fp64 before the solve (same polynomial, no cancellation).
//
// Newton steps are computed by a Riccati recursion on the stage-wise KKT system
// (inequalities condensed by the barrier); the algorithmic rules follow IPOPT's
// default configuration used by MPC.py:151-161 (gradient-based objective scaling,
// monotone barrier update, fraction to the boundary, inertia correction, filter
// line search) plus a second-order correction that re-rolls the shooting states.
#pragma once
#include "mr_common.h"
#include "gen_dynamics.h"
#ifndef MR_PROF
#define MR_PROF(slot, stmt) stmt
#endif

namespace mr {

enum ModelId { MODEL_KIN = 0, MODEL_DYN = 1, MODEL_BLEND = 2, MODEL_BLEND_PACEJKA = 3, MODEL_DYN_PACEJKA = 4 };

constexpr int NX = 11, NU = 3, NZ = 14, NROW = 7, NI = 17;
constexpr int NZS = NZ + 1;  // stored stage vector: z plus one unused slot (index 14, always 0)
constexpr int JL = 14;       // slots 14, 15, 16: lane rows e_C + m + t >= 0, m - e_C + t >= 0, t >= 0
constexpr int NH = NZ * (NZ + 1) / 2;  // packed upper triangle of the 14x14 stage Hessian
constexpr int NP = NX * (NX + 1) / 2;  // packed P
// IPOPT's inertia correction delta_w I regularises the NLP's own variables (the reference's States, S_hat
// and U, control/MPC.py:62-64).  In the stage-wise restatement those are x_k[0..5], S = x_k[6] and
// u_k[0..1]; the restatement's extra variables -- Delta-S (u_k[2]), the previous-control copy p (x_k[7..8])
// and the frozen U[:,0] copy w (x_k[9..10]), each fixed by equality rows -- get no shift, so the regularised
// Newton step is the one IPOPT computes in the reference's variables (a shift on the copies would add
// further terms to the reference variables' diagonal through those rows).  MR_DELTA_ALL=1: every stage
// variable shifted (the round-2 rule, A/B).
#ifndef MR_DELTA_ALL
#define MR_DELTA_ALL 0
#endif
MR_HD constexpr bool delta_var(int i) { return MR_DELTA_ALL ? i < NZ : (i <= 6 || i == 11 || i == 12); }
// IPOPT's optimality error (scaled stationarity, primal and complementarity) measured on the reference's NLP
// rather than the restatement: the stationarity of each reference variable is the sum of its restated
// copies' (U_k = u_k[0..1] + p_{k+1} (+ every w_j for U_0); S_k = S_k + Delta-S_{k-1} - Delta-S_k), the
// equality multipliers are the vehicle rows' nu_k[0..5] plus those of the initial-state rows X_0 = state0,
// S_0 = s0, which the restatement eliminates and which are therefore carried as nu_0[0..6] (stepped by the
// stage-0 costate, P_0 dx_0 + p_0 with dx_0 = 0), m_e = 6N + 7.  The restoration phase keeps the
// restatement's measure.  MR_KKT_RESTATED=1: the restatement's measure throughout (round 2, A/B).
#ifndef MR_KKT_RESTATED
#define MR_KKT_RESTATED 0
#endif

// Workspace fields per stage (SoA: element (k, f) of instance i at base[(k*NF + f)*stride + i]).
struct WF {
  enum {
    Z0 = 0, Z1 = Z0 + NZS, DZ = Z1 + NZS, S0 = DZ + NZS, S1 = S0 + NI, LAM = S1 + NI, DLAM = LAM + NI,
    DS = DLAM + NI, DNU = DS + NI, H = DNU + NX, G0 = H + NH, G1 = G0 + NZ, GL = G1 + NZ,
    J = GL + NZ, C = J + 48, P = C + NX, PV0 = P + NP, PV1 = PV0 + NX, K = PV1 + NX, K0 = K + NU * NX,
    K1 = K0 + NU,
    // watchdog snapshot: the iterate and the search direction where the watchdog started
    WZ = K1 + NU, WSL = WZ + NZS, WLAM = WSL + NI, WDZ = WLAM + NI, WDS = WDZ + NZS,
    WDLAM = WDS + NI, WDNU = WDLAM + NI,
    // restoration phase: row relaxations p, n, their bound duals and steps, the reference point z_R
    RP = WDNU + NX, RN = RP + NI, RVP = RN + NI, RVN = RVP + NI, RDP = RVN + NI, RDN = RDP + NI, RDVP = RDN + NI,
    RDVN = RDVP + NI, RY = RDVN + NI, RDY = RY + NI, RZ = RDY + NI,
    // restoration relaxations of the 6 vehicle dynamics rows of x_{k+1} = F(x_k, u_k) (stage k < N):
    // p, n, duals, steps, and the condensed disturbance weight / gradient for the Riccati sweep
    CP = RZ + NZS, CN = CP + 6, CVP = CN + 6, CVN = CVP + 6, CDP = CVN + 6, CDN = CDP + 6, CDVP = CDN + 6,
    CDVN = CDVP + 6, CSW = CDVN + 6, CGW0 = CSW + 6, CGW1 = CGW0 + 6, NF = CGW1 + 6
  };
};

MR_HD int hidx(int i, int j) {  // packed upper index of symmetric NZ x NZ
  if (i > j) { int t = i; i = j; j = t; }
  return i * NZ - (i * (i - 1)) / 2 + (j - i);
}
MR_HD int pidx(int i, int j) {  // packed upper index of symmetric NX x NX
  if (i > j) { int t = i; i = j; j = t; }
  return i * NX - (i * (i - 1)) / 2 + (j - i);
}

template <typename T>
struct ProbParams {
  int N, model, lane;
  T Ts;
  // control/ControllerParameters.py FixedControllerParameters
  T lambda_s, alpha_L, min_steer, max_steer, min_thr, max_dsteer, min_dsteer, max_dthr, min_dthr, q_vmax, v_max,
      min_ds;
  VehParams<T> veh;
  TyreCoef<T> tf, tr;
  // solver options
  T tol, acc_tol;
  int acc_iter, max_iter;
};

// Per-instance inputs in solver coordinates.
template <typename T>
struct Inst {
  T x0[6];
  T thr0, steer0;
  int has_thr0, has_steer0;
  T ax[5], ay[5];  // ascending coefficients in sigma = s - s0, minus the (X0, Y0) origin
  T max_err, alpha_c, d_max, q_vy, beta;
  int n;
  T org[3];  // global X0, Y0, s0 of the solver origin (the restoration phase's proximity scaling)
};

template <typename T>
struct WS {
  T* base;
  int64_t stride;
  MR_HD T& operator()(int k, int f) const { return base[((int64_t)k * WF::NF + f) * stride]; }
};

// ----------------------------------------------------------------------------------------
// Model dispatch
// ----------------------------------------------------------------------------------------
template <typename T, int MODEL>
struct Dyn {
  static MR_HD void slip(const ProbParams<T>& P, const T* x, const T* u, T& af, T& ar) {
    const VehParams<T>& V = P.veh;
    T vel = mr_sqrt(x[3] * x[3] + x[4] * x[4]) * T(3.6);
    T gain = T(-0.001971664699) * vel + T(0.986547);
    T delta = (u[1] * gain * V.max_steer / T(360)) * T(2) * T(3.14);
    af = delta - mr_atan2(x[4] + V.lf * x[5], x[3] + T(0.1));
    ar = -mr_atan2(x[4] - V.lr * x[5], x[3] + T(0.1));
  }
  // blend region: 0 -> kinematic (lambda = 0), 1 -> dynamic (lambda = 1), 2 -> blend law
  static MR_HD int region(const ProbParams<T>& P, const T* x) {
    T vel = mr_sqrt(x[3] * x[3] + x[4] * x[4]);
    if (vel <= P.veh.Vblendmin) return 0;
    if (vel >= P.veh.Vblendmax) return 1;
    return 2;
  }
  static MR_HD void f(const ProbParams<T>& P, const T* x, const T* u, T* out) {
    const VehParams<T>& V = P.veh;
    if (MODEL == MODEL_KIN) { kin_f(V, P.Ts, x, u, out); return; }
    if (MODEL == MODEL_DYN) { dyn_lin_f(V, P.Ts, x, u, out); return; }
    TyreJet<T> jf{}, jr{};
    if (MODEL == MODEL_BLEND_PACEJKA || MODEL == MODEL_DYN_PACEJKA) {
      T af, ar;
      slip(P, x, u, af, ar);
      jf = pacejka_jet(P.tf, af);
      jr = pacejka_jet(P.tr, ar);
    }
    if (MODEL == MODEL_DYN_PACEJKA) { dyn_tyre_f(V, P.Ts, x, u, jf, jr, out); return; }
    int rg = region(P, x);
    if (rg == 0) { kin_f(V, P.Ts, x, u, out); return; }
    if (MODEL == MODEL_BLEND) {
      if (rg == 1) dyn_lin_f(V, P.Ts, x, u, out); else blend_lin_f(V, P.Ts, x, u, out);
    } else {
      if (rg == 1) dyn_tyre_f(V, P.Ts, x, u, jf, jr, out); else blend_tyre_f(V, P.Ts, x, u, jf, jr, out);
    }
  }
  static MR_HD void fjh(const ProbParams<T>& P, const T* x, const T* u, const T* nu, T* out, T* J, T* H) {
    const VehParams<T>& V = P.veh;
    if (MODEL == MODEL_KIN) { kin_fjh(V, P.Ts, x, u, nu, out, J, H); return; }
    if (MODEL == MODEL_DYN) { dyn_lin_fjh(V, P.Ts, x, u, nu, out, J, H); return; }
    TyreJet<T> jf{}, jr{};
    if (MODEL == MODEL_BLEND_PACEJKA || MODEL == MODEL_DYN_PACEJKA) {
      T af, ar;
      slip(P, x, u, af, ar);
      jf = pacejka_jet(P.tf, af);
      jr = pacejka_jet(P.tr, ar);
    }
    if (MODEL == MODEL_DYN_PACEJKA) { dyn_tyre_fjh(V, P.Ts, x, u, nu, jf, jr, out, J, H); return; }
    int rg = region(P, x);
    if (rg == 0) { kin_fjh(V, P.Ts, x, u, nu, out, J, H); return; }
    if (MODEL == MODEL_BLEND) {
      if (rg == 1) dyn_lin_fjh(V, P.Ts, x, u, nu, out, J, H); else blend_lin_fjh(V, P.Ts, x, u, nu, out, J, H);
    } else {
      if (rg == 1) dyn_tyre_fjh(V, P.Ts, x, u, nu, jf, jr, out, J, H);
      else blend_tyre_fjh(V, P.Ts, x, u, nu, jf, jr, out, J, H);
    }
  }
};

// ----------------------------------------------------------------------------------------
// Centerline polynomial (util.make_poly) and the contouring / lag errors (MPC.py:71-81)
// ----------------------------------------------------------------------------------------
template <typename T>
struct Err {
  T eC, eL;
  T gC[3], gL[3];  // gradients over (X, Y, S)
  T hC[6], hL[6];  // packed 3x3 upper: (XX, XY, XS, YY, YS, SS)
};

template <typename T>
MR_HD void poly3(const T* a, T s, T& g0, T& g1, T& g2, T& g3) {
  g0 = (((a[4] * s + a[3]) * s + a[2]) * s + a[1]) * s + a[0];
  g1 = ((T(4) * a[4] * s + T(3) * a[3]) * s + T(2) * a[2]) * s + a[1];
  g2 = (T(12) * a[4] * s + T(6) * a[3]) * s + T(2) * a[2];
  g3 = T(24) * a[4] * s + T(6) * a[3];
}

template <typename T>
MR_HD void errors(const Inst<T>& I, T X, T Y, T S, Err<T>& e, bool second) {
  T gx, dgx, hx, tx, gy, dgy, hy, ty;
  poly3(I.ax, S, gx, dgx, hx, tx);
  poly3(I.ay, S, gy, dgy, hy, ty);
  T a = X - gx, b = Y - gy;
  e.eC = dgy * a - dgx * b;
  e.eL = -dgx * a - dgy * b;
  e.gC[0] = dgy; e.gC[1] = -dgx; e.gC[2] = hy * a - hx * b;
  e.gL[0] = -dgx; e.gL[1] = -dgy; e.gL[2] = -hx * a - hy * b + dgx * dgx + dgy * dgy;
  if (second) {
    e.hC[0] = T(0); e.hC[1] = T(0); e.hC[2] = hy; e.hC[3] = T(0); e.hC[4] = -hx;
    e.hC[5] = ty * a - tx * b - hy * dgx + hx * dgy;
    e.hL[0] = T(0); e.hL[1] = T(0); e.hL[2] = -hx; e.hL[3] = T(0); e.hL[4] = -hy;
    e.hL[5] = -tx * a - ty * b + T(3) * (dgx * hx + dgy * hy);
  }
}

template <typename T>
MR_HD void ipow(T e, int n, T& v, T& d1, T& d2) {
  // e^n, n e^(n-1), n(n-1) e^(n-2) for integer n >= 1
  T p2 = T(1);
  #pragma unroll
  for (int i = 0; i < n - 2; ++i) p2 *= e;
  if (n >= 2) {
    d2 = T(n) * T(n - 1) * p2;
    d1 = T(n) * p2 * e;
    v = p2 * e * e;
  } else {
    d2 = T(0);
    d1 = T(1);
    v = e;
  }
}

// ----------------------------------------------------------------------------------------
// Inequality rows (MPC.py:134-149, optional lane row :135): lo <= c(z) <= hi
// ----------------------------------------------------------------------------------------
template <typename T>
struct Row {
  int active, n;
  int idx[3];
  T a[3];
  T c, lo, hi;
  int lane;
};

template <typename T>
MR_HD void make_row(const ProbParams<T>& P, const Inst<T>& I, int k, int r, const T* z, const Err<T>* e, Row<T>& R) {
  const int N = P.N;
  R.active = 0; R.n = 0; R.lane = 0; R.c = T(0); R.lo = T(0); R.hi = T(0);
  if (k == N) return;  // terminal stage: only the lane rows (lane_active)
  switch (r) {
    case 0:  // MPC.py:138-139 (upper = class attribute d_max, quirk)
      R.active = 1; R.n = 1; R.idx[0] = 11; R.a[0] = T(1); R.c = z[11]; R.lo = P.min_thr; R.hi = I.d_max; break;
    case 1:  // MPC.py:140-141
      R.active = 1; R.n = 1; R.idx[0] = 12; R.a[0] = T(1); R.c = z[12]; R.lo = P.min_steer; R.hi = P.max_steer; break;
    case 2:  // MPC.py:134: 0.1 <= S_i - S_{i-1} <= Ts*v_max
      R.active = 1; R.n = 1; R.idx[0] = 13; R.a[0] = T(1); R.c = z[13]; R.lo = P.min_ds; R.hi = P.Ts * P.v_max; break;
    case 3:  // MPC.py:142 (k >= 1) / :145-146 (k == 0 against state0.throttle)
      if (k >= 1 || I.has_thr0) {
        R.active = 1; R.n = 2; R.idx[0] = 11; R.a[0] = T(1); R.idx[1] = 7; R.a[1] = T(-1);
        R.c = z[11] - z[7]; R.lo = P.min_dthr; R.hi = P.max_dthr;
      }
      break;
    case 4:  // MPC.py:143 / :148-149
      if (k >= 1 || I.has_steer0) {
        R.active = 1; R.n = 2; R.idx[0] = 12; R.a[0] = T(1); R.idx[1] = 8; R.a[1] = T(-1);
        R.c = z[12] - z[8]; R.lo = P.min_dsteer; R.hi = P.max_dsteer;
      }
      break;
    case 5:  // MPC.py:142 at i = 0: U[0,0] - U[0,N-1] via the frozen copy w
      if (k == N - 1 && N >= 2) {
        R.active = 1; R.n = 2; R.idx[0] = 9; R.a[0] = T(1); R.idx[1] = 11; R.a[1] = T(-1);
        R.c = z[9] - z[11]; R.lo = P.min_dthr; R.hi = P.max_dthr;
      }
      break;
    case 6:  // MPC.py:143 at i = 0
      if (k == N - 1 && N >= 2) {
        R.active = 1; R.n = 2; R.idx[0] = 10; R.a[0] = T(1); R.idx[1] = 12; R.a[1] = T(-1);
        R.c = z[10] - z[12]; R.lo = P.min_dsteer; R.hi = P.max_dsteer;
      }
      break;
  }
}

// Lane rows on states i = 1..N (the commented MPC.py:135), two one-sided rows as the reference's
// opti.bounded(-max_error, e_hat_C, max_error): e_C + m >= 0, m - e_C >= 0.  An infeasible start is the
// restoration phase's business (IPOPT's way), not an elastic reformulation.
template <typename T>
MR_HD bool lane_active(const ProbParams<T>& P, int k) { return P.lane && k >= 1; }

template <typename T>
MR_HD void lane_d(const Inst<T>& I, T eC, T t, T* d) {  // t: the unused slot 14 (0)
  d[0] = eC + I.max_err + t;
  d[1] = I.max_err - eC + t;
  d[2] = t;
}

// ----------------------------------------------------------------------------------------
// Stage cost (MPC.py:86-98), scaled by obj_scale.  Stage 0 has no cost.
// ----------------------------------------------------------------------------------------
template <typename T>
MR_HD T stage_cost(const ProbParams<T>& P, const Inst<T>& I, int k, const T* z, const Err<T>& e, T sc, T* g, T* H) {
  // g: gradient (NZ), H: packed Hessian (NH) accumulated; either may be null
  if (k == 0) return T(0);
  const int N = P.N;
  T val = T(0);
  // q_v_y * vy^2
  T vy = z[4];
  val += I.q_vy * vy * vy;
  if (g) g[4] += sc * T(2) * I.q_vy * vy;
  if (H) H[hidx(4, 4)] += sc * T(2) * I.q_vy;
  // exp(q_v_max (vx - v_max))
  T ex = mr_exp(P.q_vmax * (z[3] - P.v_max));
  val += ex;
  if (g) g[3] += sc * P.q_vmax * ex;
  if (H) H[hidx(3, 3)] += sc * P.q_vmax * P.q_vmax * ex;
  // alpha_c eC^n + alpha_L eL^2 over (X, Y, S) = indices (0, 1, 6)
  T cv, c1, c2;
  ipow(e.eC, I.n, cv, c1, c2);
  val += I.alpha_c * cv + P.alpha_L * e.eL * e.eL;
  const int id3[3] = {0, 1, 6};
  if (g) {
    #pragma unroll
    for (int a = 0; a < 3; ++a)
      g[id3[a]] += sc * (I.alpha_c * c1 * e.gC[a] + T(2) * P.alpha_L * e.eL * e.gL[a]);
  }
  if (H) {
    int q = 0;
    #pragma unroll
    for (int a = 0; a < 3; ++a)
      #pragma unroll
      for (int b = a; b < 3; ++b, ++q) {
        T hv = I.alpha_c * (c2 * e.gC[a] * e.gC[b] + c1 * e.hC[q]) +
               T(2) * P.alpha_L * (e.gL[a] * e.gL[b] + e.eL * e.hL[q]);
        H[hidx(id3[a], id3[b])] += sc * hv;
      }
  }
  if (k == N) {
    // terminal: -lambda_s * S_N (MPC.py:86)
    val += -P.lambda_s * z[6];
    if (g) g[6] += -sc * P.lambda_s;
  } else {
    // beta_delta (U1_i - U1_{i-1})^2 with U1_{i-1} = p_steer (MPC.py:97)
    T du = z[12] - z[8];
    val += I.beta * du * du;
    if (g) { g[12] += sc * T(2) * I.beta * du; g[8] -= sc * T(2) * I.beta * du; }
    if (H) {
      H[hidx(12, 12)] += sc * T(2) * I.beta;
      H[hidx(8, 8)] += sc * T(2) * I.beta;
      H[hidx(8, 12)] -= sc * T(2) * I.beta;
    }
  }
  return sc * val;
}

// Augmented dynamics value (vehicle block + linear S, p, w parts).
template <typename T, int MODEL>
MR_HD void faug(const ProbParams<T>& P, int k, const T* z, T* xn) {
  Dyn<T, MODEL>::f(P, z, z + NX, xn);
  xn[6] = z[6] + z[13];
  xn[7] = z[11];
  xn[8] = z[12];
  xn[9] = (k == 0) ? z[11] : z[9];
  xn[10] = (k == 0) ? z[12] : z[10];
}

// Restoration objective's proximity term (zeta/2) sum D_i^2 (z_i - zR_i)^2 over the reference's own
// variables (MPC.py:62-64): States X_i and S_hat_i (stage indices 0..6, k >= 1; X_0, S_0 are fixed) and
// U (indices 11, 12, k < N); D_i = min(1, 1/|zR_i|) of the global value.  Adds gradient / diagonal
// Hessian (either may be null), returns the term.
template <typename T>
MR_HD T prox_term(const Inst<T>& I, int k, int N, const T* z, const T* zr, T zeta, T* g, T* H) {
  T v = T(0);
  for (int i = 0; i < NZ; ++i) {
    const bool on = (i <= 6 && k >= 1) || ((i == 11 || i == 12) && k < N);
    if (!on) continue;
    const T glob = zr[i] + (i == 0 ? I.org[0] : (i == 1 ? I.org[1] : (i == 6 ? I.org[2] : T(0))));
    const T D = mr_min(T(1), T(1) / mr_max(mr_abs(glob), T(1e-30)));
    const T w = zeta * D * D, dz = z[i] - zr[i];
    v += T(0.5) * w * dz * dz;
    if (g) g[i] += w * dz;
    if (H) H[hidx(i, i)] += w;
  }
  return v;
}

// ----------------------------------------------------------------------------------------
// Small dense helpers
// ----------------------------------------------------------------------------------------
template <typename T>
MR_HD bool chol3(T* R, T* L) {  // R packed upper 3x3 (00,01,02,11,12,22) -> L lower (00,10,11,20,21,22)
  T l00 = R[0];
  if (!(l00 > T(0))) return false;
  l00 = mr_sqrt(l00);
  T l10 = R[1] / l00, l20 = R[2] / l00;
  T d1 = R[3] - l10 * l10;
  if (!(d1 > T(0))) return false;
  T l11 = mr_sqrt(d1);
  T l21 = (R[4] - l20 * l10) / l11;
  T d2 = R[5] - l20 * l20 - l21 * l21;
  if (!(d2 > T(0))) return false;
  T l22 = mr_sqrt(d2);
  L[0] = l00; L[1] = l10; L[2] = l11; L[3] = l20; L[4] = l21; L[5] = l22;
  return true;
}
template <typename T>
MR_HD void chol3_solve(const T* L, T* b) {  // solves (L L^T) x = b in place
  T y0 = b[0] / L[0];
  T y1 = (b[1] - L[1] * y0) / L[2];
  T y2 = (b[2] - L[3] * y0 - L[4] * y1) / L[5];
  T x2 = y2 / L[5];
  T x1 = (y1 - L[4] * x2) / L[2];
  T x0 = (y0 - L[1] * x1 - L[3] * x2) / L[0];
  b[0] = x0; b[1] = x1; b[2] = x2;
}

// y = A v for the augmented dynamics Jacobian w.r.t. x (11x11); J is the 6x8 vehicle Jacobian
template <typename T>
MR_HD void apply_A(const T* J, int k, const T* v, T* y) {
  #pragma unroll
  for (int i = 0; i < 6; ++i) {
    T acc = T(0);
    #pragma unroll
    for (int j = 0; j < 6; ++j) acc += J[i * 8 + j] * v[j];
    y[i] = acc;
  }
  y[6] = v[6];
  y[7] = T(0);
  y[8] = T(0);
  y[9] = (k == 0) ? T(0) : v[9];
  y[10] = (k == 0) ? T(0) : v[10];
}
// y = B w (11x3)
template <typename T>
MR_HD void apply_B(const T* J, int k, const T* w, T* y) {
  #pragma unroll
  for (int i = 0; i < 6; ++i) y[i] = J[i * 8 + 6] * w[0] + J[i * 8 + 7] * w[1];
  y[6] = w[2];
  y[7] = w[0];
  y[8] = w[1];
  y[9] = (k == 0) ? w[0] : T(0);
  y[10] = (k == 0) ? w[1] : T(0);
}
// y = A^T v (11); v, y may be of a wider type V than the Jacobian (fp64 multipliers of an fp32 solve)
template <typename T, typename V>
MR_HD void apply_At(const T* J, int k, const V* v, V* y) {
  #pragma unroll
  for (int j = 0; j < 6; ++j) {
    V acc = V(0);
    #pragma unroll
    for (int i = 0; i < 6; ++i) acc += V(J[i * 8 + j]) * v[i];
    y[j] = acc;
  }
  y[6] = v[6];
  y[7] = V(0);
  y[8] = V(0);
  y[9] = (k == 0) ? V(0) : v[9];
  y[10] = (k == 0) ? V(0) : v[10];
}
// y = B^T v (3)
template <typename T, typename V>
MR_HD void apply_Bt(const T* J, int k, const V* v, V* y) {
  V a0 = v[7], a1 = v[8];
  if (k == 0) { a0 += v[9]; a1 += v[10]; }
  #pragma unroll
  for (int i = 0; i < 6; ++i) { a0 += V(J[i * 8 + 6]) * v[i]; a1 += V(J[i * 8 + 7]) * v[i]; }
  y[0] = a0; y[1] = a1; y[2] = v[6];
}

// ----------------------------------------------------------------------------------------
// One-sided inequality rows in the Newton system (regular and restoration phase)
// ----------------------------------------------------------------------------------------
// A row d(z) >= 0 is d(z) - s = 0 with the slack s >= 0 (bound dual lam, the row multiplier).  In the
// restoration phase (IPOPT's l1 restoration NLP, Waechter & Biegler 2006 sec. 3.3) it is relaxed to
// d(z) - s - p + n = 0 with p, n >= 0 (bound duals vp, vn) and cost rho (p + n).  The slack-like
// variables are condensed out of the Newton system: the row adds sig a a^T to the Hessian and
// a (c0 + mu c1) to the gradient (a = grad d):
//   regular:      sig = lam / s,                          c0 = sig (d - s),  c1 = -1 / s
//   restoration:  1 / sig = s / lam + p / vp + n / vn,    r = d - s - p + n,
//                 c0 = sig (r - rho (n / vn - p / vp)),   c1 = -sig (1 / lam + 1 / vp - 1 / vn)
template <typename T>
MR_HD void row_cond(T d, T s, T lam, T& sig, T& c0, T& c1) {
  sig = lam / s;
  c0 = sig * (d - s);
  c1 = -T(1) / s;
}
template <typename T>
MR_HD void row_cond_r(T d, T s, T lam, T p, T n, T vp, T vn, T rho, T& sig, T& c0, T& c1) {
  const T is = s / lam, ip = p / vp, in = n / vn;
  sig = T(1) / (is + ip + in);
  c0 = sig * ((d - s - p + n) - rho * (in - ip));
  c1 = -sig * (T(1) / lam + T(1) / vp - T(1) / vn);
}
// Restoration row steps from the linearised residual e = (d - s - p + n) + a.dz: the new row
// multiplier eta = sig (G - e), G = rho (n/vn - p/vp) + mu (1/lam + 1/vp - 1/vn), then
//   ds = (mu/s - eta) s/lam,  dp = (mu/p - rho - eta) p/vp,  dn = (mu/n - rho + eta) n/vn,
//   dlam = eta - lam,  dvp = rho + eta - vp,  dvn = rho - eta - vn   (primal-dual bound-dual steps)
template <typename T>
MR_HD void row_steps_r(T e, T s, T lam, T p, T n, T vp, T vn, T rho, T mu, T& ds, T& dp, T& dn, T& dlam, T& dvp,
                       T& dvn) {
  const T is = s / lam, ip = p / vp, in = n / vn;
  const T sig = T(1) / (is + ip + in);
  const T G = rho * (in - ip) + mu * (T(1) / lam + T(1) / vp - T(1) / vn);
  const T eta = sig * (G - e);
  ds = (mu / s - eta) * is;
  dp = (mu / p - rho - eta) * ip;
  dn = (mu / n - rho + eta) * in;
  dlam = eta - lam;
  dvp = rho + eta - vp;
  dvn = rho - eta - vn;
}
// IPOPT's closed-form start of the restoration variables for a row residual c = d - s (so that
// c - p + n = 0): n = b + sqrt(b^2 + mu c / (2 rho)), b = (mu - rho c) / (2 rho), p = c + n; written
// without cancellation for b < 0
template <typename T>
MR_HD void resto_pn(T c, T mu, T rho, T& p, T& n) {
  const T b = (mu - rho * c) / (T(2) * rho), q = mu * c / (T(2) * rho);
  const T r = mr_sqrt(b * b + q);
  n = b >= T(0) ? b + r : q / (r - b);
  p = c + n;
}
// Restoration phase, relaxed vehicle dynamics rows F_i(x_k, u_k) - x_{k+1,i} - p_i + n_i = 0 (i < 6):
// the relaxation enters x_{k+1} as a disturbance w = dn - dp with cost 1/2 sw w^2 + (gw0 + mu gw1) w
// (p, n condensed as in row_cond_r: 1/sw = p/vp + n/vn, gw0 = sw rho (n/vn - p/vp),
// gw1 = sw (1/vp - 1/vn)).  Minimising the cost-to-go of stage k+1, V(xi) = 1/2 xi^T P xi +
// (p0 + mu p1)^T xi, over w gives the cost-to-go of xi = y + E w as a function of y:
//   M = P_vv + diag(sw) = L L^T,  Y = L^-1 P_v.,  P~ = P - Y^T Y,  p~ = p - Y^T L^-1 (p_v + gw)
// (false if M is not positive definite: the stage's inertia is wrong, as for a failed Q_uu pivot).
template <typename T>
MR_HD bool chol6(const T* M, T* L) {  // M, L: 6x6 row-major, L lower
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j <= i; ++j) {
      T v = M[i * 6 + j];
      for (int q = 0; q < j; ++q) v -= L[i * 6 + q] * L[j * 6 + q];
      if (i == j) {
        if (!(v > T(0))) return false;
        L[i * 6 + i] = mr_sqrt(v);
      } else {
        L[i * 6 + j] = v / L[j * 6 + j];
      }
    }
  return true;
}
template <typename T>
MR_HD void lsolve6(const T* L, T* b) {
  for (int i = 0; i < 6; ++i) {
    T v = b[i];
    for (int q = 0; q < i; ++q) v -= L[i * 6 + q] * b[q];
    b[i] = v / L[i * 6 + i];
  }
}
template <typename T>
MR_HD void ltsolve6(const T* L, T* b) {
  for (int i = 5; i >= 0; --i) {
    T v = b[i];
    for (int q = i + 1; q < 6; ++q) v -= L[q * 6 + i] * b[q];
    b[i] = v / L[i * 6 + i];
  }
}
// Evaluated in fp64 whatever T: where a relaxation is active (small sw) the vehicle block of P~ is the
// difference of two nearly equal terms of the size of P_vv (P_vv - P_vv M^-1 P_vv -> the parallel sum of
// P_vv and diag(sw)); in fp32 that difference is rounding noise of order eps |P_vv|, the next stages' Q_uu
// lose definiteness and the inertia correction climbs to 1e6..1e10 (profiles/r03_resto_fp64cond.json).
// Only restoration-phase factorisations run this.
template <typename T>
MR_HD bool noise_cond(T* Pm, T* p0, T* p1, const T* sw, const T* gw0, const T* gw1) {
  typedef double D;
  D M[36], L[36];
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) M[i * 6 + j] = (D)Pm[pidx(i, j)] + (i == j ? (D)sw[i] : 0.0);
  if (!chol6(M, L)) return false;
  D Y[6][NX], y0[6], y1[6];
  for (int j = 0; j < NX; ++j) {
    D col[6];
    for (int i = 0; i < 6; ++i) col[i] = (D)Pm[pidx(i, j)];
    lsolve6(L, col);
    for (int i = 0; i < 6; ++i) Y[i][j] = col[i];
  }
  for (int i = 0; i < 6; ++i) { y0[i] = (D)p0[i] + (D)gw0[i]; y1[i] = (D)p1[i] + (D)gw1[i]; }
  lsolve6(L, y0);
  lsolve6(L, y1);
  for (int i = 0; i < NX; ++i) {
    for (int j = i; j < NX; ++j) {
      D v = (D)Pm[pidx(i, j)];
      for (int a = 0; a < 6; ++a) v -= Y[a][i] * Y[a][j];
      Pm[pidx(i, j)] = (T)v;
    }
  }
  for (int i = 0; i < NX; ++i) {
    D v0 = (D)p0[i], v1 = (D)p1[i];
    for (int a = 0; a < 6; ++a) { v0 -= Y[a][i] * y0[a]; v1 -= Y[a][i] * y1[a]; }
    p0[i] = (T)v0;
    p1[i] = (T)v1;
  }
  return true;
}
// the disturbance step w = -M^-1 (nu_y[0..5] + gw), nu_y = P y + p the cost-to-go gradient at y
template <typename T>
MR_HD void noise_step(const T* Pm, const T* sw, const T* rhs, T* w) {
  T M[36], L[36];
  for (int i = 0; i < 6; ++i)
    for (int j = 0; j < 6; ++j) M[i * 6 + j] = Pm[pidx(i, j)] + (i == j ? sw[i] : T(0));
  chol6(M, L);
  for (int i = 0; i < 6; ++i) w[i] = -rhs[i];
  lsolve6(L, w);
  ltsolve6(L, w);
}
// the relaxation steps of one dynamics row from its disturbance step w (eta = sw (w + G)):
//   dp = (-eta - rho + mu/p) p/vp,  dn = (eta - rho + mu/n) n/vn,  dvp = rho + eta - vp,  dvn = rho - eta - vn
template <typename T>
MR_HD void dyn_steps_r(T w, T p, T n, T vp, T vn, T rho, T mu, T& dp, T& dn, T& dvp, T& dvn) {
  const T ip = p / vp, in = n / vn;
  const T sw = T(1) / (ip + in);
  const T G = rho * (in - ip) + mu * (T(1) / vp - T(1) / vn);
  const T eta = sw * (w + G);
  dp = (-eta - rho + mu / p) * ip;
  dn = (eta - rho + mu / n) * in;
  dvp = rho + eta - vp;
  dvn = rho - eta - vn;
}
// restoration-phase constants (IPOPT resto_penalty_parameter, required_infeasibility_reduction,
// bound_mult_reset_threshold)
constexpr double RESTO_RHO = 1000.0, RESTO_KAPPA = 0.9, RESTO_MULT_RESET = 1000.0;

// ----------------------------------------------------------------------------------------
// The solver
// ----------------------------------------------------------------------------------------
struct SolveOut {
  int status, iters;
  double kkt, obj;
};

#ifndef MR_FMAX
#define MR_FMAX 16
#endif
#ifndef MR_FILTER_RESET_TRIGGER
#define MR_FILTER_RESET_TRIGGER 5  // IPOPT filter_reset_trigger (0: heuristic off)
#endif
#ifndef MR_MAX_FILTER_RESETS
#define MR_MAX_FILTER_RESETS 5  // IPOPT max_filter_resets
#endif
#ifndef MR_LS_FAIL_MAX
#define MR_LS_FAIL_MAX 1000000
#endif
#ifndef MR_WD_TRIGGER
#define MR_WD_TRIGGER 10  // IPOPT watchdog_shortened_iter_trigger (0: watchdog off)
#endif
#ifndef MR_WD_TRIAL_MAX
#define MR_WD_TRIAL_MAX 3  // IPOPT watchdog_trial_iter_max
#endif
constexpr int FMAX = MR_FMAX;

template <typename T, int MODEL>
struct Solver {
  const ProbParams<T>& P;
  const Inst<T>& I;
  WS<T> W;
  int N;
  // iteration state
  int cur;          // which z/s buffer holds the current iterate
  T mu, sc, delta_last;
  T alpha_p, alpha_d;  // last accepted primal / dual step (lazy update)
  T theta_max, theta_min;
  T filt_th[FMAX], filt_ph[FMAX];
  int nfilt;
  // iteration aggregates (eval sweep)
  T stat_max, pr_max, theta, slam_max, slam_min, nu1, lam1, fval, logs;
  int me, mi;
  // restoration phase: mode, its penalty and proximity weight, and the original problem's state
  bool resto = false;
  T rho = T(RESTO_RHO), zeta = T(0);
  T mu_o, th_entry, delta_last_o, theta_max_o, theta_min_o;
  T ofilt_th[FMAX], ofilt_ph[FMAX];
  int onfilt;
  T tho_acc, pho_acc;  // original theta / barrier objective of the last trial point (restoration)
  double* trace = nullptr;  // optional per-iteration record (diagnostics)
  int trace_cap = 0;
  // the dynamics rows' multipliers nu_k (x_k = F(x_{k-1}, u_{k-1}), k >= 1) and their watchdog copy, fp64
  // in both precisions (correction form: eval_sweep)
  double nub[64][NX], wnub[64][NX];

  MR_HD Solver(const ProbParams<T>& P_, const Inst<T>& I_, WS<T> W_) : P(P_), I(I_), W(W_), N(P_.N) {}

  MR_HD int zf(int b) const { return b ? WF::Z1 : WF::Z0; }
  MR_HD int sf(int b) const { return b ? WF::S1 : WF::S0; }

  MR_HD void load_z(int k, int b, T* z) const {  // z[NZS]
    const int f = zf(b);
    for (int i = 0; i < NZS; ++i) z[i] = W(k, f + i);
    if (k == N) { z[11] = T(0); z[12] = T(0); z[13] = T(0); }
  }
  MR_HD void store_z(int k, int b, const T* z) const {
    const int f = zf(b);
    for (int i = 0; i < NZS; ++i) W(k, f + i) = z[i];
  }

  // one-sided row values d_j (slots 0..16) of stage k at z; returns row-active mask bits
  MR_HD void row_values(int k, const T* z, const Err<T>& e, T* d, int* act, Row<T>* rows) const {
    for (int r = 0; r < NROW; ++r) {
      make_row(P, I, k, r, z, &e, rows[r]);
      act[2 * r] = act[2 * r + 1] = rows[r].active;
      d[2 * r] = rows[r].c - rows[r].lo;
      d[2 * r + 1] = rows[r].hi - rows[r].c;
    }
    const int la = lane_active(P, k) ? 1 : 0;
    act[JL] = act[JL + 1] = la;
    act[JL + 2] = 0;  // (slot JL + 2 unused)
    lane_d(I, e.eC, z[14], d + JL);
  }

  // ---------------- initialisation (MPC.py:100-131) ----------------
  // u_init: optional strided [2][N] initial controls of this instance (element (r, k) at u_init[(r*N+k)*ustride])
  MR_HD void init(const double* u_init, int64_t ustride) {
    cur = 0;
    T z[NZS], zn[NX];
    for (int i = 0; i < NZS; ++i) z[i] = T(0);
    for (int i = 0; i < 6; ++i) z[i] = I.x0[i];
    z[7] = I.has_thr0 ? I.thr0 : T(0);
    z[8] = I.has_steer0 ? I.steer0 : T(0);
    T gmax = T(0);
    for (int k = 0; k <= N; ++k) {
      if (k < N) {
        if (u_init) { z[11] = T(u_init[(int64_t)k * ustride]); z[12] = T(u_init[(int64_t)(N + k) * ustride]); }
        else { z[11] = I.thr0; z[12] = I.steer0; }
        z[13] = P.Ts * P.v_max;  // S_i = s0 + i*Ts*v_max (MPC.py:127)
      } else {
        z[11] = z[12] = z[13] = T(0);
      }
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      z[14] = T(0);
      store_z(k, 0, z);
#ifdef MR_DEBUG_PRINT
      if (trace) printf("init k=%d vx=%g readback=%g X=%g S=%g\n", k, (double)z[3], (double)W(k, WF::Z0 + 3),
                        (double)z[0], (double)z[6]);
#endif
      // objective gradient for the gradient-based scaling
      T g[NZ];
      for (int i = 0; i < NZ; ++i) g[i] = T(0);
      stage_cost(P, I, k, z, e, T(1), g, (T*)nullptr);
      for (int i = 0; i < NZ; ++i) gmax = mr_max(gmax, mr_abs(g[i]));
      if (k < N) {
        faug<T, MODEL>(P, k, z, zn);
        for (int i = 0; i < NX; ++i) z[i] = zn[i];
      }
    }
    sc = gmax > T(0) ? mr_min(T(1), T(100) / gmax) : T(1);
    // slacks (IPOPT bound push), multipliers
    T th = T(0);
    for (int k = 0; k <= N; ++k) {
      load_z(k, 0, z);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      for (int j = 0; j < NI; ++j) {
        T push;
        if (j < JL) {
          const Row<T>& R = rows[j / 2];
          T bnd = (j & 1) ? mr_abs(R.hi) : mr_abs(R.lo);
          push = mr_min(T(1e-2) * mr_max(T(1), bnd), T(1e-2) * (R.hi - R.lo));
        } else {
          push = j < JL + 2 ? T(1e-2) * mr_max(T(1), I.max_err) : T(1e-2);
        }
        T s = act[j] ? mr_max(d[j], push) : T(1);
        W(k, WF::S0 + j) = s;
        W(k, WF::LAM + j) = act[j] ? T(1) : T(0);
        W(k, WF::DLAM + j) = T(0);
        if (act[j]) th += mr_abs(d[j] - s);
      }
      for (int i = 0; i < NX; ++i) { nub[k][i] = 0.0; W(k, WF::DNU + i) = T(0); }
    }
    mu = T(0.1);
    delta_last = T(0);
    alpha_p = alpha_d = T(0);
    theta_max = T(1e4) * mr_max(T(1), th);
    theta_min = T(1e-4) * mr_max(T(1), th);
    nfilt = 0;
  }

  // ---------------- sweep 1: evaluation, KKT error, stage QP data ----------------
  // Applies the lazy dual update of the previous accepted step first.
  MR_HD void eval_sweep(T mu_prev) {
    const T kappa_sigma = T(1e10);
    zeta = mr_sqrt(mu_prev);  // restoration proximity weight (IPOPT: resto_proximity_weight sqrt(mu))
    stat_max = pr_max = theta = T(0);
    slam_max = T(0);
    slam_min = T(1e30);
    nu1 = lam1 = fval = logs = T(0);
    const bool refk = !MR_KKT_RESTATED && !resto;  // the optimality error on the reference's NLP
    me = refk ? 6 * N + 7 : NX * (N + 1);
    mi = 0;
    if (refk)  // multipliers of the initial-state rows X_0 = state0, S_0 = s0 (lazy update, as nu_{k >= 1})
      for (int i = 0; i <= 6; ++i) {
        nub[0][i] += (double)alpha_p * (double)W(0, WF::DNU + i);
        nu1 += mr_abs(T(nub[0][i]));
      }
    T sref_b = T(0), sref_u[2] = {T(0), T(0)}, sref_u0[2] = {T(0), T(0)}, sref_w[2] = {T(0), T(0)};
    T z[NZS], znext[NZS], nun[NX];
    load_z(0, cur, z);
    for (int k = 0; k <= N; ++k) {
      // multipliers of x_{k+1} = F(x_k, u_k): lazy update nu += alpha_p * dnu (fp64), T copies for the
      // Hessian weights
      if (k < N) {
        for (int i = 0; i < NX; ++i) {
          const double v = nub[k + 1][i] + (double)alpha_p * (double)W(k + 1, WF::DNU + i);
          nub[k + 1][i] = v;
          nun[i] = T(v);
          if (!refk || i < 6) nu1 += mr_abs(nun[i]);
        }
        load_z(k + 1, cur, znext);
#ifdef MR_DEBUG_PRINT
        if (trace && mu_prev == T(0.1) && alpha_p == T(0))
          printf("eval k=%d cur=%d z.vx=%g znext.vx=%g znext.X=%g\n", k, cur, (double)z[3], (double)znext[3],
                 (double)znext[0]);
#endif
      }
      T H[NH], g0[NZ], g1[NZ], gl[NZ], st[NZ];
      double dd[NZ];
      for (int i = 0; i < NH; ++i) H[i] = T(0);
      for (int i = 0; i < NZ; ++i) { g0[i] = g1[i] = gl[i] = st[i] = T(0); dd[i] = 0.0; }
      if (k < N) {
        T Hd[36], J[48], fx[6];
        Dyn<T, MODEL>::fjh(P, z, z + NX, nun, fx, J, Hd);
        // vehicle-block Hessian over (x0..x5, u0, u1) -> stage indices
        const int map[8] = {0, 1, 2, 3, 4, 5, 11, 12};
        int q = 0;
        for (int a = 0; a < 8; ++a)
          for (int bb = a; bb < 8; ++bb, ++q) H[hidx(map[a], map[bb])] += Hd[q];
        // defect c_k = F(x_k, u_k) - x_{k+1}
        T c[NX];
        for (int i = 0; i < 6; ++i) c[i] = fx[i] - znext[i];
        c[6] = z[6] + z[13] - znext[6];
        c[7] = z[11] - znext[7];
        c[8] = z[12] - znext[8];
        c[9] = (k == 0 ? z[11] : z[9]) - znext[9];
        c[10] = (k == 0 ? z[12] : z[10]) - znext[10];
        if (resto) {  // relaxed vehicle rows F - x' - p + n (the S / previous-control rows are definitions)
          const T kappa_sigma = T(1e10);
          for (int i = 0; i < 6; ++i) {
            const T p = W(k, WF::CP + i), n = W(k, WF::CN + i);
            T vp = W(k, WF::CVP + i) + alpha_d * W(k, WF::CDVP + i);
            T vn = W(k, WF::CVN + i) + alpha_d * W(k, WF::CDVN + i);
            vp = mr_min(mr_max(vp, mu_prev / (kappa_sigma * p)), kappa_sigma * mu_prev / p);
            vn = mr_min(mr_max(vn, mu_prev / (kappa_sigma * n)), kappa_sigma * mu_prev / n);
            W(k, WF::CVP + i) = vp;
            W(k, WF::CVN + i) = vn;
            c[i] += n - p;
            const T ip = p / vp, in = n / vn, sw = T(1) / (ip + in);
            W(k, WF::CSW + i) = sw;
            // + nu_{k+1}: the Riccati right-hand side is in correction form (below), the disturbance's is not
            W(k, WF::CGW0 + i) = sw * rho * (in - ip) + nun[i];
            W(k, WF::CGW1 + i) = sw * (T(1) / vp - T(1) / vn);
            slam_max = mr_max(slam_max, mr_max(p * vp, n * vn));
            slam_min = mr_min(slam_min, mr_min(p * vp, n * vn));
            lam1 += mr_abs(vp) + mr_abs(vn);
            logs += mr_log(p) + mr_log(n);
            mi += 2;
            fval += rho * (p + n);
            stat_max = mr_max(stat_max, mr_max(mr_abs(rho - nun[i] - vp), mr_abs(rho + nun[i] - vn)));
          }
        }
        for (int i = 0; i < NX; ++i) {
          W(k, WF::C + i) = c[i];
          pr_max = mr_max(pr_max, mr_abs(c[i]));
          theta += mr_abs(c[i]);
        }
        for (int i = 0; i < 48; ++i) W(k, WF::J + i) = J[i];
        // the dynamics rows' terms of the Lagrangian gradient, dd = [A^T nu_{k+1} - nu_k ; B^T nu_{k+1}],
        // in fp64.  Correction form: the Riccati right-hand side is g0 + dd, so the sweeps solve for the
        // multiplier step dnu directly (forward: dnu = P dx + p); g0 + dd and the stationarity residual are
        // small near a solution and keep full relative precision.  (In fp32 the absolute form, nu_new =
        // P dx + p with p ~ nu ~ 1e3, cannot resolve the stationarity below the fp32 ulp of the costates,
        // 1.2e-4 at 1e3, above a 1e-4 tolerance.)
        apply_At(J, k, nub[k + 1], dd);
        apply_Bt(J, k, nub[k + 1], dd + NX);
      }
      if (k >= 1 || refk)  // (k = 0: nu_0 of the initial-state rows, zero unless refk)
        for (int i = 0; i < NX; ++i) dd[i] -= nub[k][i];
      // cost: the scaled objective, or the restoration phase's proximity term
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, true);
      if (resto) {
        T zr[NZS];
        for (int i = 0; i < NZS; ++i) zr[i] = W(k, WF::RZ + i);
        fval += prox_term(I, k, N, z, zr, zeta, gl, H);
      } else {
        fval += stage_cost(P, I, k, z, e, sc, gl, H);
      }
      for (int i = 0; i < NZ; ++i) { g0[i] += gl[i]; st[i] += gl[i]; }
      // inequality rows: lazy dual update, barrier terms
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      T lam_j[NI], sig_j[NI], c0_j[NI], c1_j[NI], y_j[NI];  // y: the row multiplier in W and grad L
      auto clip = [&](T v, T x) { return mr_min(mr_max(v, mu_prev / (kappa_sigma * x)), kappa_sigma * mu_prev / x); };
      for (int j = 0; j < NI; ++j) {
        lam_j[j] = sig_j[j] = c0_j[j] = c1_j[j] = y_j[j] = T(0);
        if (!act[j]) continue;
        T s = W(k, sf(cur) + j);
        T lam = clip(W(k, WF::LAM + j) + alpha_d * W(k, WF::DLAM + j), s);
        W(k, WF::LAM + j) = lam;
        lam_j[j] = lam;
        y_j[j] = lam;  // regular phase: the slack's bound dual is the row multiplier
        T rd = d[j] - s;
        T sl = s * lam;
        slam_max = mr_max(slam_max, sl);
        slam_min = mr_min(slam_min, sl);
        lam1 += mr_abs(lam);
        logs += mr_log(s);
        mi += 1;
        if (resto) {
          const T p = W(k, WF::RP + j), n = W(k, WF::RN + j);
          const T vp = clip(W(k, WF::RVP + j) + alpha_d * W(k, WF::RDVP + j), p);
          const T vn = clip(W(k, WF::RVN + j) + alpha_d * W(k, WF::RDVN + j), n);
          W(k, WF::RVP + j) = vp;
          W(k, WF::RVN + j) = vn;
          // restoration: the row's equality multiplier y is its own variable (IPOPT's y_d, started at 0,
          // stepped with the primal step size), tied to the slack's bound dual only through stationarity
          const T y = W(k, WF::RY + j) + alpha_p * W(k, WF::RDY + j);
          W(k, WF::RY + j) = y;
          y_j[j] = y;
#ifndef MR_RESTO_YSTAT
#define MR_RESTO_YSTAT 1
#endif
          if (MR_RESTO_YSTAT) stat_max = mr_max(stat_max, mr_abs(y - lam));
          rd = rd - p + n;
          slam_max = mr_max(slam_max, mr_max(p * vp, n * vn));
          slam_min = mr_min(slam_min, mr_min(p * vp, n * vn));
          lam1 += mr_abs(vp) + mr_abs(vn);
          logs += mr_log(p) + mr_log(n);
          mi += 2;
          fval += rho * (p + n);
          stat_max = mr_max(stat_max, mr_max(mr_abs(rho + y - vp), mr_abs(rho - y - vn)));
          row_cond_r(d[j], s, lam, p, n, vp, vn, rho, sig_j[j], c0_j[j], c1_j[j]);
        } else {
          row_cond(d[j], s, lam, sig_j[j], c0_j[j], c1_j[j]);
        }
        pr_max = mr_max(pr_max, mr_abs(rd));
        theta += mr_abs(rd);
      }
      for (int r = 0; r < NROW; ++r) {
        const Row<T>& R = rows[r];
        if (!R.active) continue;
        T sig_sum = T(0), gsc0 = T(0), gsc1 = T(0), lamdiff = T(0);
        for (int sd = 0; sd < 2; ++sd) {
          int j = 2 * r + sd;
          T sgn = sd == 0 ? T(1) : T(-1);
          sig_sum += sig_j[j];
          gsc0 += sgn * c0_j[j];
          gsc1 += sgn * c1_j[j];
          lamdiff += sgn * y_j[j];
        }
        for (int a = 0; a < R.n; ++a) {
          g0[R.idx[a]] += R.a[a] * gsc0;
          g1[R.idx[a]] += R.a[a] * gsc1;
          st[R.idx[a]] -= lamdiff * R.a[a];
          for (int bb = a; bb < R.n; ++bb) H[hidx(R.idx[a], R.idx[bb])] += sig_sum * R.a[a] * R.a[bb];
        }
      }
      if (lane_active(P, k)) {
        // hard lane rows e_C + m >= 0 (slot JL) and m - e_C >= 0 (JL+1), nonlinear in (X, Y, S)
        const int id3[3] = {0, 1, 6};
        const T sig_sum = sig_j[JL] + sig_j[JL + 1];
        const T gz0 = c0_j[JL] - c0_j[JL + 1], gz1 = c1_j[JL] - c1_j[JL + 1];
        const T lamdiff = y_j[JL] - y_j[JL + 1];
        int q = 0;
        for (int a = 0; a < 3; ++a) {
          g0[id3[a]] += e.gC[a] * gz0;
          g1[id3[a]] += e.gC[a] * gz1;
          st[id3[a]] -= lamdiff * e.gC[a];
          for (int bb = a; bb < 3; ++bb, ++q)
            H[hidx(id3[a], id3[bb])] += sig_sum * e.gC[a] * e.gC[bb] - lamdiff * e.hC[q];
        }
      }
      // stationarity: x-part for k >= 1, u-part for k < N
      if (refk) {  // of the reference's variables (States, S_hat, U), see MR_KKT_RESTATED
        T sti[NZ];
        for (int i = 0; i < NZ; ++i) sti[i] = T((double)st[i] + dd[i]);
        for (int i = 0; i < 6; ++i) stat_max = mr_max(stat_max, mr_abs(sti[i]));  // X_k (k = 0: + nu_0)
        const T b = k < N ? sti[13] : T(0);
        stat_max = mr_max(stat_max, mr_abs(sti[6] + sref_b - b));  // S_k
        sref_b = b;
        if (k >= 1) {  // U_{k-1} with its copy p_k; U_0 waits for the w copies
          for (int a = 0; a < 2; ++a) {
            const T u = sref_u[a] + sti[7 + a];
            if (k == 1) sref_u0[a] = u; else stat_max = mr_max(stat_max, mr_abs(u));
            sref_w[a] += sti[9 + a];
          }
        }
        if (k < N) { sref_u[0] = sti[11]; sref_u[1] = sti[12]; }
        if (k == N)
          for (int a = 0; a < 2; ++a) stat_max = mr_max(stat_max, mr_abs(sref_u0[a] + sref_w[a]));
      } else {
        for (int i = 0; i < NZ; ++i) {
          const T sti = T((double)st[i] + dd[i]);
          if (i < NX ? k >= 1 : k < N) stat_max = mr_max(stat_max, mr_abs(sti));
        }
      }
      for (int i = 0; i < NH; ++i) W(k, WF::H + i) = H[i];
      for (int i = 0; i < NZ; ++i) {
        W(k, WF::G0 + i) = T((double)g0[i] + dd[i]);
        W(k, WF::G1 + i) = g1[i];
        W(k, WF::GL + i) = gl[i];
      }
      // advance
      if (k < N)
        for (int i = 0; i < NZS; ++i) z[i] = znext[i];
    }
  }

  MR_HD T kkt_error(T m) const {
    const T smax = T(100);
    T sd = mr_max(smax, (nu1 + lam1) / T(me + (mi > 0 ? mi : 1))) / smax;
    T scm = mr_max(smax, lam1 / T(mi > 0 ? mi : 1)) / smax;
    T cerr = mr_max(mr_abs(slam_max - m), mr_abs(m - slam_min));
    if (mi == 0) cerr = T(0);
    return mr_max(mr_max(stat_max / sd, pr_max), cerr / scm);
  }

  // ---------------- sweep 2: Riccati factorisation (backward) ----------------
  MR_HD bool riccati(T delta) {
    T Pm[NP], p0[NX], p1[NX];
    {
      const int k = N;
      for (int i = 0; i < NX; ++i)
        for (int j = i; j < NX; ++j) Pm[pidx(i, j)] = W(k, WF::H + hidx(i, j)) + (i == j && delta_var(i) ? delta : T(0));
      for (int i = 0; i < NX; ++i) { p0[i] = W(k, WF::G0 + i); p1[i] = W(k, WF::G1 + i); }
      for (int i = 0; i < NP; ++i) W(k, WF::P + i) = Pm[i];
      for (int i = 0; i < NX; ++i) { W(k, WF::PV0 + i) = p0[i]; W(k, WF::PV1 + i) = p1[i]; }
    }
    for (int k = N - 1; k >= 0; --k) {
      T J[48], c[NX];
      for (int i = 0; i < 48; ++i) J[i] = W(k, WF::J + i);
      for (int i = 0; i < NX; ++i) c[i] = W(k, WF::C + i);
      if (resto) {  // the relaxed vehicle rows of x_{k+1} = F(x_k, u_k): minimise over the disturbance
        T sw[6], gw0[6], gw1[6];
        for (int i = 0; i < 6; ++i) { sw[i] = W(k, WF::CSW + i); gw0[i] = W(k, WF::CGW0 + i); gw1[i] = W(k, WF::CGW1 + i); }
        if (!noise_cond(Pm, p0, p1, sw, gw0, gw1)) return false;
      }
      // PA (11x11) column by column and PB (11x3)
      T PA[NX][NX], PB[NX][NU];
      for (int j = 0; j < NX; ++j) {
        T col[NX], e[NX];
        for (int i = 0; i < NX; ++i) e[i] = T(0);
        e[j] = T(1);
        apply_A(J, k, e, col);  // column j of A
        for (int i = 0; i < NX; ++i) {
          T acc = T(0);
          for (int l = 0; l < NX; ++l) acc += Pm[pidx(i, l)] * col[l];
          PA[i][j] = acc;
        }
      }
      for (int j = 0; j < NU; ++j) {
        T col[NX], e3[NU] = {T(0), T(0), T(0)};
        e3[j] = T(1);
        apply_B(J, k, e3, col);
        for (int i = 0; i < NX; ++i) {
          T acc = T(0);
          for (int l = 0; l < NX; ++l) acc += Pm[pidx(i, l)] * col[l];
          PB[i][j] = acc;
        }
      }
      // Rhat = R + B^T P B, Shat = S + B^T P A, Qhat = Q + A^T P A
      T Rh[6];
      {
        int q = 0;
        for (int a = 0; a < NU; ++a)
          for (int b = a; b < NU; ++b, ++q) {
            T colb[NX];
            for (int i = 0; i < NX; ++i) colb[i] = PB[i][b];
            T bt[NU];
            apply_Bt(J, k, colb, bt);
            Rh[q] = W(k, WF::H + hidx(NX + a, NX + b)) + bt[a] + (a == b && delta_var(NX + a) ? delta : T(0));
          }
      }
      T Sh[NU][NX];
      for (int j = 0; j < NX; ++j) {
        T colj[NX], bt[NU];
        for (int i = 0; i < NX; ++i) colj[i] = PA[i][j];
        apply_Bt(J, k, colj, bt);
        for (int a = 0; a < NU; ++a) Sh[a][j] = W(k, WF::H + hidx(j, NX + a)) + bt[a];
      }
      T L[6];
      if (!chol3(Rh, L)) return false;
      // vector parts
      T pc0[NX];
      for (int i = 0; i < NX; ++i) {
        T acc = p0[i];
        for (int l = 0; l < NX; ++l) acc += Pm[pidx(i, l)] * c[l];
        pc0[i] = acc;
      }
      T rh0[NU], rh1[NU];
      apply_Bt(J, k, pc0, rh0);
      apply_Bt(J, k, p1, rh1);
      for (int a = 0; a < NU; ++a) {
        rh0[a] += W(k, WF::G0 + NX + a);
        rh1[a] += W(k, WF::G1 + NX + a);
      }
      T k0[NU] = {-rh0[0], -rh0[1], -rh0[2]}, k1[NU] = {-rh1[0], -rh1[1], -rh1[2]};
      chol3_solve(L, k0);
      chol3_solve(L, k1);
      T Kg[NU][NX];
      for (int j = 0; j < NX; ++j) {
        T col[NU] = {-Sh[0][j], -Sh[1][j], -Sh[2][j]};
        chol3_solve(L, col);
        for (int a = 0; a < NU; ++a) Kg[a][j] = col[a];
      }
      // new P = Q + A^T P A + Sh^T K ; p = q + A^T pc + Sh^T kff
      T Pn[NP];
      for (int j = 0; j < NX; ++j) {
        T colj[NX], at[NX];
        for (int i = 0; i < NX; ++i) colj[i] = PA[i][j];
        apply_At(J, k, colj, at);  // column j of A^T P A
        for (int i = 0; i <= j; ++i) {
          T v = at[i] + W(k, WF::H + hidx(i, j)) + (i == j && delta_var(i) ? delta : T(0));
          for (int a = 0; a < NU; ++a) v += Sh[a][i] * Kg[a][j];
          Pn[pidx(i, j)] = v;
        }
      }
      T pn0[NX], pn1[NX], t0[NX], t1[NX];
      apply_At(J, k, pc0, t0);
      apply_At(J, k, p1, t1);
      for (int i = 0; i < NX; ++i) {
        T v0 = W(k, WF::G0 + i) + t0[i], v1 = W(k, WF::G1 + i) + t1[i];
        for (int a = 0; a < NU; ++a) { v0 += Sh[a][i] * k0[a]; v1 += Sh[a][i] * k1[a]; }
        pn0[i] = v0;
        pn1[i] = v1;
      }
      for (int a = 0; a < NU; ++a) {
        for (int j = 0; j < NX; ++j) W(k, WF::K + a * NX + j) = Kg[a][j];
        W(k, WF::K0 + a) = k0[a];
        W(k, WF::K1 + a) = k1[a];
      }
      for (int i = 0; i < NP; ++i) { Pm[i] = Pn[i]; W(k, WF::P + i) = Pn[i]; }
      for (int i = 0; i < NX; ++i) {
        p0[i] = pn0[i]; p1[i] = pn1[i];
        W(k, WF::PV0 + i) = pn0[i]; W(k, WF::PV1 + i) = pn1[i];
      }
    }
    return true;
  }

  // ---------------- sweep 3: forward substitution, slack/dual steps ----------------
  // fraction-to-boundary primal/dual step and the directional derivative of phi_mu
  MR_HD void forward(T& ap, T& ad, T& gphi) {
    const T tau = mr_max(T(0.99), T(1) - mu);
    ap = T(1);
    ad = T(1);
    gphi = T(0);
    T dx[NX];
    for (int i = 0; i < NX; ++i) dx[i] = T(0);
    if (!MR_KKT_RESTATED && !resto)  // the initial-state rows' multiplier step: stage 0's costate (dx_0 = 0)
      for (int i = 0; i < NX; ++i) W(0, WF::DNU + i) = W(0, WF::PV0 + i) + mu * W(0, WF::PV1 + i);
    T z[NZS];
    for (int k = 0; k <= N; ++k) {
      T dz[NZS];
      for (int i = 0; i < NX; ++i) dz[i] = dx[i];
      if (k < N) {
        for (int a = 0; a < NU; ++a) {
          T v = W(k, WF::K0 + a) + mu * W(k, WF::K1 + a);
          for (int j = 0; j < NX; ++j) v += W(k, WF::K + a * NX + j) * dx[j];
          dz[NX + a] = v;
        }
      } else {
        dz[11] = dz[12] = dz[13] = T(0);
      }
      for (int i = 0; i < NZ; ++i) gphi += W(k, WF::GL + i) * dz[i];
      // rows
      load_z(k, cur, z);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      T adz[NI];
      for (int r = 0; r < NROW; ++r) {
        T v = T(0);
        for (int a = 0; a < rows[r].n; ++a) v += rows[r].a[a] * dz[rows[r].idx[a]];
        adz[2 * r] = v;
        adz[2 * r + 1] = -v;
      }
      dz[14] = T(0);
      if (lane_active(P, k)) {
        const T gdz = e.gC[0] * dz[0] + e.gC[1] * dz[1] + e.gC[2] * dz[6];
        adz[JL] = gdz;
        adz[JL + 1] = -gdz;
        adz[JL + 2] = T(0);
      }
      for (int i = 0; i < NZS; ++i) W(k, WF::DZ + i) = dz[i];
      for (int j = 0; j < NI; ++j) {
        if (!act[j]) continue;
        T s = W(k, sf(cur) + j), lam = W(k, WF::LAM + j);
        T ds, dl;
        if (resto) {
          const T p = W(k, WF::RP + j), n = W(k, WF::RN + j), vp = W(k, WF::RVP + j), vn = W(k, WF::RVN + j);
          T dp, dn, dvp, dvn;
          row_steps_r(adz[j] + (d[j] - s - p + n), s, lam, p, n, vp, vn, rho, mu, ds, dp, dn, dl, dvp, dvn);
          W(k, WF::RDP + j) = dp;
          W(k, WF::RDN + j) = dn;
          W(k, WF::RDVP + j) = dvp;
          W(k, WF::RDVN + j) = dvn;
          W(k, WF::RDY + j) = lam + dl - W(k, WF::RY + j);  // eta - y
          gphi += (rho - mu / p) * dp + (rho - mu / n) * dn;
          if (dp < T(0)) ap = mr_min(ap, -tau * p / dp);
          if (dn < T(0)) ap = mr_min(ap, -tau * n / dn);
          if (dvp < T(0)) ad = mr_min(ad, -tau * vp / dvp);
          if (dvn < T(0)) ad = mr_min(ad, -tau * vn / dvn);
        } else {
          ds = adz[j] + (d[j] - s);
          dl = mu / s - lam - (lam / s) * ds;
        }
        W(k, WF::DS + j) = ds;
        W(k, WF::DLAM + j) = dl;
        gphi -= mu * ds / s;
        if (ds < T(0)) ap = mr_min(ap, -tau * s / ds);
        if (dl < T(0)) ad = mr_min(ad, -tau * lam / dl);
      }
      if (k < N) {
        T J[48], t[NX], tb[NX];
        for (int i = 0; i < 48; ++i) J[i] = W(k, WF::J + i);
        apply_A(J, k, dx, t);
        apply_B(J, k, dz + NX, tb);
        for (int i = 0; i < NX; ++i) dx[i] = t[i] + tb[i] + W(k, WF::C + i);
        if (resto) {  // + the disturbance of the relaxed vehicle rows, w = -M^-1 (nu_y + gw)
          T Pn[NP], sw[6], rhs[6], w[6];
          for (int i = 0; i < NP; ++i) Pn[i] = W(k + 1, WF::P + i);
          for (int i = 0; i < 6; ++i) {
            T v = W(k + 1, WF::PV0 + i) + mu * W(k + 1, WF::PV1 + i);
            for (int l = 0; l < NX; ++l) v += Pn[pidx(i, l)] * dx[l];
            rhs[i] = v + W(k, WF::CGW0 + i) + mu * W(k, WF::CGW1 + i);
            sw[i] = W(k, WF::CSW + i);
          }
          noise_step(Pn, sw, rhs, w);
          for (int i = 0; i < 6; ++i) {
            dx[i] += w[i];
            const T p = W(k, WF::CP + i), n = W(k, WF::CN + i), vp = W(k, WF::CVP + i), vn = W(k, WF::CVN + i);
            T dp, dn, dvp, dvn;
            dyn_steps_r(w[i], p, n, vp, vn, rho, mu, dp, dn, dvp, dvn);
            W(k, WF::CDP + i) = dp;
            W(k, WF::CDN + i) = dn;
            W(k, WF::CDVP + i) = dvp;
            W(k, WF::CDVN + i) = dvn;
            gphi += (rho - mu / p) * dp + (rho - mu / n) * dn;
            if (dp < T(0)) ap = mr_min(ap, -tau * p / dp);
            if (dn < T(0)) ap = mr_min(ap, -tau * n / dn);
            if (dvp < T(0)) ad = mr_min(ad, -tau * vp / dvp);
            if (dvn < T(0)) ad = mr_min(ad, -tau * vn / dvn);
          }
        }
        // multiplier step dnu_{k+1} = P_{k+1} dx_{k+1} + p_{k+1} (correction form, eval_sweep)
        for (int i = 0; i < NX; ++i) {
          T v = W(k + 1, WF::PV0 + i) + mu * W(k + 1, WF::PV1 + i);
          for (int l = 0; l < NX; ++l) v += W(k + 1, WF::P + pidx(i, l)) * dx[l];
          W(k + 1, WF::DNU + i) = v;  // correction form: the multiplier step itself
        }
      }
    }
  }

  // ---------------- sweep 4: line-search trial point ----------------
  // Writes the trial iterate into buffer 1-cur; returns false if a slack is not positive.
  MR_HD bool trial(T alpha, bool soc, T& th_t, T& ph_t) {
    const int nb = 1 - cur;
    th_t = T(0);
    T fv = T(0), lg = T(0), lgr = T(0), tho = T(0), fo = T(0);  // lgr, tho, fo: restoration phase only
    T z[NZS], zt[NZS], zpl[NZS], zroll[NX];
    bool ok = true;
    for (int k = 0; k <= N; ++k) {
      load_z(k, cur, z);
      for (int i = 0; i < NZS; ++i) zt[i] = z[i] + alpha * W(k, WF::DZ + i);
      if (k == 0)
        for (int i = 0; i < NX; ++i) zt[i] = z[i];  // x_0 fixed
      if (k == N) { zt[11] = zt[12] = zt[13] = T(0); }
      for (int i = 0; i < NZS; ++i) zpl[i] = zt[i];
      if (soc && k >= 1)
        for (int i = 0; i < NX; ++i) zt[i] = zroll[i];
      // rows: slack trial s + alpha ds (+ SOC shift d(z_soc) - d(z_plain))
      Err<T> e, ep;
      errors(I, zt[0], zt[1], zt[6], e, false);
      T d[NI], dp[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, zt, e, d, act, rows);
      if (soc) {
        errors(I, zpl[0], zpl[1], zpl[6], ep, false);
        int actp[NI];
        Row<T> rowsp[NROW];
        row_values(k, zpl, ep, dp, actp, rowsp);
      }
      T dyn = T(0);  // this stage's share of theta not from rows (the dynamics defect)
      for (int j = 0; j < NI; ++j) {
        if (!act[j]) continue;
        T st = W(k, sf(cur) + j) + alpha * W(k, WF::DS + j);
        if (soc) st += d[j] - dp[j];
        if (!(st > T(0))) ok = false;
        W(k, sf(nb) + j) = st;
        lg += mr_log(st > T(0) ? st : T(1));
        if (resto) {
          const T pt = W(k, WF::RP + j) + alpha * W(k, WF::RDP + j), nt = W(k, WF::RN + j) + alpha * W(k, WF::RDN + j);
          if (!(pt > T(0)) || !(nt > T(0))) ok = false;
          th_t += mr_abs(d[j] - st - pt + nt);
          tho += mr_abs(d[j] - st);
          lgr += mr_log(pt > T(0) ? pt : T(1)) + mr_log(nt > T(0) ? nt : T(1));
          fv += rho * (pt + nt);
        } else {
          th_t += mr_abs(d[j] - st);
        }
      }
      if (resto) {
        T zr[NZS];
        for (int i = 0; i < NZS; ++i) zr[i] = W(k, WF::RZ + i);
        fv += prox_term(I, k, N, zt, zr, zeta, (T*)nullptr, (T*)nullptr);
        fo += stage_cost(P, I, k, zt, e, sc, (T*)nullptr, (T*)nullptr);
      } else {
        fv += stage_cost(P, I, k, zt, e, sc, (T*)nullptr, (T*)nullptr);
      }
      if (k < N) {
        T xn[NX];
        faug<T, MODEL>(P, k, zt, xn);
        if (soc) {
          for (int i = 0; i < NX; ++i) zroll[i] = xn[i];
        } else {
          for (int i = 0; i < NX; ++i) {
            T xt = W(k + 1, zf(cur) + i) + alpha * W(k + 1, WF::DZ + i);
            T rel = T(0);
            if (resto && i < 6) {  // the relaxed vehicle rows
              const T pt = W(k, WF::CP + i) + alpha * W(k, WF::CDP + i), nt = W(k, WF::CN + i) + alpha * W(k, WF::CDN + i);
              if (!(pt > T(0)) || !(nt > T(0))) ok = false;
              rel = nt - pt;
              lgr += mr_log(pt > T(0) ? pt : T(1)) + mr_log(nt > T(0) ? nt : T(1));
              fv += rho * (pt + nt);
              tho += mr_abs(xn[i] - xt);
            }
            dyn += mr_abs(xn[i] - xt + rel);
            if (resto && i >= 6) tho += mr_abs(xn[i] - xt);
          }
        }
      }
      th_t += dyn;
      if (!resto) tho += dyn;
      store_z(k, nb, zt);
    }
    ph_t = fv - mu * (lg + lgr);
    if (resto) {  // the point measured as the original problem sees it (restoration exit test)
      tho_acc = tho;
      pho_acc = fo - mu_o * lg;
    }
    if (!(th_t == th_t) || !(ph_t == ph_t)) ok = false;
    return ok;
  }

  MR_HD bool filter_ok(T th, T ph) const {
    for (int i = 0; i < FMAX; ++i)
      if (i < nfilt && th >= filt_th[i] && ph >= filt_ph[i]) return false;
    return true;
  }
  MR_HD void filter_add(T th, T ph) {
    if (nfilt < FMAX) {
      filt_th[nfilt] = th;
      filt_ph[nfilt] = ph;
      nfilt++;
    } else {  // drop the oldest entry
      for (int i = 0; i < FMAX - 1; ++i) { filt_th[i] = filt_th[i + 1]; filt_ph[i] = filt_ph[i + 1]; }
      filt_th[FMAX - 1] = th;
      filt_ph[FMAX - 1] = ph;
    }
  }

  MR_HD T lane_violation() const {
    T v = T(0);
    if (!P.lane) return v;
    for (int k = 1; k <= N; ++k) v = mr_max(v, W(k, zf(cur) + 14));
    return v;
  }

  // Filter backtracking line search (Waechter & Biegler 2006; IPOPT's order of tests): alpha = a0,
  // a0/2, ... down to a_min, one second-order correction after the first rejected trial when it did
  // not decrease theta; acceptance = theta_max, then the switching / Armijo or sufficient-decrease
  // test against (th, ph, gphi), then the filter.  The accepted trial is in buffer 1-cur.  nls counts
  // the halvings (in/out).
  MR_HD bool backtrack(T a0, T ap, T th, T ph, T gphi, T a_min, T th_pow, T& alpha, bool& ftype, bool& rej_filter,
                       int& nls) {
    const T s_phi = T(2.3), delta_sw = T(1), eta = T(1e-4), g_th = T(1e-5), g_ph = T(1e-5);
    (void)ap;
    alpha = a0;
    const int nls0 = nls;
    // backtracking ends below a_min, or below 1e-30: a_min is 0 when theta is (and may flush to 0
    // in fp32), and halving alpha to 0 would never leave the loop
    while (alpha >= a_min && alpha >= T(1e-30)) {
      for (int pass = 0; pass < 2; ++pass) {
        bool soc = pass == 1;
        T th_t, ph_t;
        bool ok;
        MR_PROF(3, ok = trial(alpha, soc, th_t, ph_t));
        if (ok) ok = th_t <= theta_max;
        if (ok) {
          bool sw = gphi < T(0) && alpha * mr_exp(s_phi * mr_log(-gphi)) > delta_sw * th_pow;
          if (th <= theta_min && sw) {
            ok = ph_t <= ph + eta * alpha * gphi + T(1e-14) * mr_abs(ph);
            ftype = true;
          } else {
            ok = th_t <= (T(1) - g_th) * th || ph_t <= ph - g_ph * th + T(1e-14) * mr_abs(ph);
            ftype = false;
          }
        }
        // the filter last (IPOPT's order: theta_max, sufficient decrease, then the filter), so a
        // rejection by the filter itself is known for the reset heuristic
        if (ok && !filter_ok(th_t, ph_t)) { ok = false; rej_filter = true; }
        if (ok) return true;
        // second-order correction only after the first rejected trial with theta not decreased (not in
        // the restoration phase: its rows carry the relaxations p, n)
        if (!(nls == 0 && !soc && th_t >= th) || resto) break;
      }
      alpha *= T(0.5);
      nls++;
    }
    return false;
  }

  // watchdog snapshot of the current iterate (buffer cur, multipliers) and search direction
  MR_HD void wd_save() {
    for (int k = 0; k <= N; ++k) {
      for (int i = 0; i < NZS; ++i) { W(k, WF::WZ + i) = W(k, zf(cur) + i); W(k, WF::WDZ + i) = W(k, WF::DZ + i); }
      for (int j = 0; j < NI; ++j) {
        W(k, WF::WSL + j) = W(k, sf(cur) + j); W(k, WF::WLAM + j) = W(k, WF::LAM + j);
        W(k, WF::WDS + j) = W(k, WF::DS + j); W(k, WF::WDLAM + j) = W(k, WF::DLAM + j);
      }
      for (int i = 0; i < NX; ++i) { wnub[k][i] = nub[k][i]; W(k, WF::WDNU + i) = W(k, WF::DNU + i); }
    }
  }
  MR_HD void wd_restore() {
    for (int k = 0; k <= N; ++k) {
      for (int i = 0; i < NZS; ++i) { W(k, zf(cur) + i) = W(k, WF::WZ + i); W(k, WF::DZ + i) = W(k, WF::WDZ + i); }
      for (int j = 0; j < NI; ++j) {
        W(k, sf(cur) + j) = W(k, WF::WSL + j); W(k, WF::LAM + j) = W(k, WF::WLAM + j);
        W(k, WF::DS + j) = W(k, WF::WDS + j); W(k, WF::DLAM + j) = W(k, WF::WDLAM + j);
      }
      for (int i = 0; i < NX; ++i) { nub[k][i] = wnub[k][i]; W(k, WF::DNU + i) = W(k, WF::WDNU + i); }
    }
  }

  // ---------------- the restoration phase (IPOPT's l1 restoration, W&B 2006 sec. 3.3) ----------------
  // Entered when the filter line search finds no acceptable step at an infeasible point (pr_max > tol).
  // The restoration NLP relaxes every constraint of the reference NLP: the 6 vehicle dynamics rows of
  // each stage (F - x' - p + n = 0) and every inequality row (d(z) - s - p + n = 0); the definitional rows
  // of the restatement (S+ = S + dS, the previous-control copies) are not constraints of the reference:
  //   min rho sum (p + n) + zeta/2 sum D^2 (z - z_R)^2,  p, n >= 0,
  // rho = 1000, zeta = sqrt(mu), D = min(1, 1/|z_R|) on the reference's variables; solved by the same
  // IPM (eval / Riccati / forward / filter line search with its own filter and barrier parameter,
  // starting at max(mu, max violation)).  It returns to the original problem at the first accepted
  // step whose point reduces the original theta to <= 0.9 theta(z_R) and is acceptable to the original
  // filter (augmented with z_R's entry on entering).
  MR_HD void resto_enter(T th, T ph) {
    const T g_th = T(1e-5), g_ph = T(1e-5);
    filter_add((T(1) - g_th) * th, ph - g_ph * th);
    onfilt = nfilt;
    for (int i = 0; i < FMAX; ++i) { ofilt_th[i] = filt_th[i]; ofilt_ph[i] = filt_ph[i]; }
    mu_o = mu;
    th_entry = th;
    delta_last_o = delta_last;
    theta_max_o = theta_max;
    theta_min_o = theta_min;
    const T mu_r = mr_max(mu, pr_max);
    T th_rows = T(0);
    for (int k = 0; k <= N; ++k) {
      T z[NZS];
      load_z(k, cur, z);
      for (int i = 0; i < NZS; ++i) W(k, WF::RZ + i) = z[i];
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      for (int j = 0; j < NI; ++j) {
        T p = T(1), n = T(1);
        if (act[j]) {
          const T c = d[j] - W(k, sf(cur) + j);
          th_rows += mr_abs(c);
          resto_pn(c, mu_r, rho, p, n);
        }
        W(k, WF::RP + j) = p;
        W(k, WF::RN + j) = n;
        W(k, WF::RVP + j) = mu_r / p;
        W(k, WF::RVN + j) = mu_r / n;
        W(k, WF::RDP + j) = W(k, WF::RDN + j) = W(k, WF::RDVP + j) = W(k, WF::RDVN + j) = T(0);
        W(k, WF::RY + j) = W(k, WF::RDY + j) = T(0);  // the rows' equality multipliers start at 0
        W(k, WF::DLAM + j) = T(0);
#ifndef MR_RESTO_LAMINIT
#define MR_RESTO_LAMINIT 2
#endif
        if (act[j]) {
          if (MR_RESTO_LAMINIT == 1) W(k, WF::LAM + j) = mr_min(W(k, WF::LAM + j), rho);
          if (MR_RESTO_LAMINIT == 2) W(k, WF::LAM + j) = mu_r / W(k, sf(cur) + j);
        }
      }
      for (int i = 0; i < NX; ++i) { nub[k][i] = 0.0; W(k, WF::DNU + i) = T(0); }
      if (k < N)
        for (int i = 0; i < 6; ++i) {  // the vehicle rows start satisfied too (p - n = F - x')
          T p, n;
          const T c = W(k, WF::C + i);
          th_rows += mr_abs(c);
          resto_pn(c, mu_r, rho, p, n);
          W(k, WF::CP + i) = p;
          W(k, WF::CN + i) = n;
          W(k, WF::CVP + i) = mu_r / p;
          W(k, WF::CVN + i) = mu_r / n;
          W(k, WF::CDP + i) = W(k, WF::CDN + i) = W(k, WF::CDVP + i) = W(k, WF::CDVN + i) = T(0);
        }
    }
    alpha_p = alpha_d = T(0);
    mu = mu_r;
    resto = true;
    nfilt = 0;
    delta_last = T(0);
    const T th_r = mr_max(theta - th_rows, T(0));  // relaxed rows start satisfied: the definitional rows only
    theta_max = T(1e4) * mr_max(T(1), th_r);
    theta_min = T(1e-4) * mr_max(T(1), th_r);
  }
  MR_HD bool resto_done() const {  // the accepted restoration step's point, seen by the original problem
    if (!(tho_acc <= T(RESTO_KAPPA) * th_entry)) return false;
    for (int i = 0; i < FMAX; ++i)
      if (i < onfilt && tho_acc >= ofilt_th[i] && pho_acc >= ofilt_ph[i]) return false;
    return true;
  }
  MR_HD void resto_exit() {
    // bound multipliers: a Newton step for complementarity at the new point (mu/s), reset to 1 where it
    // changes them by more than bound_mult_reset_threshold; equality multipliers reset to 0
    // (constr_mult_reset_threshold = 0); IPOPT's barrier parameter, filter and perturbation state back
    for (int k = 0; k <= N; ++k) {
      for (int j = 0; j < NI; ++j) {
        const T s = W(k, sf(cur) + j), lam = W(k, WF::LAM + j) + alpha_d * W(k, WF::DLAM + j);
        T ln = mu_o / s;
        if (mr_abs(ln - lam) > T(RESTO_MULT_RESET)) ln = T(1);
        W(k, WF::LAM + j) = W(k, WF::LAM + j) == T(0) ? T(0) : ln;  // inactive slots stay 0
        W(k, WF::DLAM + j) = T(0);
      }
      for (int i = 0; i < NX; ++i) { nub[k][i] = 0.0; W(k, WF::DNU + i) = T(0); }
    }
    alpha_p = alpha_d = T(0);
    mu = mu_o;
    nfilt = onfilt;
    for (int i = 0; i < FMAX; ++i) { filt_th[i] = ofilt_th[i]; filt_ph[i] = ofilt_ph[i]; }
    theta_max = theta_max_o;
    theta_min = theta_min_o;
    delta_last = delta_last_o;
    resto = false;
  }

  // ---------------- the IPM loop ----------------
  MR_HD SolveOut solve() {
    const T kappa_eps = T(10), kappa_mu = T(0.2), theta_mu = T(1.5);
    const T mu_min = P.tol / T(10);
    const T s_phi = T(2.3), s_theta = T(1.1), delta_sw = T(1), eta = T(1e-4), g_th = T(1e-5), g_ph = T(1e-5);
    SolveOut out{2, 0, 0.0, 0.0};
    T mu_prev = mu;
    int acc_count = 0;
    int ls_fail = 0;  // consecutive iterations without an acceptable line-search step
    // IPOPT's filter reset heuristic (filter_reset_trigger = 5, max_filter_resets = 5): after this many
    // successive iterations whose line search had a trial point rejected by the filter, clear it
    int filt_rej_iters = 0, filt_resets = 0;
    // watchdog state and the reference values of the point where it started
    bool in_wd = false;
    int wd_short = 0, wd_trial = 0;
    T wd_th = T(0), wd_ph = T(0), wd_gphi = T(0), wd_ap = T(0), wd_ad = T(0), wd_amin = T(0), wd_thpow = T(0);
    int it = 0;
    for (it = 0;; ++it) {
      MR_PROF(0, eval_sweep(mu_prev));
      if (trace && it == 0 && trace_cap >= 100 + N + 1) {  // diagnostics: initial defects per stage
        for (int k = 0; k < N; ++k) {
          double* tr = trace + 8 * (100 + k);
          for (int i = 0; i < 6; ++i) tr[i] = (double)W(k, WF::C + i);
          tr[6] = (double)(mr_abs(W(k, WF::C + 6)) + mr_abs(W(k, WF::C + 7)) + mr_abs(W(k, WF::C + 8)) +
                           mr_abs(W(k, WF::C + 9)) + mr_abs(W(k, WF::C + 10)));
          tr[7] = (double)W(k + 1, zf(cur) + 3);
        }
      }
      T kkt = kkt_error(T(0));
      if (!(kkt == kkt) || !(fval == fval)) { out.status = 3; break; }
#ifdef MR_RESTO_DEBUG
      if (trace) printf("it %d resto %d kkt %.3e stat %.3e pr %.3e smax %.3e smin %.3e nu1 %.3e lam1 %.3e mi %d mu %.3e fval %.6e theta %.4e\n", it, (int)resto, (double)kkt, (double)stat_max, (double)pr_max, (double)slam_max, (double)slam_min, (double)nu1, (double)lam1, mi, (double)mu, (double)fval, (double)theta);
#endif
      if (resto) {
        // the restoration NLP converged at a point the original problem does not accept: IPOPT's
        // "converged to a point of local infeasibility"
        if (kkt <= P.tol) { out.status = MR_STATUS_INFEASIBLE; break; }
      } else {
        out.kkt = (double)kkt;
        out.obj = (double)(fval / sc);
        if (kkt <= P.tol) { out.status = 0; break; }
        if (P.acc_iter > 0) {
          acc_count = (kkt <= P.acc_tol) ? acc_count + 1 : 0;
          if (acc_count >= P.acc_iter) { out.status = 1; break; }
        }
      }
      if (it >= P.max_iter) { out.status = 2; break; }
      T mu_old = mu;
      while (kkt_error(mu) <= kappa_eps * mu && mu > mu_min) {
        T m1 = kappa_mu * mu, m2 = mr_exp(theta_mu * mr_log(mu));
        mu = mr_max(mu_min, mr_min(m1, m2));
      }
      if (mu != mu_old) {  // IPOPT resets its line search with a new barrier problem: filter and watchdog
        nfilt = 0;
        in_wd = false;
        wd_short = 0;
      }
      // inertia-corrected factorisation
      T delta = T(0);
      bool first = true, fact_ok = false;
      for (int tries = 0; tries < 60; ++tries) {
        bool rok;
        MR_PROF(1, rok = riccati(delta));
        if (rok) { fact_ok = true; break; }
        if (first) {
          delta = delta_last == T(0) ? T(1e-4) : mr_max(T(1e-20), delta_last / T(3));
          first = false;
        } else {
          delta *= (delta_last == T(0) ? T(100) : T(8));
        }
        if (delta > T(1e40)) break;
      }
      if (!fact_ok) { out.status = 3; break; }
      if (delta > T(0)) delta_last = delta;
      T ap, ad, gphi;
      MR_PROF(2, forward(ap, ad, gphi));
      // filter line search
      T th = theta, ph = fval - mu * logs;
      T th_pow = mr_exp(s_theta * mr_log(mr_max(th, T(1e-30))));
      T a_min;
      if (gphi < T(0)) {
        T t1 = g_ph * th / (-gphi);
        T t2 = delta_sw * th_pow / mr_exp(s_phi * mr_log(-gphi));
        // IPOPT (W&B 2006 eq. 23, CalculateAlphaMin): the switching term only at theta <= theta_min
        a_min = T(0.05) * mr_min(g_th, th <= theta_min ? mr_min(t1, t2) : t1);
      } else {
        a_min = T(0.05) * g_th;
      }
      if (resto) {  // a restoration-phase step: its own filter, no watchdog, no second-order correction
        T alpha = ap;
        bool ftype = false, rej_filter = false;
        int nls = 0;
        const bool accepted = backtrack(ap, ap, th, ph, gphi, a_min, th_pow, alpha, ftype, rej_filter, nls);
        if (!accepted) { out.status = 3; break; }  // IPOPT: restoration failed
        for (int k = 0; k <= N; ++k) {
          for (int j = 0; j < NI; ++j) {
            W(k, WF::RP + j) += alpha * W(k, WF::RDP + j);
            W(k, WF::RN + j) += alpha * W(k, WF::RDN + j);
          }
          if (k < N)
            for (int i = 0; i < 6; ++i) {
              W(k, WF::CP + i) += alpha * W(k, WF::CDP + i);
              W(k, WF::CN + i) += alpha * W(k, WF::CDN + i);
            }
        }
        if (!ftype) filter_add((T(1) - g_th) * th, ph - g_ph * th);
        if (trace && it < trace_cap) {
          double* tr = trace + 8 * it;
          tr[0] = (double)kkt; tr[1] = (double)mu; tr[2] = (double)alpha; tr[3] = (double)ad;
          tr[4] = (double)delta; tr[5] = (double)th; tr[6] = (double)tho_acc; tr[7] = -200.0 - nls;
        }
        alpha_p = alpha;
        alpha_d = ad;
        mu_prev = mu;
        cur = 1 - cur;
        if (resto_done()) {
          resto_exit();
          mu_prev = mu;
          in_wd = false;
          wd_short = 0;
          acc_count = 0;
          filt_rej_iters = 0;
        }
        continue;
      }
#if MR_WD_TRIGGER > 0
      // IPOPT's watchdog (watchdog_shortened_iter_trigger, watchdog_trial_iter_max): after that many
      // successive iterations whose accepted step was shorter than the fraction-to-boundary step, store
      // the iterate and its search direction and take full steps tentatively; they are judged against
      // the stored point, and after watchdog_trial_iter_max iterations without an acceptable one the
      // solver returns to the stored point and backtracks along its direction (skipping the full step)
      if (!in_wd && wd_short >= MR_WD_TRIGGER) {
        wd_save();
        wd_th = th; wd_ph = ph; wd_gphi = gphi; wd_ap = ap; wd_ad = ad; wd_amin = a_min; wd_thpow = th_pow;
        in_wd = true;
        wd_trial = 0;
      }
#endif
      T alpha = ap;
      bool accepted = false, ftype = false, rej_filter = false, take_anyway = false;
      int nls = 0;
      if (in_wd) {
        accepted = backtrack(ap, ap, wd_th, wd_ph, wd_gphi, ap, wd_thpow, alpha, ftype, rej_filter, nls);
        if (accepted) {
          in_wd = false;
          wd_short = 0;
          th = wd_th; ph = wd_ph;  // the filter entry is the watchdog point's (the acceptor's reference)
        } else if (++wd_trial <= MR_WD_TRIAL_MAX) {
          take_anyway = true;  // the full step is taken tentatively (its trial is in buffer 1-cur)
          alpha = ap;
          T th_t, ph_t;
          trial(alpha, false, th_t, ph_t);  // (re-)write the plain full-step point (the last trial may be a SOC)
        } else {
          // back to the watchdog point: its iterate and direction, a regular backtracking line search
          // that skips the full step
          wd_restore();
          in_wd = false;
          wd_short = 0;
          th = wd_th; ph = wd_ph; gphi = wd_gphi; ap = wd_ap; ad = wd_ad; a_min = wd_amin; th_pow = wd_thpow;
          alpha = T(0.5) * ap;
          nls = 1;
          accepted = backtrack(alpha, ap, th, ph, gphi, a_min, th_pow, alpha, ftype, rej_filter, nls);
        }
      } else {
        accepted = backtrack(ap, ap, th, ph, gphi, a_min, th_pow, alpha, ftype, rej_filter, nls);
      }
      // no acceptable step at an infeasible point: the restoration phase (from the next iteration on)
      if (!accepted && !take_anyway && pr_max > P.tol) {
        resto_enter(th, ph);
        mu_prev = mu;
        in_wd = false;
        wd_short = 0;
        acc_count = 0;
        if (trace && it < trace_cap) {
          double* tr = trace + 8 * it;
          tr[0] = (double)kkt; tr[1] = (double)mu; tr[2] = (double)0; tr[3] = (double)0;
          tr[4] = (double)delta; tr[5] = (double)th; tr[6] = (double)ph; tr[7] = -300.0;
        }
        continue;
      }
      // no acceptable step at a point feasible to the tolerance: the shortest tried step (see mr_wave.h)
      ls_fail = (accepted || take_anyway) ? 0 : ls_fail + 1;
      if (ls_fail >= MR_LS_FAIL_MAX) { out.status = 3; break; }
      if (!accepted && !take_anyway) {
        alpha = mr_min(mr_max(alpha, a_min), ap);
        T th_t, ph_t;
        trial(alpha, false, th_t, ph_t);
        ftype = false;
      }
      if (!take_anyway) wd_short = (accepted && alpha < ap) ? wd_short + 1 : 0;
#if MR_FILTER_RESET_TRIGGER > 0
      if (filt_resets < MR_MAX_FILTER_RESETS) {
        filt_rej_iters = rej_filter ? filt_rej_iters + 1 : 0;
        if (filt_rej_iters >= MR_FILTER_RESET_TRIGGER) {
          nfilt = 0;
          filt_resets++;
          filt_rej_iters = 0;
        }
      }
#endif
      if (!ftype && !take_anyway) filter_add((T(1) - g_th) * th, ph - g_ph * th);
      if (trace && it < trace_cap) {
        double* tr = trace + 8 * it;
        tr[0] = (double)kkt; tr[1] = (double)mu; tr[2] = (double)alpha; tr[3] = (double)ad;
        tr[4] = (double)delta; tr[5] = (double)th; tr[6] = (double)ph;
        tr[7] = (double)(take_anyway ? -100 - wd_trial : (accepted ? nls : -1));
      }
      alpha_p = alpha;
      alpha_d = ad;
      mu_prev = mu;
      cur = 1 - cur;
    }
    out.iters = it;
    if (trace && it < trace_cap) {  // final record: why the loop ended
      double* tr = trace + 8 * it;
      tr[0] = (double)out.kkt; tr[1] = (double)fval; tr[2] = (double)theta; tr[3] = (double)stat_max;
      tr[4] = (double)pr_max; tr[5] = (double)sc; tr[6] = (double)mu; tr[7] = 1000.0 + out.status;
    }
    return out;
  }
};

}  // namespace mr
