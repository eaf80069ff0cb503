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
#ifdef MR_RESTO_DEBUG
#include <cstdio>
#endif
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
    // IPOPT's inequality-row multipliers y_d (slot of the row: every box slot, the lower slot of a
    // two-sided row) and their step; the slack block's share of the inertia correction (delta_s):
    // HD = sum over rows of a a^T, GD = sum of a (d - s); the Cholesky factor of Q_uu (second-order
    // corrections re-solve on the stored factorisation)
    Y = K1 + NU, DY = Y + NI, HD = DY + NI, GD = HD + NH, LQ = GD + NZ,
    // second-order correction: the accumulated right-hand sides c_soc (dynamics rows) / r_soc (rows),
    // its direction and the vector part of its backward pass
    SC = LQ + 6, SR = SC + NX, SDZ = SR + NI, SDS = SDZ + NZS, SDLAM = SDS + NI, SDY = SDLAM + NI,
    SDNU = SDY + NI, SPV = SDNU + NX, SK0 = SPV + NX,
    // watchdog snapshot: the iterate and the search direction where the watchdog started
    WZ = SK0 + NU, WSL = WZ + NZS, WLAM = WSL + NI, WDZ = WLAM + NI, WDS = WDZ + NZS,
    WDLAM = WDS + NI, WDNU = WDLAM + NI, WY = WDNU + NX, WDY = WY + NI,
    // restoration phase: row relaxations p, n, their bound duals and steps, the reference point z_R
    RP = WDY + NI, RN = RP + NI, RVP = RN + NI, RVN = RVP + NI, RDP = RVN + NI, RDN = RDP + NI, RDVP = RDN + NI,
    RDVN = RDVP + NI, RY = RDVN + NI, RDY = RY + NI, RZ = RDY + NI,
    // restoration relaxations of the 6 vehicle dynamics rows of x_{k+1} = F(x_k, u_k) (stage k < N):
    // p, n, duals, steps, and the condensed disturbance weight / gradient for the Riccati sweep
    CP = RZ + NZS, CN = CP + 6, CVP = CN + 6, CVN = CVP + 6, CDP = CVN + 6, CDN = CDP + 6, CDVP = CDN + 6,
    CDVN = CDVP + 6, CSW = CDVN + 6, CGW0 = CSW + 6, CGW1 = CGW0 + 6,
    // the restoration phase's entry point (slacks, bound duals: the bound-multiplier update on return)
    // and IPOPT's stored acceptable iterate (returned if the line search fails at an almost feasible point)
    RS0 = CGW1 + 6, RLAM = RS0 + NI, AZ = RLAM + NI,
    ASL = AZ + NZS, ALAM = ASL + NI, AY = ALAM + NI,  // its slacks and multipliers
    NF = AY + NI
  };
};

MR_HD int hidx(int i, int j) {  // packed upper index of symmetric NZ x NZ
  if (i > j) { int t = i; i = j; j = t; }
  return i * NZ - (i * (i - 1)) / 2 + (j - i);
}
// Structural nonzeros of the stage Hessian (entries any stage, model, lane setting or phase can make
// nonzero): the vehicle dynamics block {X, Y, psi, vx, vy, r, thr, steer} (Dyn::fjh), the contouring / lag
// cost and lane rows on {X, Y, S} (stage_cost, lane rows), the rows' pairs (thr, p_thr), (steer, p_steer)
// (also the steering-rate cost), (w_thr, thr), (w_steer, steer), and the diagonal (row barriers,
// restoration proximity term).  48 of the 105 packed entries; the wave kernel's stage record stores only
// these (mr_wave.h RCF::H, compact index hcidx).
MR_HD constexpr bool h_dyn(int a) { return a <= 5 || a == 11 || a == 12; }
MR_HD constexpr bool h_xys(int a) { return a == 0 || a == 1 || a == 6; }
MR_HD constexpr bool h_struct(int i, int j) {
  return i == j || (h_dyn(i) && h_dyn(j)) || (h_xys(i) && h_xys(j)) || (i == 7 && j == 11) || (i == 11 && j == 7) ||
         (i == 8 && j == 12) || (i == 12 && j == 8) || (i == 9 && j == 11) || (i == 11 && j == 9) ||
         (i == 10 && j == 12) || (i == 12 && j == 10);
}
// compact index of the structural entry (i, j) (either order) in row-major upper order, -1 if not structural
MR_HD constexpr int hcidx(int i, int j) {
  if (i > j) { const int t = i; i = j; j = t; }
  if (!h_struct(i, j)) return -1;
  int n = 0;
  for (int a = 0; a < NZ; ++a)
    for (int b = a; b < NZ; ++b) {
      if (a == i && b == j) return n;
      if (h_struct(a, b)) ++n;
    }
  return -1;
}
constexpr int NHC = [] {
  int n = 0;
  for (int a = 0; a < NZ; ++a)
    for (int b = a; b < NZ; ++b) n += h_struct(a, b) ? 1 : 0;
  return n;
}();
static_assert(NHC == 48, "structural nonzeros of the stage Hessian");
// packed index (hidx) of the q-th structural entry: the compact store / gather loops run over q with
// compile-time table entries (no index search at run time)
struct HCTab {
  int p[NHC];
};
constexpr HCTab make_hctab() {
  HCTab t{};
  int n = 0;
  for (int a = 0; a < NZ; ++a)
    for (int b = a; b < NZ; ++b)
      if (h_struct(a, b)) t.p[n++] = a * NZ - (a * (a - 1)) / 2 + (b - a);
  return t;
}
constexpr HCTab HCT = make_hctab();
// packed index -> compact index (-1: structural zero), for run-time lookups (the Riccati's gather plan)
struct HCInv {
  int c[NH];
};
constexpr HCInv make_hcinv() {
  HCInv t{};
  for (int i = 0; i < NH; ++i) t.c[i] = -1;
  for (int q = 0; q < NHC; ++q) t.c[HCT.p[q]] = q;
  return t;
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

// IPOPT's bound_relax_factor (1e-8), capped by constr_viol_tol (1e-4): every inequality bound handed to
// IPOPT is relaxed by min(1e-4, 1e-8 max(1, |b|)) before the solve (equality rows are not).
template <typename T>
MR_HD T relax_amt(T b) { return mr_min(T(1e-4), T(1e-8) * mr_max(T(1), mr_abs(b))); }
// Opti's rows as IPOPT receives them (oracle.nlp.MPCProblem.ipopt_ineq): the throttle / steer boxes are
// two separate one-sided rows each (U < d_max, U > min: MPC.py:138-141), so the two slots of rows 0 / 1
// are independent IPOPT rows (own slack, own multiplier y, linear damping kappa_d); every other row is an
// opti.bounded row (MPC.py:134, :142-149, lane :135) -- ONE IPOPT slack s with two bounds, held here as
// the pair of distances t_L = s - lo (slot 2r) and t_U = hi - s (slot 2r + 1, moved rigidly with t_L:
// dt_U = -dt_L), its multiplier y in slot 2r.
MR_HD constexpr bool two_sided_row(int r) { return r >= 2; }
// slot j holds a row multiplier y (every slot of rows 0 / 1, the lower slot of a two-sided row)
MR_HD constexpr bool yslot(int j) { return j < 4 || (j < JL + 2 && (j & 1) == 0); }
// one-sided slots (the box rows): kappa_d damping
MR_HD constexpr bool oneslot(int j) { return j < 4; }
// sign of slot j's distance in IPOPT's slack: t = s - lo (lower, +1) or hi - s (upper, -1)
MR_HD constexpr int slot_sign(int j) { return (j & 1) ? -1 : 1; }

template <typename T>
MR_HD void make_row_raw(const ProbParams<T>& P, const Inst<T>& I, int k, int r, const T* z, const Err<T>* e,
                        Row<T>& R) {
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

template <typename T>
MR_HD void make_row(const ProbParams<T>& P, const Inst<T>& I, int k, int r, const T* z, const Err<T>* e, Row<T>& R) {
  make_row_raw(P, I, k, r, z, e, R);
  R.lo -= relax_amt(R.lo);
  R.hi += relax_amt(R.hi);
}

// Lane rows on states i = 1..N (the commented MPC.py:135): the reference's
// opti.bounded(-max_error, e_hat_C, max_error), one IPOPT row with two (relaxed) bounds, held as the
// distances e_C + m >= 0 (slot JL) and m - e_C >= 0 (JL + 1).  An infeasible start is the restoration
// phase's business (IPOPT's way), not an elastic reformulation.
template <typename T>
MR_HD bool lane_active(const ProbParams<T>& P, int k) { return P.lane && k >= 1; }

template <typename T>
MR_HD void lane_d(const Inst<T>& I, T eC, T t, T* d) {  // t: the unused slot 14 (0)
  const T m = I.max_err + relax_amt(I.max_err);
  d[0] = eC + m + t;
  d[1] = m - eC + t;
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
  double viol;  // IPOPT's unscaled constraint violation of the returned point (max-norm, mr_outputs.constr_viol)
};

#ifndef MR_F32_STALL
#define MR_F32_STALL 15  // fp32 stall exit at the mu floor (iterations; 0 = off), see Solver::solve
#endif
// The line-search filter.  IPOPT's is unbounded; here it holds FCAP = FMAX + 64 FOVF entries, more than a
// solve can add at max_iter <= 500 (at most one entry per iteration, the restoration phase's own filter
// separate), so it never drops one there (the round-4 build kept the last 32, which the C3 audits showed
// binding: 47-196 entries on long solves, profiles/r05_audit_C3_ipopt.jsonl).  The wave kernel keeps the
// first FMAX entries in LDS and the rest in the instance's cold fields (mr_wave.h CSF::FOV).
#ifndef MR_FMAX
#define MR_FMAX 32  // filter entries in LDS (wave kernel)
#endif
#ifndef MR_FOVF
#define MR_FOVF 8   // overflow fields of 64 entries each (wave kernel: cold fields per bank)
#endif
#ifndef MR_FILTER_RESET_TRIGGER
#define MR_FILTER_RESET_TRIGGER 5  // IPOPT filter_reset_trigger (0: heuristic off)
#endif
#ifndef MR_MAX_FILTER_RESETS
#define MR_MAX_FILTER_RESETS 5  // IPOPT max_filter_resets
#endif
// IPOPT's tiny-step rule (tiny_step_tol 10 eps of double, tiny_step_y_tol 1e-2): a step below 10 eps
// relative in every component of the reference's variables and slacks is taken without a line search and
// forces a barrier decrease (at the smallest mu: "search direction becomes too small", status 3).  The
// threshold is IPOPT's double epsilon in both precisions (an fp32 solve approximates IPOPT's fp64 one).
#ifndef MR_TINY_STEP
#define MR_TINY_STEP 0
#endif
// IPOPT's soft restoration phase (soft_resto_pderror_reduction_factor, max_soft_resto_iters)
#ifndef MR_SOFT_RESTO
#define MR_SOFT_RESTO 1
#endif
// IPOPT's least-square multipliers of the restoration problem at its start (RestoIterateInitializer with
// constr_mult_init_max 1000; Solver::ls_resto, mr_wave.h ls_resto): implemented, OFF by default -- on the
// product's restoration NLP (a two-sided row's two distances relaxed separately) the estimate
// is not IPOPT's, and with it on the host build's statuses on the C3 sample's 23 restoration instances agree
// with IPOPT's on 17 (wave) / 16 (scalar) against 19 / 18 off (profiles/r06_resto_rules.json); 0: the rows'
// multipliers start at 0
#ifndef MR_RESTO_LS_MULT
#define MR_RESTO_LS_MULT 0
#endif
constexpr double IP_SOFT_RESTO_FACTOR = 0.9999;
constexpr int IP_MAX_SOFT_RESTO = 10;
constexpr double IP_TINY_STEP_TOL = 10.0 * 2.220446049250313e-16;
#ifndef MR_LS_FAIL_MAX
#define MR_LS_FAIL_MAX 1000000
#endif
#ifndef MR_WD_TRIGGER
#define MR_WD_TRIGGER 10  // IPOPT watchdog_shortened_iter_trigger (0: watchdog off)
#endif
#ifndef MR_WD_TRIAL_MAX
#define MR_WD_TRIAL_MAX 3  // IPOPT watchdog_trial_iter_max
#endif
constexpr int FMAX = MR_FMAX, FOVF = MR_FOVF, FCAP = MR_FMAX + 64 * MR_FOVF;

// IPOPT 3.14 option defaults the solver restates beyond W&B 2006's line-search constants (the dense
// restatement oracle/ipopt.py implements the same rules; DESIGN.md §2 lists them)
constexpr double IP_KAPPA_D = 1e-5;                                                     // kappa_d
constexpr double IP_CONSTR_VIOL_TOL = 1e-4, IP_COMPL_INF_TOL = 1e-4, IP_DUAL_INF_TOL = 1.0;  // unscaled
constexpr double IP_ACC_DUAL_INF = 1e10, IP_ACC_CONSTR_VIOL = 1e-2, IP_ACC_COMPL = 1e-2;      // acceptable_*
constexpr double IP_OBJ_MAX_INC = 5.0, IP_KAPPA_SOC = 0.99, IP_MULT_INIT_MAX = 1000.0;
constexpr int IP_MAX_SOC = 4;
// backtracking halvings per line search (IPOPT has no cap; a_min > 0 ends it unless theta is exactly 0)
constexpr int IP_LS_MAX = 200;

// Reference values of a line search (FilterLSAcceptor's reference point: the current iterate, or the
// watchdog's stored point)
template <typename T>
struct LSRef {
  T th, ph, gphi, thpow;
};

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
  T filt_th[FCAP], filt_ph[FCAP];
  int nfilt;
  // iteration aggregates (eval sweep): dual infeasibility (stat), primal infeasibility of the equality
  // rows (pr_eq) and of the inequality rows' d - s (pr_rows; pr_max = both), the violation of the
  // inequality rows' bounds (viol), theta, complementarity extremes, multiplier 1-norms, f, barrier sums
  T stat_max, pr_max, pr_eq, viol_max, theta, slam_max, slam_min, nu1, y1, lam1, fval, logs, lins;
  T pr_o;  // restoration phase: the original problem's primal infeasibility at the current point
  int me, mi, mrow;
  T delta_it;  // the accepted factorisation's delta (slack block: delta_s = delta_x)
  bool rej_filter = false;
  // restoration phase: mode, its penalty and proximity weight, and the original problem's state
  bool resto = false;
  T rho = T(RESTO_RHO), zeta = T(0);
  T mu_o, th_entry, delta_last_o, theta_max_o, theta_min_o;
  T ofilt_th[FCAP], ofilt_ph[FCAP];
  int onfilt;
  T tho_acc, pho_acc;  // original theta / barrier objective of the last trial point (restoration)
  T fo_acc = T(0), fo_cur = T(0);  // original (scaled) objective of the last trial point / the current iterate
  bool have_acc = false;  // an acceptable iterate is stored (AZ)
  bool resto_first = false;  // the restoration phase's first iteration (no barrier update)
  double* trace = nullptr;  // optional per-iteration record (diagnostics)
  int trace_cap = 0;
  // the dynamics rows' multipliers nu_k (x_k = F(x_{k-1}, u_{k-1}), k >= 1) and their watchdog copy, fp64
  // in both precisions (correction form: eval_sweep)
  double nub[64][NX], wnub[64][NX], anub[64][NX];  // (anub: the stored acceptable point's)

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
  // the row gradient a (stage indices, values) of slot pair r (< NROW) or the lane rows (r == NROW)
  MR_HD int row_grad(int r, const Row<T>* rows, const Err<T>& e, int* idx, T* a) const {
    if (r < NROW) {
      for (int q = 0; q < rows[r].n; ++q) { idx[q] = rows[r].idx[q]; a[q] = rows[r].a[q]; }
      return rows[r].n;
    }
    idx[0] = 0; idx[1] = 1; idx[2] = 6;
    a[0] = e.gC[0]; a[1] = e.gC[1]; a[2] = e.gC[2];
    return 3;
  }
  // IPOPT's residual c - s of the row in slot j (a y-slot) from the slot distances: box lower d - t,
  // box upper -(d - t), two-sided d_L - t_L
  static MR_HD T ipopt_res(int j, const T* d, const T* t) { return T(slot_sign(j)) * (d[j] - t[j]); }

  // ---------------- initialisation (MPC.py:100-131; IPOPT's DefaultIterateInitializer) ----------------
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
    // slacks (IPOPT's slack_bound_push / slack_bound_frac 1e-2: a one-sided row's slack at least
    // 1e-2 max(1, |b|) inside its bound; a two-sided row's slack s projected into [lo + p_L, hi - p_U],
    // p = min(1e-2 max(1, |b|), 1e-2 (hi - lo))), bound duals 1, multipliers 0 (ls_init below)
    T th = T(0);
    for (int k = 0; k <= N; ++k) {
      load_z(k, 0, z);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      T t[NI];
      for (int j = 0; j < NI; ++j) t[j] = T(1);
      for (int r = 0; r <= NROW; ++r) {
        const int j0 = r < NROW ? 2 * r : JL;
        if (!act[j0]) continue;
        if (r < 2) {  // the box rows: two one-sided rows
          t[j0] = mr_max(d[j0], T(1e-2) * mr_max(T(1), mr_abs(rows[r].lo)));
          t[j0 + 1] = mr_max(d[j0 + 1], T(1e-2) * mr_max(T(1), mr_abs(rows[r].hi)));
        } else {
          T c, lo, hi;
          if (r < NROW) { c = rows[r].c; lo = rows[r].lo; hi = rows[r].hi; }
          else { hi = I.max_err + relax_amt(I.max_err); lo = -hi; c = e.eC; }
          const T rng = hi - lo;
          const T pL = mr_min(T(1e-2) * mr_max(T(1), mr_abs(lo)), T(1e-2) * rng);
          const T pU = mr_min(T(1e-2) * mr_max(T(1), mr_abs(hi)), T(1e-2) * rng);
          const T sv = mr_min(mr_max(c, lo + pL), hi - pU);
          t[j0] = sv - lo;
          t[j0 + 1] = hi - sv;
        }
      }
      for (int j = 0; j < NI; ++j) {
        W(k, WF::S0 + j) = t[j];
        W(k, WF::LAM + j) = act[j] ? T(1) : T(0);
        W(k, WF::DLAM + j) = T(0);
        W(k, WF::Y + j) = T(0);
        W(k, WF::DY + j) = T(0);
        if (act[j] && yslot(j)) th += mr_abs(d[j] - t[j]);
      }
      for (int i = 0; i < NX; ++i) { nub[k][i] = 0.0; W(k, WF::DNU + i) = T(0); }
    }
    mu = T(0.1);
    delta_last = T(0);
    alpha_p = alpha_d = T(0);
    theta_max = T(1e4) * mr_max(T(1), th);
    theta_min = T(1e-4) * mr_max(T(1), th);
    nfilt = 0;
    have_acc = false;
    ls_init();
  }

  // IPOPT's least-square multipliers (constr_mult_init_max 1000): y_c, y_d minimising
  // ||grad_x L||^2 + ||grad_s L||^2 at the initial point, i.e. the augmented system with W = 0,
  // D_x = D_s = I -- here the stage QP  min 1/2 sx' M sx + g' sx  s.t. the linearised dynamics with
  // c = 0, M = I on the reference's variables (delta_var) + sum over rows a a^T, g = grad f - sum a rs
  // (rs = v_L - v_U of the row), solved by the Riccati recursion: the costates are the dynamics rows'
  // multipliers, y_d = a.sx - rs.  Both are set to zero if one exceeds 1000 in magnitude.
  MR_HD void ls_init() {
    T z[NZS];
    for (int k = 0; k <= N; ++k) {
      load_z(k, 0, z);
      T H[NH], g[NZ], J[48];
      for (int i = 0; i < NH; ++i) H[i] = T(0);
      for (int i = 0; i < NZ; ++i) g[i] = T(0);
      for (int i = 0; i < 48; ++i) J[i] = T(0);
      if (k < N) {
        T Hd[36], fx[6], nz[NX];
        for (int i = 0; i < NX; ++i) nz[i] = T(0);
        Dyn<T, MODEL>::fjh(P, z, z + NX, nz, fx, J, Hd);
      }
      for (int i = 0; i < NZ; ++i)
        if (delta_var(i)) H[hidx(i, i)] = T(1);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      stage_cost(P, I, k, z, e, sc, g, (T*)nullptr);
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      for (int r = 0; r <= NROW; ++r) {
        const int j0 = r < NROW ? 2 * r : JL;
        if (!act[j0]) continue;
        int idx[3];
        T a[3];
        const int na = row_grad(r, rows, e, idx, a);
        // the IPOPT rows on this gradient: two one-sided (box) or one two-sided, each a a^T; rs = v_L - v_U
        const T nrow = r < 2 ? T(2) : T(1);
        const T rs = r < 2 ? (W(k, WF::LAM + j0) - W(k, WF::LAM + j0 + 1)) : T(0);
        for (int q = 0; q < na; ++q) {
          g[idx[q]] -= a[q] * rs;
          for (int q2 = q; q2 < na; ++q2) H[hidx(idx[q], idx[q2])] += nrow * a[q] * a[q2];
        }
      }
      for (int i = 0; i < NH; ++i) { W(k, WF::H + i) = H[i]; W(k, WF::HD + i) = T(0); }
      for (int i = 0; i < NZ; ++i) { W(k, WF::G0 + i) = g[i]; W(k, WF::G1 + i) = T(0); W(k, WF::GD + i) = T(0); }
      for (int i = 0; i < NX; ++i) W(k, WF::C + i) = T(0);
      for (int i = 0; i < 48; ++i) W(k, WF::J + i) = J[i];
    }
    if (!riccati(T(0))) return;  // (M is positive definite on the dynamics' null space; never fails)
    // forward: sx and the costates
    T dx[NX];
    for (int i = 0; i < NX; ++i) dx[i] = T(0);
    bool ok = true;
    const T big = T(IP_MULT_INIT_MAX);
    for (int k = 0; k <= N; ++k) {
      T dz[NZS];
      for (int i = 0; i < NZS; ++i) dz[i] = T(0);
      for (int i = 0; i < NX; ++i) dz[i] = dx[i];
      if (k < N)
        for (int a = 0; a < NU; ++a) {
          T v = W(k, WF::K0 + a);
          for (int j = 0; j < NX; ++j) v += W(k, WF::K + a * NX + j) * dx[j];
          dz[NX + a] = v;
        }
      // costate of stage k: the multipliers of x_k = F(x_{k-1}, u_{k-1}) (k >= 1) or of the
      // initial-state rows (k = 0)
      for (int i = 0; i < NX; ++i) {
        T v = W(k, WF::PV0 + i);
        for (int l = 0; l < NX; ++l) v += W(k, WF::P + pidx(i, l)) * dx[l];
        nub[k][i] = (double)v;
        if (i < 6 || (k == 0 && i == 6)) ok = ok && (mr_abs(v) <= big);
      }
      load_z(k, 0, z);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      for (int r = 0; r <= NROW; ++r) {
        const int j0 = r < NROW ? 2 * r : JL;
        if (!act[j0]) continue;
        int idx[3];
        T a[3];
        const int na = row_grad(r, rows, e, idx, a);
        T adz = T(0);
        for (int q = 0; q < na; ++q) adz += a[q] * dz[idx[q]];
        if (r < 2) {  // y_d = a.sx - rs per one-sided row: rs = v_L (lower) / -v_U (upper)
          const T y0 = adz - W(k, WF::LAM + j0), y1 = adz + W(k, WF::LAM + j0 + 1);
          W(k, WF::Y + j0) = y0;
          W(k, WF::Y + j0 + 1) = y1;
          ok = ok && mr_abs(y0) <= big && mr_abs(y1) <= big;
        } else {
          W(k, WF::Y + j0) = adz;
          ok = ok && mr_abs(adz) <= big;
        }
      }
      if (k < N) {
        T J[48], t[NX], tb[NX];
        for (int i = 0; i < 48; ++i) J[i] = W(k, WF::J + i);
        apply_A(J, k, dx, t);
        apply_B(J, k, dz + NX, tb);
        for (int i = 0; i < NX; ++i) dx[i] = t[i] + tb[i];
      }
    }
    if (!ok)
      for (int k = 0; k <= N; ++k) {
        for (int i = 0; i < NX; ++i) nub[k][i] = 0.0;
        for (int j = 0; j < NI; ++j) W(k, WF::Y + j) = T(0);
      }
  }

  // ---------------- sweep 1: evaluation, KKT error, stage QP data ----------------
  // Applies the lazy dual update of the previous accepted step first.
  MR_HD void eval_sweep(T mu_prev) {
    const T kappa_sigma = T(1e10);
    zeta = mr_sqrt(mu_prev);  // restoration proximity weight (IPOPT: resto_proximity_weight sqrt(mu))
    stat_max = pr_eq = pr_max = viol_max = theta = T(0);
    pr_o = T(0);
    slam_max = T(0);
    slam_min = T(1e30);
    nu1 = y1 = lam1 = fval = logs = lins = T(0);
    T pr_rows = T(0);
    const bool refk = !MR_KKT_RESTATED && !resto;  // the optimality error on the reference's NLP
    me = refk ? 6 * N + 7 : NX * (N + 1);
    mi = 0;
    mrow = 0;
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
      }
      T H[NH], g0[NZ], g1[NZ], gl[NZ], st[NZ], HD[NH], GD[NZ];
      double dd[NZ];
      for (int i = 0; i < NH; ++i) { H[i] = T(0); HD[i] = T(0); }
      for (int i = 0; i < NZ; ++i) { g0[i] = g1[i] = gl[i] = st[i] = GD[i] = T(0); dd[i] = 0.0; }
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
        for (int i = 0; i < NX; ++i) pr_o = mr_max(pr_o, mr_abs(c[i]));
        if (resto) {  // relaxed vehicle rows F - x' - p + n (the S / previous-control rows are definitions)
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
          pr_eq = mr_max(pr_eq, mr_abs(c[i]));
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
      T lam_j[NI], sig_j[NI], c0_j[NI], c1_j[NI], y_j[NI], t_j[NI];
      auto clip = [&](T v, T x) { return mr_min(mr_max(v, mu_prev / (kappa_sigma * x)), kappa_sigma * mu_prev / x); };
      for (int j = 0; j < NI; ++j) {
        lam_j[j] = sig_j[j] = c0_j[j] = c1_j[j] = y_j[j] = T(0);
        t_j[j] = T(1);
        if (!act[j]) continue;
        T s = W(k, sf(cur) + j);
        T lam = clip(W(k, WF::LAM + j) + alpha_d * W(k, WF::DLAM + j), s);
        W(k, WF::LAM + j) = lam;
        lam_j[j] = lam;
        t_j[j] = s;
        sig_j[j] = lam / s;
        T rd = d[j] - s;
        T sl = s * lam;
        slam_max = mr_max(slam_max, sl);
        slam_min = mr_min(slam_min, sl);
        lam1 += mr_abs(lam);
        logs += mr_log(s);
        mi += 1;
        viol_max = mr_max(viol_max, -d[j]);  // bound violation of the row value (max with 0: viol_max >= 0)
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
          stat_max = mr_max(stat_max, mr_abs(y - lam));
          if (yslot(j)) pr_o = mr_max(pr_o, mr_abs(rd));
          rd = rd - p + n;
          slam_max = mr_max(slam_max, mr_max(p * vp, n * vn));
          slam_min = mr_min(slam_min, mr_min(p * vp, n * vn));
          lam1 += mr_abs(vp) + mr_abs(vn);
          logs += mr_log(p) + mr_log(n);
          mi += 2;
          fval += rho * (p + n);
          stat_max = mr_max(stat_max, mr_max(mr_abs(rho + y - vp), mr_abs(rho - y - vn)));
          row_cond_r(d[j], s, lam, p, n, vp, vn, rho, sig_j[j], c0_j[j], c1_j[j]);
          pr_rows = mr_max(pr_rows, mr_abs(rd));
          theta += mr_abs(rd);
        } else if (yslot(j)) {  // an IPOPT row: its multiplier y_d (lazy update with the primal step)
          const T y = W(k, WF::Y + j) + alpha_p * W(k, WF::DY + j);
          W(k, WF::Y + j) = y;
          y_j[j] = y;
          y1 += mr_abs(y);
          mrow += 1;
          pr_rows = mr_max(pr_rows, mr_abs(rd));
          theta += mr_abs(rd);
        }
        if (oneslot(j)) lins += s;
      }
      if (resto) {
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
      } else {
        // IPOPT's rows condensed into the stage QP (slacks eliminated):  H += (Sigma_s) a a^T,
        // g += a (Sigma_s (d - s) + grad_s phi) with grad_s phi = -mu/t_L + mu/t_U (+-kappa_d mu for a
        // one-sided row) split into its mu-free (g0) and mu (g1) parts; the Lagrangian gradient gets
        // y a (L = f + y (d - s)), the slack's stationarity -y - v_L + v_U enters the dual infeasibility;
        // HD / GD: the inertia correction's slack shift delta_s = delta (delta a a^T, delta a (d - s))
        for (int r = 0; r <= NROW; ++r) {
          const int j0 = r < NROW ? 2 * r : JL, j1 = j0 + 1;
          if (!act[j0]) continue;
          int idx[3];
          T a[3];
          const int na = row_grad(r, rows, e, idx, a);
          T hs, gr0, gr1, ys, hdw, gdw;
          if (r < 2) {  // two one-sided rows: lower (c >= lo) in j0, upper (c <= hi) in j1
            hs = sig_j[j0] + sig_j[j1];
            gr0 = sig_j[j0] * (d[j0] - t_j[j0]) - sig_j[j1] * (d[j1] - t_j[j1]);
            gr1 = (-T(1) / t_j[j0] + T(IP_KAPPA_D)) + (T(1) / t_j[j1] - T(IP_KAPPA_D));
            ys = y_j[j0] + y_j[j1];
            hdw = T(2);
            gdw = (d[j0] - t_j[j0]) - (d[j1] - t_j[j1]);
            stat_max = mr_max(stat_max, mr_max(mr_abs(-y_j[j0] - lam_j[j0]), mr_abs(-y_j[j1] + lam_j[j1])));
          } else {  // one two-sided row: s = lo + t_L = hi - t_U
            hs = sig_j[j0] + sig_j[j1];
            gr0 = hs * (d[j0] - t_j[j0]);
            gr1 = -T(1) / t_j[j0] + T(1) / t_j[j1];
            ys = y_j[j0];
            hdw = T(1);
            gdw = d[j0] - t_j[j0];
            stat_max = mr_max(stat_max, mr_abs(-y_j[j0] - lam_j[j0] + lam_j[j1]));
          }
          for (int q = 0; q < na; ++q) {
            g0[idx[q]] += a[q] * gr0;
            g1[idx[q]] += a[q] * gr1;
            st[idx[q]] += ys * a[q];
            GD[idx[q]] += a[q] * gdw;
            for (int q2 = q; q2 < na; ++q2) {
              H[hidx(idx[q], idx[q2])] += hs * a[q] * a[q2];
              HD[hidx(idx[q], idx[q2])] += hdw * a[q] * a[q2];
            }
          }
          if (r == NROW) {  // the lane row's curvature y * grad^2 e_C in (X, Y, S)
            const int id3[3] = {0, 1, 6};
            int q = 0;
            for (int a3 = 0; a3 < 3; ++a3)
              for (int b3 = a3; b3 < 3; ++b3, ++q) H[hidx(id3[a3], id3[b3])] += ys * e.hC[q];
          }
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
      for (int i = 0; i < NH; ++i) { W(k, WF::H + i) = H[i]; W(k, WF::HD + i) = HD[i]; }
      for (int i = 0; i < NZ; ++i) {
        W(k, WF::G0 + i) = T((double)g0[i] + dd[i]);
        W(k, WF::G1 + i) = g1[i];
        W(k, WF::GL + i) = gl[i];
        W(k, WF::GD + i) = GD[i];
      }
      // advance
      if (k < N)
        for (int i = 0; i < NZS; ++i) z[i] = znext[i];
    }
    pr_max = mr_max(pr_eq, pr_rows);
  }

  // IPOPT's optimality-error scaling s_d (over y_c, y_d and the bound duals) and s_c
  MR_HD T s_d() const {
    return mr_max(T(100), (nu1 + y1 + lam1) / T(me + mrow + (mi > 0 ? mi : 1))) / T(100);
  }
  MR_HD T s_c() const { return mr_max(T(100), lam1 / T(mi > 0 ? mi : 1)) / T(100); }
  MR_HD T compl_err(T m) const {
    if (mi == 0) return T(0);
    return mr_max(mr_abs(slam_max - m), mr_abs(m - slam_min));
  }
  // curr_nlp_error: the primal part is the violation of the constraints (|c| and d(x) outside its bounds)
  MR_HD T nlp_error() const {
    const T pr = resto ? pr_max : mr_max(pr_eq, viol_max);
    return mr_max(mr_max(stat_max / s_d(), pr), compl_err(T(0)) / s_c());
  }
  // curr_barrier_error: the primal part is the infeasibility |c|, |d - s|
  MR_HD T barrier_error(T m) const { return mr_max(mr_max(stat_max / s_d(), pr_max), compl_err(m) / s_c()); }
  MR_HD T kkt_error(T m) const { return barrier_error(m); }
  // IPOPT's unscaled termination quantities: dual infeasibility, constraint violation, complementarity
  MR_HD bool converged(T err) const {
    if (!(err <= P.tol)) return false;
    return stat_max / sc <= T(IP_DUAL_INF_TOL) && mr_max(pr_eq, viol_max) <= T(IP_CONSTR_VIOL_TOL) &&
           compl_err(T(0)) / sc <= T(IP_COMPL_INF_TOL);
  }
  MR_HD bool acceptable(T err) const {
    if (!(err <= P.acc_tol)) return false;
    return stat_max / sc <= T(IP_ACC_DUAL_INF) && mr_max(pr_eq, viol_max) <= T(IP_ACC_CONSTR_VIOL) &&
           compl_err(T(0)) / sc <= T(IP_ACC_COMPL);
  }

  // ---------------- sweep 2: Riccati factorisation (backward) ----------------
  // Stage QP data H + delta (I_var + HD), g + delta GD: IPOPT's inertia correction shifts the reference's
  // variables (delta_x, delta_var) and the slacks (delta_s = delta_x; condensed: delta a a^T and
  // delta a (d - s) per row, HD / GD from the evaluation sweep).
  MR_HD bool riccati(T delta) {
    T Pm[NP], p0[NX], p1[NX];
    auto Hq = [&](int k, int i, int j) {
      return W(k, WF::H + hidx(i, j)) + delta * W(k, WF::HD + hidx(i, j)) + (i == j && delta_var(i) ? delta : T(0));
    };
    auto Gq = [&](int k, int i) { return W(k, WF::G0 + i) + delta * W(k, WF::GD + i); };
    {
      const int k = N;
      for (int i = 0; i < NX; ++i)
        for (int j = i; j < NX; ++j) Pm[pidx(i, j)] = Hq(k, i, j);
      for (int i = 0; i < NX; ++i) { p0[i] = Gq(k, i); p1[i] = W(k, WF::G1 + i); }
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
            Rh[q] = Hq(k, NX + a, NX + b) + bt[a];
          }
      }
      T Sh[NU][NX];
      for (int j = 0; j < NX; ++j) {
        T colj[NX], bt[NU];
        for (int i = 0; i < NX; ++i) colj[i] = PA[i][j];
        apply_Bt(J, k, colj, bt);
        for (int a = 0; a < NU; ++a) Sh[a][j] = Hq(k, j, NX + a) + bt[a];
      }
      T L[6];
      if (!chol3(Rh, L)) return false;
      for (int q = 0; q < 6; ++q) W(k, WF::LQ + q) = L[q];
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
        rh0[a] += Gq(k, NX + a);
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
          T v = at[i] + Hq(k, i, j);
          for (int a = 0; a < NU; ++a) v += Sh[a][i] * Kg[a][j];
          Pn[pidx(i, j)] = v;
        }
      }
      T pn0[NX], pn1[NX], t0[NX], t1[NX];
      apply_At(J, k, pc0, t0);
      apply_At(J, k, p1, t1);
      for (int i = 0; i < NX; ++i) {
        T v0 = Gq(k, i) + t0[i], v1 = W(k, WF::G1 + i) + t1[i];
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

  // ---------------- second-order correction: the vector part of the Riccati recursion ----------------
  // IPOPT's SOC solves the Newton system with the stored factorisation and the constraint right-hand
  // sides replaced by c_soc (dynamics rows, field SC) and r_soc (the rows' d - s, field SR): only the
  // stage gradients' row terms a D (d - s) (D = Sigma_s + delta) change, so the costate vector p and the
  // feed-forward k are recomputed (P, K, the Q_uu factor are the factorisation's):
  //   pc = P_{k+1} c_k + p_{k+1},  r = g_u + B^T pc,  k = -Q_uu^-1 r,  p_k = g_x + A^T pc + K^T r.
  MR_HD void soc_backward() {
    T pv[NX];
    const T dl = delta_it;
    // the stage gradient with the SOC's row residuals
    auto gsoc = [&](int k, T* g) {
      for (int i = 0; i < NZ; ++i) g[i] = W(k, WF::G0 + i) + mu * W(k, WF::G1 + i) + dl * W(k, WF::GD + i);
      T z[NZS];
      load_z(k, cur, z);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      for (int r = 0; r <= NROW; ++r) {
        const int j0 = r < NROW ? 2 * r : JL, j1 = j0 + 1;
        if (!act[j0]) continue;
        int idx[3];
        T a[3];
        const int na = row_grad(r, rows, e, idx, a);
        const T t0 = W(k, sf(cur) + j0), t1 = W(k, sf(cur) + j1);
        const T s0 = W(k, WF::LAM + j0) / t0, s1 = W(k, WF::LAM + j1) / t1;
        T dg;  // sum over the rows on a of D (r_soc - r)
        if (r < 2) {
          const T r0 = d[j0] - t0, r1 = -(d[j1] - t1);
          dg = (s0 + dl) * (W(k, WF::SR + j0) - r0) + (s1 + dl) * (W(k, WF::SR + j1) - r1);
        } else {
          dg = (s0 + s1 + dl) * (W(k, WF::SR + j0) - (d[j0] - t0));
        }
        for (int q = 0; q < na; ++q) g[idx[q]] += a[q] * dg;
      }
    };
    T g[NZ];
    gsoc(N, g);
    for (int i = 0; i < NX; ++i) { pv[i] = g[i]; W(N, WF::SPV + i) = pv[i]; }
    for (int k = N - 1; k >= 0; --k) {
      T J[48];
      for (int i = 0; i < 48; ++i) J[i] = W(k, WF::J + i);
      gsoc(k, g);
      T pc[NX];
      for (int i = 0; i < NX; ++i) {
        T acc = pv[i];
        for (int l = 0; l < NX; ++l) acc += W(k + 1, WF::P + pidx(i, l)) * W(k, WF::SC + l);
        pc[i] = acc;
      }
      T r[NU];
      apply_Bt(J, k, pc, r);
      for (int a = 0; a < NU; ++a) r[a] += g[NX + a];
      T L[6];
      for (int q = 0; q < 6; ++q) L[q] = W(k, WF::LQ + q);
      T kf[NU] = {-r[0], -r[1], -r[2]};
      chol3_solve(L, kf);
      for (int a = 0; a < NU; ++a) W(k, WF::SK0 + a) = kf[a];
      T at[NX];
      apply_At(J, k, pc, at);
      for (int i = 0; i < NX; ++i) {
        T v = g[i] + at[i];
        for (int a = 0; a < NU; ++a) v += W(k, WF::K + a * NX + i) * r[a];
        pv[i] = v;
        W(k, WF::SPV + i) = v;
      }
    }
  }

  // ---------------- sweep 3: forward substitution, slack/dual steps ----------------
  // The search direction from the factorisation (soc = false: fields DZ, DS, DLAM, DY, DNU) or of a
  // second-order correction (soc = true: the vector part SK0 / SPV and the right-hand sides SC / SR,
  // into SDZ, SDS, SDLAM, SDY, SDNU).  Returns the fraction-to-boundary primal / dual step sizes and the
  // directional derivative of the barrier objective (regular direction).
  MR_HD void forward(T& ap, T& ad, T& gphi, bool soc = false) {
    const T tau = mr_max(T(0.99), T(1) - mu);
    const T dl = delta_it, kd = T(IP_KAPPA_D);
    const int fDZ = soc ? WF::SDZ : WF::DZ, fDS = soc ? WF::SDS : WF::DS, fDL = soc ? WF::SDLAM : WF::DLAM,
              fDY = soc ? WF::SDY : WF::DY, fDN = soc ? WF::SDNU : WF::DNU;
    ap = T(1);
    ad = T(1);
    gphi = T(0);
    T dx[NX];
    for (int i = 0; i < NX; ++i) dx[i] = T(0);
    if (!MR_KKT_RESTATED && !resto)  // the initial-state rows' multiplier step: stage 0's costate (dx_0 = 0)
      for (int i = 0; i < NX; ++i)
        W(0, fDN + i) = soc ? W(0, WF::SPV + i) : W(0, WF::PV0 + i) + mu * W(0, WF::PV1 + i);
    T z[NZS];
    for (int k = 0; k <= N; ++k) {
      T dz[NZS];
      for (int i = 0; i < NX; ++i) dz[i] = dx[i];
      if (k < N) {
        for (int a = 0; a < NU; ++a) {
          T v = soc ? W(k, WF::SK0 + a) : W(k, WF::K0 + a) + mu * W(k, WF::K1 + a);
          for (int j = 0; j < NX; ++j) v += W(k, WF::K + a * NX + j) * dx[j];
          dz[NX + a] = v;
        }
      } else {
        dz[11] = dz[12] = dz[13] = T(0);
      }
      if (!soc)
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
      adz[JL] = adz[JL + 1] = adz[JL + 2] = T(0);
      if (lane_active(P, k)) {
        const T gdz = e.gC[0] * dz[0] + e.gC[1] * dz[1] + e.gC[2] * dz[6];
        adz[JL] = gdz;
        adz[JL + 1] = -gdz;
      }
      for (int i = 0; i < NZS; ++i) W(k, fDZ + i) = dz[i];
      if (resto) {
        for (int j = 0; j < NI; ++j) {
          if (!act[j]) continue;
          T s = W(k, sf(cur) + j), lam = W(k, WF::LAM + j);
          T ds, dlv;
          const T p = W(k, WF::RP + j), n = W(k, WF::RN + j), vp = W(k, WF::RVP + j), vn = W(k, WF::RVN + j);
          T dp, dn, dvp, dvn;
          row_steps_r(adz[j] + (d[j] - s - p + n), s, lam, p, n, vp, vn, rho, mu, ds, dp, dn, dlv, dvp, dvn);
          W(k, WF::RDP + j) = dp;
          W(k, WF::RDN + j) = dn;
          W(k, WF::RDVP + j) = dvp;
          W(k, WF::RDVN + j) = dvn;
          W(k, WF::RDY + j) = lam + dlv - W(k, WF::RY + j);  // eta - y
          gphi += (rho - mu / p) * dp + (rho - mu / n) * dn;
          if (dp < T(0)) ap = mr_min(ap, -tau * p / dp);
          if (dn < T(0)) ap = mr_min(ap, -tau * n / dn);
          if (dvp < T(0)) ad = mr_min(ad, -tau * vp / dvp);
          if (dvn < T(0)) ad = mr_min(ad, -tau * vn / dvn);
          W(k, WF::DS + j) = ds;
          W(k, WF::DLAM + j) = dlv;
          gphi -= mu * ds / s;
          if (ds < T(0)) ap = mr_min(ap, -tau * s / ds);
          if (dlv < T(0)) ad = mr_min(ad, -tau * lam / dlv);
        }
      } else {
        // IPOPT's rows: the slack step ds = a.dz + (d - s) of each row (r_soc for a correction), the
        // distance steps (upper distance of a two-sided row: -ds), the bound-dual steps
        // dv = mu/t - v - (v/t) dt, the multiplier step dy = (Sigma_s + delta) ds + grad_s phi - y
        T t[NI];
        for (int j = 0; j < NI; ++j) t[j] = act[j] ? W(k, sf(cur) + j) : T(1);
        for (int r = 0; r <= NROW; ++r) {
          const int j0 = r < NROW ? 2 * r : JL, j1 = j0 + 1;
          if (!act[j0]) continue;
          const T l0 = W(k, WF::LAM + j0), l1 = W(k, WF::LAM + j1);
          const T s0 = l0 / t[j0], s1 = l1 / t[j1];
          T dt0, dt1;
          if (r < 2) {
            const T R0 = soc ? W(k, WF::SR + j0) : d[j0] - t[j0];
            const T R1 = soc ? W(k, WF::SR + j1) : -(d[j1] - t[j1]);
            const T Ds0 = adz[j0] + R0, Ds1 = -adz[j1] + R1;  // IPOPT's slack steps of the two rows
            dt0 = Ds0;
            dt1 = -Ds1;
            W(k, fDY + j0) = (s0 + dl) * Ds0 - mu / t[j0] + kd * mu - W(k, WF::Y + j0);
            W(k, fDY + j1) = (s1 + dl) * Ds1 + mu / t[j1] - kd * mu - W(k, WF::Y + j1);
            if (!soc) gphi += kd * mu * (dt0 + dt1);
          } else {
            const T R0 = soc ? W(k, WF::SR + j0) : d[j0] - t[j0];
            const T Ds = adz[j0] + R0;
            dt0 = Ds;
            dt1 = -Ds;
            W(k, fDY + j0) = (s0 + s1 + dl) * Ds - mu / t[j0] + mu / t[j1] - W(k, WF::Y + j0);
            W(k, fDY + j1) = T(0);
          }
          const T dts[2] = {dt0, dt1};
          for (int sd = 0; sd < 2; ++sd) {
            const int j = j0 + sd;
            const T lam = sd ? l1 : l0, dtj = dts[sd];
            const T dlv = mu / t[j] - lam - (lam / t[j]) * dtj;
            W(k, fDS + j) = dtj;
            W(k, fDL + j) = dlv;
            if (!soc) gphi -= mu * dtj / t[j];
            if (dtj < T(0)) ap = mr_min(ap, -tau * t[j] / dtj);
            if (dlv < T(0)) ad = mr_min(ad, -tau * lam / dlv);
          }
        }
      }
      if (k < N) {
        T J[48], tt[NX], tb[NX];
        for (int i = 0; i < 48; ++i) J[i] = W(k, WF::J + i);
        apply_A(J, k, dx, tt);
        apply_B(J, k, dz + NX, tb);
        for (int i = 0; i < NX; ++i) dx[i] = tt[i] + tb[i] + (soc ? W(k, WF::SC + i) : W(k, WF::C + i));
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
          T v = soc ? W(k + 1, WF::SPV + i) : W(k + 1, WF::PV0 + i) + mu * W(k + 1, WF::PV1 + i);
          for (int l = 0; l < NX; ++l) v += W(k + 1, WF::P + pidx(i, l)) * dx[l];
          W(k + 1, fDN + i) = v;  // correction form: the multiplier step itself
        }
      }
    }
  }
  // the accepted second-order correction becomes the iteration's search direction
  MR_HD void soc_commit() {
    for (int k = 0; k <= N; ++k) {
      for (int i = 0; i < NZS; ++i) W(k, WF::DZ + i) = W(k, WF::SDZ + i);
      for (int j = 0; j < NI; ++j) {
        W(k, WF::DS + j) = W(k, WF::SDS + j);
        W(k, WF::DLAM + j) = W(k, WF::SDLAM + j);
        W(k, WF::DY + j) = W(k, WF::SDY + j);
      }
      for (int i = 0; i < NX; ++i) W(k, WF::DNU + i) = W(k, WF::SDNU + i);
    }
  }

  // ---------------- sweep 4: line-search trial point ----------------
  // Writes the trial iterate (along the direction, or the SOC direction) into buffer 1-cur; returns
  // false if a slack is not positive or a value is not finite.  acc >= 0: accumulate the trial's
  // constraint values into the second-order correction's right-hand sides, SC = acc SC + c(trial),
  // SR = acc SR + (d - s)(trial) (IPOPT's c_soc update).
  MR_HD bool trial(T alpha, bool soc, T& th_t, T& ph_t, T acc = T(-1)) {
    const int nb = 1 - cur;
    const int fDZ = soc ? WF::SDZ : WF::DZ, fDS = soc ? WF::SDS : WF::DS;
    th_t = T(0);
    T fv = T(0), lg = T(0), lgr = T(0), tho = T(0), fo = T(0), lin = T(0);  // lgr, tho, fo: restoration only
    T z[NZS], zt[NZS];
    bool ok = true;
    for (int k = 0; k <= N; ++k) {
      load_z(k, cur, z);
      for (int i = 0; i < NZS; ++i) zt[i] = z[i] + alpha * W(k, fDZ + i);
      if (k == 0)
        for (int i = 0; i < NX; ++i) zt[i] = z[i];  // x_0 fixed
      if (k == N) { zt[11] = zt[12] = zt[13] = T(0); }
      Err<T> e;
      errors(I, zt[0], zt[1], zt[6], e, false);
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, zt, e, d, act, rows);
      T stv[NI];
      for (int j = 0; j < NI; ++j) {
        stv[j] = T(1);
        if (!act[j]) continue;
        T st = W(k, sf(cur) + j) + alpha * W(k, fDS + j);
        if (!(st > T(0))) ok = false;
        stv[j] = st;
        W(k, sf(nb) + j) = st;
        lg += mr_log(st > T(0) ? st : T(1));
        if (oneslot(j)) lin += st;
        if (resto) {
          const T pt = W(k, WF::RP + j) + alpha * W(k, WF::RDP + j), nt = W(k, WF::RN + j) + alpha * W(k, WF::RDN + j);
          if (!(pt > T(0)) || !(nt > T(0))) ok = false;
          th_t += mr_abs(d[j] - st - pt + nt);
          if (yslot(j)) tho += mr_abs(d[j] - st);
          lgr += mr_log(pt > T(0) ? pt : T(1)) + mr_log(nt > T(0) ? nt : T(1));
          fv += rho * (pt + nt);
        } else if (yslot(j)) {
          th_t += mr_abs(d[j] - st);
          if (acc >= T(0)) W(k, WF::SR + j) = acc * W(k, WF::SR + j) + T(slot_sign(j)) * (d[j] - st);
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
        for (int i = 0; i < NX; ++i) {
          T xt = W(k + 1, zf(cur) + i) + alpha * W(k + 1, fDZ + i);
          T rel = T(0);
          if (resto && i < 6) {  // the relaxed vehicle rows
            const T pt = W(k, WF::CP + i) + alpha * W(k, WF::CDP + i), nt = W(k, WF::CN + i) + alpha * W(k, WF::CDN + i);
            if (!(pt > T(0)) || !(nt > T(0))) ok = false;
            rel = nt - pt;
            lgr += mr_log(pt > T(0) ? pt : T(1)) + mr_log(nt > T(0) ? nt : T(1));
            fv += rho * (pt + nt);
          }
          th_t += mr_abs(xn[i] - xt + rel);
          tho += mr_abs(xn[i] - xt);
          if (acc >= T(0) && !resto) W(k, WF::SC + i) = acc * W(k, WF::SC + i) + (xn[i] - xt);
        }
      }
      store_z(k, nb, zt);
    }
    const T kdm = T(IP_KAPPA_D) * mu;
    ph_t = fv - mu * (lg + lgr) + kdm * lin;
    if (resto) {  // the point measured as the original problem sees it (restoration exit test)
      tho_acc = tho;
      fo_acc = fo;
      pho_acc = fo - mu_o * lg + T(IP_KAPPA_D) * mu_o * lin;
    }
    if (!(th_t == th_t) || !(ph_t == ph_t)) ok = false;
    return ok;
  }

  MR_HD bool filter_ok(T th, T ph) const {
    for (int i = 0; i < nfilt; ++i)
      if (th >= filt_th[i] && ph >= filt_ph[i]) return false;
    return true;
  }
  MR_HD void filter_add(T th, T ph) {
    const T g_th = T(1e-5), g_ph = T(1e-5);
    const T a = (T(1) - g_th) * th, b = ph - g_ph * th;
    if (nfilt < FCAP) {  // (full -- beyond max_iter 500 -- the entry is dropped, as in the wave kernel)
      filt_th[nfilt] = a;
      filt_ph[nfilt] = b;
      nfilt++;
    }
  }

  MR_HD T lane_violation() const {
    T v = T(0);
    if (!P.lane) return v;
    for (int k = 1; k <= N; ++k) v = mr_max(v, W(k, zf(cur) + 14));
    return v;
  }

  // FilterLSAcceptor's tests (IPOPT: Compare_le with 10 eps |reference|, obj_max_inc 5)
  static MR_HD bool cmp_le(T lhs, T rhs, T bas) { return lhs - rhs <= T(10) * mr_eps<T>() * mr_abs(bas); }
  MR_HD bool is_ftype(T a_test, const LSRef<T>& r) const {
    return r.gphi < T(0) && a_test * mr_exp(T(2.3) * mr_log(-r.gphi)) > r.thpow;
  }
  MR_HD bool armijo(T ph_t, T a_test, const LSRef<T>& r) const {
    return cmp_le(ph_t - r.ph, T(1e-4) * a_test * r.gphi, r.ph);
  }
  MR_HD bool acc_to_iterate(T th_t, T ph_t, const LSRef<T>& r) const {
    if (ph_t > r.ph) {
      const T bas = mr_abs(r.ph) > T(10) ? mr_log(mr_abs(r.ph)) / mr_log(T(10)) : T(1);
      if (mr_log(ph_t - r.ph) / mr_log(T(10)) > T(IP_OBJ_MAX_INC) + bas) return false;
    }
    const T g = T(1e-5);
    return cmp_le(th_t, (T(1) - g) * r.th, r.th) || cmp_le(ph_t - r.ph, -g * r.th, r.ph);
  }
  MR_HD bool acceptable_point(T th_t, T ph_t, T a_test, const LSRef<T>& r) {
    if (!(th_t <= theta_max)) return false;
    bool ok;
    if (a_test > T(0) && is_ftype(a_test, r) && r.th <= theta_min) ok = armijo(ph_t, a_test, r);
    else ok = acc_to_iterate(th_t, ph_t, r);
    if (!ok) return false;
    if (!filter_ok(th_t, ph_t)) { rej_filter = true; return false; }
    return true;
  }
  MR_HD T alpha_min_of(T th, T gphi) const {
    T a = T(1e-5);
    if (gphi < T(0)) {
      a = mr_min(a, T(1e-5) * th / (-gphi));
      if (th <= theta_min) a = mr_min(a, mr_exp(T(1.1) * mr_log(mr_max(th, T(1e-300)))) / mr_exp(T(2.3) * mr_log(-gphi)));
    }
    return T(0.05) * a;
  }

  // TrySecondOrderCorrection: up to max_soc linear corrections on the stored factorisation, while
  // theta falls by kappa_soc; the first trial point (alpha a_trial, theta th_trial) is in buffer 1-cur.
  // On success the SOC direction is the iteration's (soc_commit) and its trial point is in 1-cur.
  MR_HD bool try_soc(T a_trial, T th_trial, T a_test, const LSRef<T>& ref, T& alpha, T& ph_acc) {
    // c_soc = c(x_k), r_soc = (d - s)(x_k); then c_soc = a c_soc + c(trial)
    for (int k = 0; k <= N; ++k) {
      for (int i = 0; i < NX; ++i) W(k, WF::SC + i) = k < N ? W(k, WF::C + i) : T(0);
      T z[NZS];
      load_z(k, cur, z);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI], t[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      for (int j = 0; j < NI; ++j) {
        t[j] = act[j] ? W(k, sf(cur) + j) : T(1);
        W(k, WF::SR + j) = (act[j] && yslot(j)) ? T(slot_sign(j)) * (d[j] - t[j]) : T(0);
      }
    }
    T a_soc = a_trial, th_old = T(0), dum, dum2;
    bool plain = true;  // the trial point to accumulate: the plain first trial, then each SOC trial
    for (int count = 0; count < IP_MAX_SOC; ++count) {
      if (count > 0 && !(th_trial <= T(IP_KAPPA_SOC) * th_old)) break;
      th_old = th_trial;
      // accumulate the last trial point's constraint values (re-evaluated at a_soc along its direction)
      trial(a_soc, !plain, dum, dum2, a_soc);
      soc_backward();
      T ap_s, ad_s, gd;
      forward(ap_s, ad_s, gd, true);
      T th_t, ph_t;
      const bool fin = trial(ap_s, true, th_t, ph_t);
      plain = false;
      a_soc = ap_s;
      if (!fin) break;
      if (acceptable_point(th_t, ph_t, a_test, ref)) {
        alpha = ap_s;
        ph_acc = ph_t;
        soc_commit();
        return true;
      }
      th_trial = th_t;
    }
    return false;
  }

  // DoBacktrackingLineSearch: alpha = a_max, a_max/2, ... while alpha > a_min (the first trial always;
  // skip_first: from a_max/2); in the watchdog one trial point only, judged at the watchdog's step size;
  // a second-order correction after the first trial when it did not decrease theta.  The accepted
  // point is in buffer 1-cur.
  MR_HD bool backtrack(T a_max, bool skip_first, bool in_wd, T wd_atest, const LSRef<T>& ref, T a_min, T& alpha,
                       T& a_test, T& ph_acc, int& nls, bool& soc_taken) {
    alpha = skip_first ? T(0.5) * a_max : a_max;
    nls = skip_first ? 1 : 0;
    soc_taken = false;
    for (int n = 0; n < IP_LS_MAX; ++n) {
      if (!(alpha > a_min || n == 0)) break;
      a_test = in_wd ? wd_atest : alpha;
      T th_t, ph_t;
      bool fin;
      MR_PROF(3, fin = trial(alpha, false, th_t, ph_t));
      if (fin && acceptable_point(th_t, ph_t, a_test, ref)) { ph_acc = ph_t; return true; }
      if (in_wd) break;
      if (fin && alpha == a_max && !skip_first && theta <= th_t && !resto) {
        T as, pa;
        if (try_soc(alpha, th_t, a_test, ref, as, pa)) {
          alpha = as;
          ph_acc = pa;
          soc_taken = true;
          return true;
        }
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
        W(k, WF::WY + j) = W(k, WF::Y + j); W(k, WF::WDY + j) = W(k, WF::DY + j);
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
        W(k, WF::Y + j) = W(k, WF::WY + j); W(k, WF::DY + j) = W(k, WF::WDY + j);
      }
      for (int i = 0; i < NX; ++i) { nub[k][i] = wnub[k][i]; W(k, WF::DNU + i) = W(k, WF::WDNU + i); }
    }
  }
  double acc_kkt = 0.0, acc_obj = 0.0, acc_viol = 0.0;  // the stored acceptable point's measures
  // IPOPT's backup acceptable iterate (RestoreAcceptablePoint): the whole iterate -- primal part, slacks,
  // bound duals, row multipliers y_d and the dynamics multipliers -- so a solve that returns it returns
  // multipliers that belong to it
  MR_HD void acc_save() {
    for (int k = 0; k <= N; ++k) {
      for (int i = 0; i < NZS; ++i) W(k, WF::AZ + i) = W(k, zf(cur) + i);
      for (int j = 0; j < NI; ++j) {
        W(k, WF::ASL + j) = W(k, sf(cur) + j);
        W(k, WF::ALAM + j) = W(k, WF::LAM + j);
        W(k, WF::AY + j) = W(k, WF::Y + j);
      }
      for (int i = 0; i < NX; ++i) anub[k][i] = nub[k][i];
    }
    have_acc = true;
  }
  MR_HD void acc_restore() {
    for (int k = 0; k <= N; ++k) {
      for (int i = 0; i < NZS; ++i) W(k, zf(cur) + i) = W(k, WF::AZ + i);
      for (int j = 0; j < NI; ++j) {
        W(k, sf(cur) + j) = W(k, WF::ASL + j);
        W(k, WF::LAM + j) = W(k, WF::ALAM + j);
        W(k, WF::Y + j) = W(k, WF::AY + j);
      }
      for (int i = 0; i < NX; ++i) nub[k][i] = anub[k][i];
    }
  }

  // ---------------- the restoration phase (IPOPT's l1 restoration, W&B 2006 sec. 3.3) ----------------
  // Entered when the filter line search finds no acceptable step (and the point is not acceptable / not
  // almost feasible) or when the inertia correction fails.  The restoration NLP relaxes the 6 vehicle
  // dynamics rows of each stage (F - x' - p + n = 0) and every inequality slot (d(z) - s - p + n = 0);
  // the definitional rows of the restatement (S+ = S + dS, the previous-control copies) are not
  // constraints of the reference:
  //   min rho sum (p + n) + zeta/2 sum D^2 (z - z_R)^2,  p, n >= 0,
  // rho = 1000, zeta = sqrt(mu), D = min(1, 1/|z_R|) on the reference's variables; solved by the same
  // IPM (eval / Riccati / forward / filter line search with its own filter and barrier parameter,
  // starting at max(mu, max violation)).  It returns to the original problem at the first accepted
  // step whose point reduces the original theta to <= 0.9 theta(z_R) and is acceptable to the original
  // filter (augmented with z_R's entry on entering).  (Deviations from IPOPT's restoration phase: the
  // initial-state rows X_0 = state0, S_0 = s0 stay hard (x_0 is eliminated), each slot of a two-sided
  // row is relaxed separately, y starts at 0, no inertia shift of the relaxation variables)
  MR_HD void resto_enter(T th, T ph) {
    filter_add(th, ph);
    onfilt = nfilt;
    for (int i = 0; i < nfilt; ++i) { ofilt_th[i] = filt_th[i]; ofilt_ph[i] = filt_ph[i]; }
    mu_o = mu;
    th_entry = th;
    delta_last_o = delta_last;
    theta_max_o = theta_max;
    theta_min_o = theta_min;
    // the current point's constraint values, measured here: after a watchdog restore the evaluation
    // sweep's (defects W(k, C), pr_max, theta) belong to the abandoned iterate.  IPOPT's
    // RestoIterateInitializer: mu_r = max(mu, ||c||_inf, ||d - s||_inf)
    T pr = T(0), th_r = T(0);
    fo_cur = T(0);  // the original objective at the entry point (reported if the restoration phase ends the solve)
    for (int k = 0; k <= N; ++k) {
      T z[NZS];
      load_z(k, cur, z);
      if (k < N) {
        T zn[NZS], xn[NX];
        load_z(k + 1, cur, zn);
        faug<T, MODEL>(P, k, z, xn);
        for (int i = 0; i < NX; ++i) {
          const T c = xn[i] - zn[i];
          W(k, WF::C + i) = c;
          pr = mr_max(pr, mr_abs(c));
          if (i >= 6) th_r += mr_abs(c);  // definitional rows (S, previous controls): not relaxed
        }
      }
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      for (int j = 0; j < NI; ++j)
        if (act[j] && yslot(j)) pr = mr_max(pr, mr_abs(d[j] - W(k, sf(cur) + j)));
      fo_cur += stage_cost(P, I, k, z, e, sc, (T*)nullptr, (T*)nullptr);
    }
    const T mu_r = mr_max(mu, pr);
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
        W(k, WF::RS0 + j) = W(k, sf(cur) + j);
        W(k, WF::RLAM + j) = W(k, WF::LAM + j);
        if (act[j]) resto_pn(d[j] - W(k, sf(cur) + j), mu_r, rho, p, n);
        W(k, WF::RP + j) = p;
        W(k, WF::RN + j) = n;
        W(k, WF::RVP + j) = mu_r / p;
        W(k, WF::RVN + j) = mu_r / n;
        W(k, WF::RDP + j) = W(k, WF::RDN + j) = W(k, WF::RDVP + j) = W(k, WF::RDVN + j) = T(0);
        W(k, WF::RY + j) = W(k, WF::RDY + j) = T(0);  // the rows' equality multipliers start at 0
        W(k, WF::DLAM + j) = T(0);
        // the slacks' bound duals: the original problem's, but not above rho (RestoIterateInitializer)
        if (act[j]) W(k, WF::LAM + j) = mr_min(W(k, WF::LAM + j), rho);
      }
      for (int i = 0; i < NX; ++i) { nub[k][i] = 0.0; W(k, WF::DNU + i) = T(0); }
      if (k < N)
        for (int i = 0; i < 6; ++i) {  // the vehicle rows start satisfied too (p - n = F - x')
          T p, n;
          resto_pn(W(k, WF::C + i), mu_r, rho, p, n);
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
    resto_first = true;
    nfilt = 0;
    delta_last = T(0);
    theta_max = T(1e4) * mr_max(T(1), th_r);
    theta_min = T(1e-4) * mr_max(T(1), th_r);
    if (MR_RESTO_LS_MULT) ls_resto();
  }

  // IPOPT's least-square multipliers of the restoration NLP at its starting point (RestoIterateInitializer ->
  // least_square_mults, constr_mult_init_max 1000; oracle/ipopt.py _Alg.ls_mults on the restoration problem):
  // the multipliers y minimising || grad f_R - z + J^T y ||^2 over every primal variable of the restoration
  // NLP -- the reference's variables, the slacks and the relaxations p, n.  As in ls_init, the dual QP
  //   min 1/2 |u|^2 + q^T u  s.t. J u = 0   (q = grad f_R - z: 0 on the variables (the proximity term's
  //   gradient vanishes at z_R), -v on a slack, rho - v_p / rho - v_n on p / n)
  // on the stage structure: a slot row a.sx - ss - sp + sn = 0 with (ss, sp, sn) condensed leaves
  // (a.sx - cg)^2 / 6, cg = v + v_p - v_n, i.e. H += a a^T / 3, g -= a cg / 3, and the row multiplier
  // y = (cg - a.sx) / 3 (the restoration rows' sign: y = v at stationarity); a relaxed vehicle row's (p, n)
  // condensed into the disturbance w = n - p leave (w + v_p - v_n)^2 / 4: sw = 1/2, gw = (v_p - v_n) / 2.
  // Solved by the restoration Riccati recursion and its forward sweep; the costates are the dynamics rows'
  // multipliers.  All of them zero if one exceeds 1000 in magnitude (the rows', the vehicle rows' and the
  // initial-state rows').
  MR_HD void ls_resto() {
    T z[NZS];
    for (int k = 0; k <= N; ++k) {
      load_z(k, cur, z);
      T H[NH], g[NZ], J[48];
      for (int i = 0; i < NH; ++i) H[i] = T(0);
      for (int i = 0; i < NZ; ++i) g[i] = T(0);
      for (int i = 0; i < 48; ++i) J[i] = T(0);
      if (k < N) {
        T Hd[36], fx[6], nz[NX];
        for (int i = 0; i < NX; ++i) nz[i] = T(0);
        Dyn<T, MODEL>::fjh(P, z, z + NX, nz, fx, J, Hd);
        for (int i = 0; i < 6; ++i) {
          W(k, WF::CSW + i) = T(0.5);
          W(k, WF::CGW0 + i) = T(0.5) * (W(k, WF::CVP + i) - W(k, WF::CVN + i));
          W(k, WF::CGW1 + i) = T(0);
        }
      }
      for (int i = 0; i < NZ; ++i)
        if (delta_var(i)) H[hidx(i, i)] = T(1);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      for (int r = 0; r <= NROW; ++r) {
        const int j0 = r < NROW ? 2 * r : JL;
        if (!act[j0]) continue;
        int idx[3];
        T a[3];
        const int na = row_grad(r, rows, e, idx, a);
        for (int sd = 0; sd < 2; ++sd) {  // slot j0 (a) and j0 + 1 (-a): each its own relaxed row
          const int j = j0 + sd;
          const T sg = sd ? T(-1) : T(1);
          const T cg = W(k, WF::LAM + j) + W(k, WF::RVP + j) - W(k, WF::RVN + j);
          for (int q = 0; q < na; ++q) {
            g[idx[q]] -= sg * a[q] * cg / T(3);
            for (int q2 = q; q2 < na; ++q2) H[hidx(idx[q], idx[q2])] += a[q] * a[q2] / T(3);
          }
        }
      }
      for (int i = 0; i < NH; ++i) { W(k, WF::H + i) = H[i]; W(k, WF::HD + i) = T(0); }
      for (int i = 0; i < NZ; ++i) { W(k, WF::G0 + i) = g[i]; W(k, WF::G1 + i) = T(0); W(k, WF::GD + i) = T(0); }
      for (int i = 0; i < NX; ++i) W(k, WF::C + i) = T(0);
      for (int i = 0; i < 48; ++i) W(k, WF::J + i) = J[i];
    }
    if (!riccati(T(0))) return;  // (not positive definite on the null space: the multipliers stay 0)
    T dx[NX];
    for (int i = 0; i < NX; ++i) dx[i] = T(0);
    bool ok = true;
    const T big = T(IP_MULT_INIT_MAX);
    double nuv[64][NX];
    T yv[64][NI];
    for (int k = 0; k <= N; ++k) {
      T dz[NZS];
      for (int i = 0; i < NZS; ++i) dz[i] = T(0);
      for (int i = 0; i < NX; ++i) dz[i] = dx[i];
      if (k < N)
        for (int a = 0; a < NU; ++a) {
          T v = W(k, WF::K0 + a);
          for (int j = 0; j < NX; ++j) v += W(k, WF::K + a * NX + j) * dx[j];
          dz[NX + a] = v;
        }
      if (k == 0)  // the initial-state rows' multipliers (dx_0 = 0): checked, not kept (x_0 is not relaxed)
        for (int i = 0; i <= 6; ++i) ok = ok && mr_abs(W(0, WF::PV0 + i)) <= big;
      load_z(k, cur, z);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      for (int j = 0; j < NI; ++j) yv[k][j] = T(0);
      for (int r = 0; r <= NROW; ++r) {
        const int j0 = r < NROW ? 2 * r : JL;
        if (!act[j0]) continue;
        int idx[3];
        T a[3];
        const int na = row_grad(r, rows, e, idx, a);
        T adz = T(0);
        for (int q = 0; q < na; ++q) adz += a[q] * dz[idx[q]];
        for (int sd = 0; sd < 2; ++sd) {
          const int j = j0 + sd;
          const T cg = W(k, WF::LAM + j) + W(k, WF::RVP + j) - W(k, WF::RVN + j);
          const T y = (cg - (sd ? -adz : adz)) / T(3);
          yv[k][j] = y;
          ok = ok && mr_abs(y) <= big;
        }
      }
      if (k < N) {
        T J[48], t[NX], tb[NX];
        for (int i = 0; i < 48; ++i) J[i] = W(k, WF::J + i);
        apply_A(J, k, dx, t);
        apply_B(J, k, dz + NX, tb);
        for (int i = 0; i < NX; ++i) dx[i] = t[i] + tb[i];
        T Pn[NP], sw[6], rhs[6], w[6];
        for (int i = 0; i < NP; ++i) Pn[i] = W(k + 1, WF::P + i);
        for (int i = 0; i < 6; ++i) {
          T v = W(k + 1, WF::PV0 + i);
          for (int l = 0; l < NX; ++l) v += Pn[pidx(i, l)] * dx[l];
          rhs[i] = v + W(k, WF::CGW0 + i);
          sw[i] = W(k, WF::CSW + i);
        }
        noise_step(Pn, sw, rhs, w);
        for (int i = 0; i < 6; ++i) dx[i] += w[i];
        for (int i = 0; i < NX; ++i) {  // the multipliers of x_{k+1} = F(x_k, u_k) (+ n - p)
          T v = W(k + 1, WF::PV0 + i);
          for (int l = 0; l < NX; ++l) v += Pn[pidx(i, l)] * dx[l];
          nuv[k + 1][i] = (double)v;
          if (i < 6) ok = ok && mr_abs(v) <= big;
        }
      }
    }
    if (!ok) return;
    for (int k = 0; k <= N; ++k) {
      for (int j = 0; j < NI; ++j) W(k, WF::RY + j) = yv[k][j];
      if (k >= 1)
        for (int i = 0; i < NX; ++i) nub[k][i] = nuv[k][i];
    }
  }
  MR_HD bool resto_done() const {  // the accepted restoration step's point, seen by the original problem
    if (!(tho_acc <= T(RESTO_KAPPA) * th_entry)) return false;
    for (int i = 0; i < onfilt; ++i)
      if (tho_acc >= ofilt_th[i] && pho_acc >= ofilt_ph[i]) return false;
    return true;
  }
  MR_HD void resto_exit() {
    // a two-sided row's slot distances were relaxed separately: one slack again (distances rescaled to
    // the row's range).  Bound duals: the whole restoration taken as one primal Newton step for
    // complementarity at the entry point, dv = mu/t0 - v0 - v0/t0 (t - t0), with the dual fraction to the
    // boundary; all reset to 1 if one exceeds bound_mult_reset_threshold (1000); y = 0
    // (constr_mult_reset_threshold 0); IPOPT's barrier parameter, filter and perturbation state back
    const T tau = mr_max(T(0.99), T(1) - mu_o);
    T ad = T(1), vmax = T(0);
    for (int k = 0; k <= N; ++k) {
      T z[NZS];
      load_z(k, cur, z);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      for (int r = 2; r <= NROW; ++r) {
        const int j0 = r < NROW ? 2 * r : JL;
        if (!act[j0]) continue;
        const T t0 = W(k, sf(cur) + j0), t1 = W(k, sf(cur) + j0 + 1), rng = d[j0] + d[j0 + 1];
        W(k, sf(cur) + j0) = t0 * rng / (t0 + t1);
        W(k, sf(cur) + j0 + 1) = t1 * rng / (t0 + t1);
      }
      for (int j = 0; j < NI; ++j) {
        if (!act[j]) continue;
        const T t0 = W(k, WF::RS0 + j), v0 = W(k, WF::RLAM + j), t = W(k, sf(cur) + j);
        const T dv = mu_o / t0 - v0 - v0 / t0 * (t - t0);
        W(k, WF::DLAM + j) = dv;
        if (dv < T(0)) ad = mr_min(ad, -tau * v0 / dv);
      }
    }
    for (int k = 0; k <= N; ++k)
      for (int j = 0; j < NI; ++j) {
        const T v0 = W(k, WF::RLAM + j);
        if (v0 == T(0)) continue;  // inactive slot
        const T v = v0 + ad * W(k, WF::DLAM + j);
        W(k, WF::LAM + j) = v;
        vmax = mr_max(vmax, mr_abs(v));
      }
    for (int k = 0; k <= N; ++k) {
      for (int j = 0; j < NI; ++j) {
        if (vmax > T(RESTO_MULT_RESET) && W(k, WF::RLAM + j) != T(0)) W(k, WF::LAM + j) = T(1);
        W(k, WF::DLAM + j) = T(0);
        W(k, WF::Y + j) = T(0);
        W(k, WF::DY + j) = T(0);
      }
      for (int i = 0; i < NX; ++i) { nub[k][i] = 0.0; W(k, WF::DNU + i) = T(0); }
    }
    alpha_p = alpha_d = T(0);
    mu = mu_o;
    nfilt = onfilt;
    for (int i = 0; i < onfilt; ++i) { filt_th[i] = ofilt_th[i]; filt_ph[i] = ofilt_ph[i]; }
    theta_max = theta_max_o;
    theta_min = theta_min_o;
    delta_last = delta_last_o;
    resto = false;
  }

  // IPOPT's primal-dual system error (the soft restoration phase's measure; oracle/ipopt.py pd_error): the
  // 1-norms of the Lagrangian gradient in the reference's variables (States, S_hat, U), of the slacks'
  // stationarity -y - v_L + v_U, of the residuals c and d - s, and of v t - mu, at iterate buffer b with
  // every multiplier stepped by a (0: the current ones).  Only ratios are used: the term count is not
  // divided out.  (mr_wave.h pd_sweep: the same sums.)
  MR_HD T pd_error(int b, T a) const {
    T sum = T(0), sref_b = T(0), sref_u[2] = {T(0), T(0)}, sref_u0[2] = {T(0), T(0)}, sref_w[2] = {T(0), T(0)};
    for (int k = 0; k <= N; ++k) {
      T z[NZS], zn[NZS];
      load_z(k, b, z);
      T st[NZ], J[48];
      double dd[NZ], nuk[NX], nun[NX];
      for (int i = 0; i < NZ; ++i) { st[i] = T(0); dd[i] = 0.0; }
      for (int i = 0; i < NX; ++i) nuk[i] = nub[k][i] + (double)a * (double)W(k, WF::DNU + i);
      if (k < N) {
        load_z(k + 1, b, zn);
        for (int i = 0; i < NX; ++i) nun[i] = nub[k + 1][i] + (double)a * (double)W(k + 1, WF::DNU + i);
        T Hd[36], fx[6], nz[NX];
        for (int i = 0; i < NX; ++i) nz[i] = T(0);
        Dyn<T, MODEL>::fjh(P, z, z + NX, nz, fx, J, Hd);
        T xn[NX];
        faug<T, MODEL>(P, k, z, xn);
        for (int i = 0; i < NX; ++i) sum += mr_abs(xn[i] - zn[i]);
        apply_At(J, k, nun, dd);
        apply_Bt(J, k, nun, dd + NX);
      }
      for (int i = 0; i < NX; ++i) dd[i] -= nuk[i];
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      stage_cost(P, I, k, z, e, sc, st, (T*)nullptr);
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      T lam_j[NI], y_j[NI];
      for (int j = 0; j < NI; ++j) {
        lam_j[j] = y_j[j] = T(0);
        if (!act[j]) continue;
        const T t = W(k, sf(b) + j);
        lam_j[j] = W(k, WF::LAM + j) + a * W(k, WF::DLAM + j);
        sum += mr_abs(lam_j[j] * t - mu);
        if (yslot(j)) {
          y_j[j] = W(k, WF::Y + j) + a * W(k, WF::DY + j);
          sum += mr_abs(d[j] - t);
        }
      }
      for (int r = 0; r <= NROW; ++r) {
        const int j0 = r < NROW ? 2 * r : JL, j1 = j0 + 1;
        if (!act[j0]) continue;
        int idx[3];
        T av[3];
        const int na = row_grad(r, rows, e, idx, av);
        T ys;
        if (r < 2) {
          ys = y_j[j0] + y_j[j1];
          sum += mr_abs(-y_j[j0] - lam_j[j0]) + mr_abs(-y_j[j1] + lam_j[j1]);
        } else {
          ys = y_j[j0];
          sum += mr_abs(-y_j[j0] - lam_j[j0] + lam_j[j1]);
        }
        for (int q = 0; q < na; ++q) st[idx[q]] += ys * av[q];
      }
      T sti[NZ];
      for (int i = 0; i < NZ; ++i) sti[i] = T((double)st[i] + dd[i]);
      for (int i = 0; i < 6; ++i) sum += mr_abs(sti[i]);  // X_k
      const T bb = k < N ? sti[13] : T(0);
      sum += mr_abs(sti[6] + sref_b - bb);  // S_k
      sref_b = bb;
      if (k >= 1)
        for (int q = 0; q < 2; ++q) {
          const T u = sref_u[q] + sti[7 + q];
          if (k == 1) sref_u0[q] = u; else sum += mr_abs(u);
          sref_w[q] += sti[9 + q];
        }
      if (k < N) { sref_u[0] = sti[11]; sref_u[1] = sti[12]; }
      if (k == N)
        for (int q = 0; q < 2; ++q) sum += mr_abs(sref_u0[q] + sref_w[q]);
    }
    return sum;
  }
  // IPOPT's TrySoftRestoStep (oracle/ipopt.py try_soft_resto): the full primal-dual step with one step size
  // a = min(alpha_primal_max, alpha_dual_max); 1: accepted by the filter / sufficient-decrease test against
  // the current point (an h-type step), 2: accepted by a primal-dual error reduction, 0: rejected.  The
  // trial point is in buffer 1-cur; alpha = a.
  MR_HD int soft_resto(const LSRef<T>& ref, T ap, T ad, T& alpha) {
    const T a = mr_min(ap, ad);
    alpha = a;
    T th_t, ph_t;
    if (!trial(a, false, th_t, ph_t)) return 0;
    if (th_t <= theta_max && acc_to_iterate(th_t, ph_t, ref) && filter_ok(th_t, ph_t)) return 1;
    return pd_error(1 - cur, a) <= T(IP_SOFT_RESTO_FACTOR) * pd_error(cur, T(0)) ? 2 : 0;
  }

  // IPOPT's tiny-step test (tiny_step_tol 10 eps): every component of the step of the reference's
  // variables (global X, Y, S) and of IPOPT's slacks s below 10 eps relative to (1 + |value|), at a point
  // with primal infeasibility <= 1e-4.  ymall: also the multipliers' step below tiny_step_y_tol (1e-2).
  MR_HD bool tiny_step(bool& ysmall) const {
    if (!(pr_max <= T(1e-4))) return false;
    const T tt = T(IP_TINY_STEP_TOL);
    ysmall = true;
    for (int k = 0; k <= N; ++k) {
      T z[NZS];
      load_z(k, cur, z);
      for (int i = 0; i < NZ; ++i) {
        if (!delta_var(i) || (k == 0 && i <= 6) || (k == N && i >= NX)) continue;
        const T org = i == 0 ? I.org[0] : (i == 1 ? I.org[1] : (i == 6 ? I.org[2] : T(0)));
        if (mr_abs(W(k, WF::DZ + i)) > tt * (T(1) + mr_abs(z[i] + org))) return false;
      }
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      Row<T> rows[NROW];
      row_values(k, z, e, d, act, rows);
      for (int j = 0; j < NI; ++j) {
        if (!act[j] || !yslot(j)) continue;
        const T c = j < JL ? rows[j / 2].c : e.eC;
        const T sv = c - T(slot_sign(j)) * (d[j] - W(k, sf(cur) + j));  // IPOPT's slack value
        if (mr_abs(W(k, WF::DS + j)) > tt * (T(1) + mr_abs(sv))) return false;
        if (!(mr_abs(W(k, WF::DY + j)) < T(1e-2))) ysmall = false;
      }
      for (int i = 0; i < NX; ++i)
        if ((i < 6 || (k == 0 && i == 6)) && !(mr_abs(W(k, WF::DNU + i)) < T(1e-2))) ysmall = false;
    }
    return true;
  }

  // ---------------- the IPM loop ----------------
  MR_HD SolveOut solve() {
    const T kappa_eps = T(10), kappa_mu = T(0.2), theta_mu = T(1.5);
    // IPOPT's monotone update keeps mu >= min(tol, compl_inf_tol) / (barrier_tol_factor + 1)
    const T mu_min = mr_max(T(1e-11), mr_min(P.tol, T(IP_COMPL_INF_TOL)) / (kappa_eps + T(1)));
    SolveOut out{2, 0, 0.0, 0.0, 0.0};
    T mu_prev = mu;
    int acc_count = 0, stall = 0;
    // IPOPT's filter reset heuristic (filter_reset_trigger = 5, max_filter_resets = 5): after this many
    // successive iterations whose line search had a trial point rejected by the filter, clear it
    int filt_rej_iters = 0, filt_resets = 0;
    // watchdog state and the reference values of the point where it started
    bool in_wd = false, tiny_flag = false, in_soft = false;
    int soft_count = 0;
    int wd_short = 0, wd_trial = 0;
    LSRef<T> wd_ref{T(0), T(0), T(0), T(0)};
    T wd_ap = T(0), wd_ad = T(0), wd_amin = T(0);
    int it = 0;
    for (it = 0;; ++it) {
      MR_PROF(0, eval_sweep(mu_prev));
      T kkt = nlp_error();
      if (!(kkt == kkt) || !(fval == fval)) { out.status = 3; break; }
#ifdef MR_RESTO_DEBUG
      if (trace) printf("it %d resto %d kkt %.3e stat %.3e pr %.3e viol %.3e smax %.3e nu1 %.3e y1 %.3e lam1 %.3e mu %.3e fval %.6e theta %.4e\n", it, (int)resto, (double)kkt, (double)stat_max, (double)pr_max, (double)viol_max, (double)slam_max, (double)nu1, (double)y1, (double)lam1, (double)mu, (double)fval, (double)theta);
      if (trace) printf("   acc %d conv %d compl/sc %.3e cv %.3e du %.3e tiny %d\n", (int)acceptable(kkt), (int)converged(kkt), (double)(compl_err(T(0)) / sc), (double)mr_max(pr_eq, viol_max), (double)(stat_max / sc), (int)tiny_flag);
#endif
      if (resto) {
        // the restoration NLP converged at a point the original problem does not accept: IPOPT's
        // "restoration converged to a feasible point unacceptable to the filter" (restoration failed)
        // when that point is feasible to 1e2 tol, else "converged to a point of local infeasibility"
        out.viol = (double)mr_max(pr_o, viol_max);  // the restoration iterate as the original problem sees it
        if (kkt <= P.tol) { out.status = pr_o <= T(100) * P.tol ? 3 : MR_STATUS_INFEASIBLE; break; }
      } else {
        out.kkt = (double)kkt;
        out.obj = (double)(fval / sc);
        out.viol = (double)mr_max(pr_eq, viol_max);
        if (converged(kkt)) { out.status = 0; break; }
        if (P.acc_iter > 0) {
          acc_count = acceptable(kkt) ? acc_count + 1 : 0;
          if (acc_count >= P.acc_iter) { out.status = 1; break; }
        }
        // fp32 only: at the mu floor, feasible to IPOPT's constr_viol_tol, without meeting
        // the convergence tests for MR_F32_STALL iterations -> the fp64 solve's outcome there (the line
        // search fails at the floor: the stored acceptable point or status 3).  In fp32 the constraint
        // violation and phi carry rounding noise well above that line search's resolution, so trial
        // points keep being accepted and the solve would run to max_iter instead.
        if (sizeof(T) == 4 && MR_F32_STALL > 0) {
          stall = (mu <= mu_min && mr_max(pr_eq, viol_max) <= T(IP_CONSTR_VIOL_TOL)) ? stall + 1 : 0;
          if (stall >= MR_F32_STALL) {
            if (have_acc) {
              acc_restore();
              out.status = 1;
              out.kkt = acc_kkt; out.obj = acc_obj; out.viol = acc_viol;
            } else {
              out.status = 3;
            }
            break;
          }
        }
      }
      if (it >= P.max_iter) { out.status = 2; break; }
      T mu_old = mu;
      bool mu_stuck = false;
      const bool skip_mu = resto && resto_first;  // IPOPT's MonotoneMuUpdate: none in the restoration phase's first iteration
      resto_first = false;
      while (!skip_mu && (barrier_error(mu) <= kappa_eps * mu || tiny_flag)) {
        const T m1 = kappa_mu * mu, m2 = mr_exp(theta_mu * mr_log(mu));
        const T mn = mr_max(mu_min, mr_min(m1, m2));
        if (mn == mu) { mu_stuck = tiny_flag; break; }
        mu = mn;
        tiny_flag = false;
      }
      if (mu_stuck) { out.status = 3; break; }  // tiny step at the smallest mu (IPOPT: search direction too small)
      tiny_flag = false;
      if (mu != mu_old) {  // IPOPT resets its line search with a new barrier problem: filter, watchdog, soft resto
        nfilt = 0;
        in_wd = false;
        wd_short = 0;
        in_soft = false;
        soft_count = 0;
      }
      const T ph_cur = fval - mu * logs + T(IP_KAPPA_D) * mu * lins;  // the barrier objective (+ damping)
      // inertia-corrected factorisation (PDPerturbationHandler: delta = 0 first; then delta_xs_init 1e-4
      // or delta_last / 3; x100 while delta_last is 0 or delta > 1e5 delta_last, else x8; up to 1e40)
      T delta = T(0);
      bool first = true, fact_ok = false;
      for (int tries = 0; tries < 200; ++tries) {
        bool rok;
        MR_PROF(1, rok = riccati(delta));
        if (rok) { fact_ok = true; break; }
        if (first) {
          delta = delta_last == T(0) ? T(1e-4) : mr_max(T(1e-20), delta_last / T(3));
          first = false;
        } else {
          delta *= (delta_last == T(0) || T(1e5) * delta_last < delta) ? T(100) : T(8);
        }
        if (delta > T(1e40)) break;
      }
      if (!fact_ok) {
        if (resto) { out.status = 3; break; }
        // IPOPT: no inertia-correct factorisation -> the restoration phase
        resto_enter(theta, ph_cur);
        mu_prev = mu;
        in_wd = false;
        wd_short = 0;
        in_soft = false;
        soft_count = 0;
        acc_count = 0;
        continue;
      }
      if (delta > T(0)) delta_last = delta;
      delta_it = delta;
      T ap, ad, gphi;
      MR_PROF(2, forward(ap, ad, gphi));
      // filter line search
      T th = theta, ph = ph_cur;
      LSRef<T> ref{th, ph, gphi, mr_exp(T(1.1) * mr_log(mr_max(th, T(1e-300))))};
      const T a_min = alpha_min_of(th, gphi);
      rej_filter = false;
      if (resto) {  // a restoration-phase step: its own filter, no watchdog, no second-order correction
        T alpha, a_test, ph_acc;
        int nls = 0;
        bool soc_taken;
        const bool accepted = backtrack(ap, false, false, T(0), ref, a_min, alpha, a_test, ph_acc, nls, soc_taken);
        if (!accepted) { out.status = 3; break; }  // IPOPT: restoration failed
        fo_cur = fo_acc;  // the accepted step's point is the last trial evaluated (no SOC here)
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
        if (!(is_ftype(a_test, ref) && armijo(ph_acc, a_test, ref))) filter_add(th, ph);
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
      if (acceptable(kkt)) {  // IPOPT stores the current iterate if it is acceptable
        acc_save();
        acc_kkt = out.kkt; acc_obj = out.obj; acc_viol = out.viol;
      }
      T alpha = ap, a_test = ap, ph_acc = ph;
      bool accepted = false, take_anyway = false, tiny = false, soc_taken = false, soft_step = false,
           soft_orig = false;
      int nls = 0;
      LSRef<T> used = ref;
      if (MR_SOFT_RESTO && in_soft) {
        // the soft restoration phase continues (IPOPT: max_soft_resto_iters): its step replaces the line search
        if (++soft_count <= IP_MAX_SOFT_RESTO) {
          const int sr = soft_resto(ref, ap, ad, alpha);
          if (sr) {
            accepted = soft_step = true;
            soft_orig = sr == 1;
            if (soft_orig) { in_soft = false; soft_count = 0; }
          }
        }
      } else {
#if MR_WD_TRIGGER > 0
        // IPOPT's watchdog (watchdog_shortened_iter_trigger, watchdog_trial_iter_max): after that many
        // successive iterations whose accepted step was shorter than the fraction-to-boundary step, store
        // the iterate and its search direction and take full steps tentatively; they are judged against
        // the stored point (at its step size), and after watchdog_trial_iter_max iterations without an
        // acceptable one the solver returns to the stored point and backtracks along its direction
        // (skipping the full step)
        if (!in_wd && wd_short >= MR_WD_TRIGGER) {
          wd_save();
          wd_ref = ref;
          wd_ap = ap; wd_ad = ad; wd_amin = a_min;
          in_wd = true;
          wd_trial = 0;
        }
#endif
        bool ysmall = false;
        if (MR_TINY_STEP && tiny_step(ysmall)) {  // IPOPT: a tiny step is taken without line search (and forces a mu decrease)
          T th_t, ph_t;
          trial(ap, false, th_t, ph_t);
          accepted = tiny = true;
          tiny_flag = ysmall;
        } else if (in_wd) {
          accepted = backtrack(ap, false, true, wd_ap, wd_ref, ap, alpha, a_test, ph_acc, nls, soc_taken);
          used = wd_ref;
          if (accepted) {
            in_wd = false;
            wd_short = 0;
          } else if (++wd_trial <= MR_WD_TRIAL_MAX) {
            take_anyway = true;  // the full step is taken tentatively
            alpha = ap;
            T th_t, ph_t;
            trial(alpha, false, th_t, ph_t);
          } else {
            // back to the watchdog point: its iterate and direction, a regular backtracking line search
            // that skips the full step
            wd_restore();
            in_wd = false;
            wd_short = 0;
            ref = wd_ref;
            used = wd_ref;
            ap = wd_ap; ad = wd_ad;
            accepted = backtrack(ap, true, false, T(0), ref, wd_amin, alpha, a_test, ph_acc, nls, soc_taken);
            th = ref.th; ph = ref.ph;
          }
        } else {
          accepted = backtrack(ap, false, false, T(0), ref, a_min, alpha, a_test, ph_acc, nls, soc_taken);
        }
        if (MR_SOFT_RESTO && !accepted && !take_anyway) {
          // IPOPT's soft restoration phase before the restoration phase proper (TrySoftRestoStep)
          const int sr = soft_resto(ref, ap, ad, alpha);
          if (sr) {
            accepted = soft_step = true;
            soft_orig = sr == 1;
            in_soft = !soft_orig;
            soft_count = 0;
            used = ref;
          }
        }
      }
#ifdef MR_RESTO_DEBUG
      if (trace) printf("   ls accepted %d take %d tiny %d alpha %.3e ap %.3e amin %.3e soc %d\n", (int)accepted, (int)take_anyway, (int)tiny, (double)alpha, (double)ap, (double)a_min, (int)soc_taken);
#endif
      if (!accepted && !take_anyway) {
        // IPOPT on a failed line search (and failed soft restoration): the current point acceptable ->
        // "acceptable point reached"; almost feasible (theta <= 1e-2 tol) -> the stored acceptable point, or
        // restoration failed; otherwise the restoration phase
        if (acceptable(kkt)) { out.status = 1; break; }
        if (theta <= T(1e-2) * P.tol ||
            (sizeof(T) == 4 && mr_max(pr_eq, viol_max) <= T(IP_CONSTR_VIOL_TOL))) {  // fp32: feasible at its resolution
          if (have_acc) {
            acc_restore();
            out.status = 1;
            out.kkt = acc_kkt; out.obj = acc_obj; out.viol = acc_viol;
          } else {
            out.status = 3;
          }
          break;
        }
        resto_enter(th, ph);
        mu_prev = mu;
        in_wd = false;
        wd_short = 0;
        in_soft = false;
        soft_count = 0;
        acc_count = 0;
        if (trace && it < trace_cap) {
          double* tr = trace + 8 * it;
          tr[0] = (double)kkt; tr[1] = (double)mu; tr[2] = (double)0; tr[3] = (double)0;
          tr[4] = (double)delta; tr[5] = (double)th; tr[6] = (double)ph; tr[7] = -300.0;
        }
        continue;
      }
      if (soc_taken) ad = wd_ad_of_commit();
      if (!take_anyway && !tiny && !soft_step) wd_short = (alpha < ap) ? wd_short + 1 : 0;
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
      // IPOPT augments the filter unless the step is f-type with the Armijo condition (a tiny step: never; a
      // soft restoration step: only when the regular criterion accepted it -- an h-type step)
      if (!take_anyway && (soft_step ? soft_orig : (!tiny && !(is_ftype(a_test, used) && armijo(ph_acc, a_test, used)))))
        filter_add(used.th, used.ph);
      if (soft_step) ad = alpha;  // the soft restoration step moves every variable by one step size
      if (trace && it < trace_cap) {
        double* tr = trace + 8 * it;
        tr[0] = (double)kkt; tr[1] = (double)mu; tr[2] = (double)alpha; tr[3] = (double)ad;
        tr[4] = (double)delta; tr[5] = (double)used.th; tr[6] = (double)used.ph;
        tr[7] = (double)(take_anyway ? -100 - wd_trial : (soc_taken ? 100 + nls : nls));
      }
      alpha_p = alpha;
      alpha_d = ad;
      mu_prev = mu;
      cur = 1 - cur;
    }
    out.iters = it;
    // ended inside the restoration phase: the returned (restoration) iterate's original objective
    if (resto) out.obj = (double)(fo_cur / sc);
    if (trace && it < trace_cap) {  // final record: why the loop ended
      double* tr = trace + 8 * it;
      tr[0] = (double)out.kkt; tr[1] = (double)fval; tr[2] = (double)theta; tr[3] = (double)stat_max;
      tr[4] = (double)pr_max; tr[5] = (double)sc; tr[6] = (double)mu; tr[7] = 1000.0 + out.status;
    }
    return out;
  }
  // the dual step size of the committed second-order-correction direction (fraction to the boundary)
  MR_HD T wd_ad_of_commit() const {
    const T tau = mr_max(T(0.99), T(1) - mu);
    T ad = T(1);
    for (int k = 0; k <= N; ++k)
      for (int j = 0; j < NI; ++j) {
        const T lam = W(k, WF::LAM + j), dl = W(k, WF::DLAM + j);
        if (lam != T(0) && dl < T(0)) ad = mr_min(ad, -tau * lam / dl);
      }
    return ad;
  }
};

}  // namespace mr
