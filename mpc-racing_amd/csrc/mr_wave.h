// Wave-per-instance interior-point solver of the racing-MPC NLP (the gfx950 product kernel).
//
// Replaces the CasADi Opti + IPOPT solve of control/MPC.py:30-181.  Same NLP, same
// stage-wise restatement and the same IPOPT-rule algorithm as the stage-level pieces in
// mr_solver.h (formulation notes there), but one 64-lane wavefront cooperates on one
// instance instead of one lane running it alone:
//
//   * lanes = stages (k = lane <= N <= 63) for every stage-parallel sweep: evaluation of
//     dynamics/derivatives/cost/rows, slack and multiplier steps, line-search trial points;
//     KKT-error and merit terms are butterfly reductions over the wave;
//   * lanes = matrix rows for the backward Riccati recursion (sequential in k): lane r owns
//     row r of the 11x11 cost-to-go P and of the 14x14 stage Q-function; the two dense
//     products P*[A B] and [A B]^T*(P*[A B]) exchange rows through ~3 KB of LDS;
//   * the forward substitution (sequential, 11+3 values) runs wave-uniform.
//
// Working set per instance (global workspace, base + i * ws_words<T>()):
//   ss[f][64]   per-stage iterate / step fields, lane-contiguous (coalesced per field); the fp32
//               product kernel keeps them in LDS instead (SSL)
//   rc[k][336]  per-stage Riccati record (stage Hessian, Jacobian, gradients, P, K)
//   cold[f][64] watchdog / restoration fields (CSF)
//   nu[2][11][64] the dynamics rows' multipliers and their watchdog copy, fp64 in both precisions
#pragma once
#include <new>

#include "mr_batch.h"
#include "mr_wave_prims.h"

// The sweeps are separate (non-inlined) device functions so each gets its own register
// allocation; only the small wave-uniform iteration state is live across the calls.
#if MR_DEVICE_BUILD && defined(MR_SWEEP_INLINE)
#define MR_SWEEP __device__ __forceinline__
#define MR_CLOCK() ((unsigned long long)__builtin_amdgcn_s_memtime())
#elif MR_DEVICE_BUILD
#define MR_SWEEP __device__ __attribute__((noinline))
#define MR_CLOCK() ((unsigned long long)__builtin_amdgcn_s_memtime())
#else
#define MR_SWEEP inline
#define MR_CLOCK() 0ull
#endif
#if MR_DEVICE_BUILD
#define MR_SCHED_BARRIER() __builtin_amdgcn_sched_barrier(0)
#else
#define MR_SCHED_BARRIER() ((void)0)
#endif

// Device sweeps are non-inlined member functions: `this` (the solver object) and the problem /
// instance constants it references live in LDS (mpcracing.hip), which the compiler cannot see
// through the generic pointers; the assumption lets it emit ds_read instead of flat loads.
// (mr_wave_kernel is the only device user of WaveSolver and always places it so.)
#if MR_DEVICE_BUILD && defined(__HIP_DEVICE_COMPILE__)
#define MR_ASSUME_LDS_STATE()                                      \
  do {                                                             \
    __builtin_assume(__builtin_amdgcn_is_shared((const void*)this));  \
    __builtin_assume(__builtin_amdgcn_is_shared((const void*)&I));    \
  } while (0)
#else
#define MR_ASSUME_LDS_STATE() ((void)0)
#endif

// the wave-uniform view of the problem constants inside a WaveSolver method (shadows the member)
#define MR_UNIFORM_P() const ProbParams<T>& P = *(const ProbParams<T>*)wu_ptr(&this->P)

#ifndef MR_PHASE_CYCLES
#define MR_PHASE_CYCLES 0  // 1: per-sweep shader-cycle counters of the trace instance (tools/phase_probe.py)
#endif
#ifndef MR_EVAL_HOIST
#define MR_EVAL_HOIST 0  // 1: the evaluation sweep loads slacks / multipliers ahead of the record stores
#endif
#ifndef MR_FWD_TREE
#define MR_FWD_TREE 0  // 1: the forward recursion's dot products as three chains (A/B option)
#endif
#ifndef MR_RIC_AHEAD
#define MR_RIC_AHEAD 2  // stages the Riccati's operand gathers run ahead of the factorisation (2 or 3)
#endif
#ifndef MR_PRIO_ITER
#define MR_PRIO_ITER 0  // > 0: the wave raises its issue priority (s_setprio) at this iteration
#endif

namespace mr {

struct SSF {
  enum {
    Z0 = 0, Z1 = Z0 + NZS, DZ = Z1 + NZS, S0 = DZ + NZS, S1 = S0 + NI, LAM = S1 + NI, DLAM = LAM + NI,
    DS = DLAM + NI, DNU = DS + NI, GL = DNU + NX, NF = GL + NZ
  };
};
// Stage record (stage-major, RC_STRIDE words per stage): the evaluation sweep's stage QP data
// (Jacobian, defect, Hessian, gradients), then the Riccati sweep's outputs.
struct RCF {
  enum {
    J = 0, C = J + 48, H = C + NX, G0 = H + NH, G1 = G0 + NZ,
    P = G1 + NZ, PV0 = P + NP, K = PV0 + NX, K0 = K + NU * NX,
    CONE = K0 + NU, CZERO, SELP, SEL0,  // constants 1, 0, [k > 0], [k == 0] (written once per solve)
    JUNK, NF                           // discard slot of the branch-free stores (any lane)
  };
};
#ifdef MR_RC_STRIDE_FORCE
constexpr int RC_STRIDE = MR_RC_STRIDE_FORCE;  // A/B option (record footprint)
#else
constexpr int RC_STRIDE = (RCF::NF + 15) / 16 * 16;  // words; 16-word (64 B) multiple (320)
#endif
static_assert(RCF::NF <= RC_STRIDE, "record");
// Cold per-stage fields [f][64] after the records: touched only by the watchdog (its snapshot of the
// iterate and the search direction) and the restoration phase (the relaxations p, n of the rows and
// of the 6 vehicle dynamics rows, their bound duals and steps, the rows' equality multipliers y, the
// reference point z_R, the condensed disturbance weights of the Riccati sweep) -- same meaning as the
// WF fields of mr_solver.h's scalar solver.
struct CSF {
  enum {
    WZ = 0, WSL = WZ + NZS, WLAM = WSL + NI, WDZ = WLAM + NI, WDS = WDZ + NZS, WDLAM = WDS + NI,
    WDNU = WDLAM + NI,
    RP = WDNU + NX, RN = RP + NI, RVP = RN + NI, RVN = RVP + NI, RDP = RVN + NI, RDN = RDP + NI, RDVP = RDN + NI,
    RDVN = RDVP + NI, RY = RDVN + NI, RDY = RY + NI, RZ = RDY + NI,
    CP = RZ + NZS, CN = CP + 6, CVP = CN + 6, CVN = CVP + 6, CDP = CVN + 6, CDN = CDP + 6, CDVP = CDN + 6,
    CDVN = CDVP + 6, CSW = CDVN + 6, CGW0 = CSW + 6, CGW1 = CGW0 + 6, NF = CGW1 + 6
  };
};
// The dynamics rows' multipliers nu (and their watchdog snapshot) in fp64 whatever the solve precision,
// [2][NX][64] doubles after the cold fields: eval_sweep forms the stationarity residual and the
// Riccati right-hand side from them in fp64 (the correction form, see there).
constexpr int64_t WS_NU_OFF = (int64_t)SSF::NF * WL + (int64_t)RC_STRIDE * WL + (int64_t)CSF::NF * WL;  // words
template <typename T>
MR_HD constexpr int64_t ws_words() { return WS_NU_OFF + 2 * NX * WL * (int64_t)(sizeof(double) / sizeof(T)); }

// Wave-uniform state of the watchdog and the restoration phase: one copy per wavefront next to the
// line-search filter (LDS on the device), every lane writing the same values -- not in the per-lane
// solver objects, whose LDS footprint sets the occupancy.
template <typename T>
struct WaveCold {
  int resto, in_wd, wd_short, wd_trial, onfilt;
  T rho, zeta, mu_o, th_entry, delta_last_o, theta_max_o, theta_min_o, tho, pho;
  T wd_th, wd_ph, wd_gphi, wd_ap, wd_ad, wd_amin, wd_thpow;
  T ofilt[2 * FMAX];  // the original problem's filter while the restoration phase runs
};
template <typename T>
struct WaveShared {
  T filt[2 * FMAX];
  WaveCold<T> cold;
};
constexpr int LDS_LD = 17;  // padded row of the 16 x 16 LDS tiles
constexpr int LX_OFF = 0, LP_OFF = 16 * LDS_LD, LDX_OFF = 32 * LDS_LD;
constexpr int LJUNK_OFF = LDX_OFF + WL * 12;  // one discard slot per lane (branch-free stores)
constexpr int LDS_WORDS = LJUNK_OFF + WL;

// lower-triangular solves with L packed (00,10,11,20,21,22) as produced by chol3
template <typename T>
MR_HD void lsolve3(const T* L, T* b) {
  b[0] = b[0] / L[0];
  b[1] = (b[1] - L[1] * b[0]) / L[2];
  b[2] = (b[2] - L[3] * b[0] - L[4] * b[1]) / L[5];
}
template <typename T>
MR_HD void ltsolve3(const T* L, T* b) {
  b[2] = b[2] / L[5];
  b[1] = (b[1] - L[4] * b[2]) / L[2];
  b[0] = (b[0] - L[1] * b[1] - L[3] * b[2]) / L[0];
}

// Inequality rows of stage k (MPC.py:134-149) with their fixed sparsity, so every index is a
// compile-time constant after unrolling (no private-memory arrays):
//   r = 0 thr box, 1 steer box, 2 dS box, 3/4 rate rows vs p (or state0 at k = 0),
//   5/6 wrap-around rate rows U[:,0] - U[:,N-1] at k = N-1 via the frozen copy w.
//   c_r(z) = sum_a RS(a) z[RI(r, a)],  lo_r <= c_r <= hi_r.
MR_HD constexpr int RN(int r) { return r < 3 ? 1 : 2; }
MR_HD constexpr int RI(int r, int a) {
  return r == 0 ? 11 : r == 1 ? 12 : r == 2 ? 13 : r == 3 ? (a ? 7 : 11) : r == 4 ? (a ? 8 : 12) : r == 5 ? (a ? 11 : 9)
                                                                                                         : (a ? 12 : 10);
}
MR_HD constexpr int RS(int a) { return a ? -1 : 1; }

template <typename T>
MR_HD void row_bounds(const ProbParams<T>& P, const Inst<T>& I, int k, int r, int& act, T& lo, T& hi) {
  const int N = P.N;
  act = 0; lo = T(0); hi = T(0);
  if (k == N) return;
  if (r == 0) { act = 1; lo = P.min_thr; hi = I.d_max; }          // MPC.py:138-139 (class-attribute d_max)
  else if (r == 1) { act = 1; lo = P.min_steer; hi = P.max_steer; }  // :140-141
  else if (r == 2) { act = 1; lo = P.min_ds; hi = P.Ts * P.v_max; }  // :134
  else if (r == 3) { act = (k >= 1 || I.has_thr0) ? 1 : 0; lo = P.min_dthr; hi = P.max_dthr; }      // :142 / :145-146
  else if (r == 4) { act = (k >= 1 || I.has_steer0) ? 1 : 0; lo = P.min_dsteer; hi = P.max_dsteer; }  // :143 / :148-149
  else if (r == 5) { act = (k == N - 1 && N >= 2) ? 1 : 0; lo = P.min_dthr; hi = P.max_dthr; }       // :142 at i = 0
  else { act = (k == N - 1 && N >= 2) ? 1 : 0; lo = P.min_dsteer; hi = P.max_dsteer; }                // :143 at i = 0
}
template <typename T>
MR_HD T row_c(int r, const T* z) { return RN(r) == 1 ? z[RI(r, 0)] : z[RI(r, 0)] - z[RI(r, 1)]; }

// 3x3 Cholesky with reciprocal pivots (3 divisions instead of one per substitution step)
template <typename T>
MR_HD bool chol3r(const T* R, T* L, T* iv) {
  // branch-free: a non-positive pivot is replaced by 1 and reported (the caller discards L)
  // (the diagonal of L is only needed through its reciprocals iv)
  const bool ok0 = R[0] > T(0);
  iv[0] = mr_rsqrt(ok0 ? R[0] : T(1));
  const T l10 = R[1] * iv[0], l20 = R[2] * iv[0];
  const T d1 = R[3] - l10 * l10;
  const bool ok1 = d1 > T(0);
  iv[1] = mr_rsqrt(ok1 ? d1 : T(1));
  const T l21 = (R[4] - l20 * l10) * iv[1];
  const T d2 = R[5] - l20 * l20 - l21 * l21;
  const bool ok2 = d2 > T(0);
  iv[2] = mr_rsqrt(ok2 ? d2 : T(1));
  L[0] = T(0); L[1] = l10; L[2] = T(0); L[3] = l20; L[4] = l21; L[5] = T(0);
  return ok0 & ok1 & ok2;
}
template <typename T>
MR_HD void lsolve3r(const T* L, const T* iv, T* b) {
  b[0] = b[0] * iv[0];
  b[1] = (b[1] - L[1] * b[0]) * iv[1];
  b[2] = (b[2] - L[3] * b[0] - L[4] * b[1]) * iv[2];
}
template <typename T>
MR_HD void ltsolve3r(const T* L, const T* iv, T* b) {
  b[2] = b[2] * iv[2];
  b[1] = (b[1] - L[4] * b[2]) * iv[1];
  b[0] = (b[0] - L[1] * b[1] - L[3] * b[2]) * iv[0];
}

// Where the per-stage fields ss[f][64] live: global workspace, or (SSL) the workgroup's LDS
// (fp32: 152 x 64 x 4 B = 38.9 KB, 3 instances per CU).  Same arithmetic either way.
template <typename T, bool SSL>
struct SSPtr { typedef MR_GLOBAL T* type; };
#if MR_DEVICE_BUILD
template <typename T>
struct SSPtr<T, true> { typedef MR_LDS T* type; };
#endif
constexpr int SS_WORDS = SSF::NF * WL;

template <typename T, int MODEL, bool SSL = false>
struct WaveSolver {
  // problem constants: device memory read through a constant-address-space pointer made wave-uniform
  // in every method (MR_UNIFORM_P), so they are scalar loads into SGPRs, not VGPRs
  const MR_CONST ProbParams<T>& P;
  const Inst<T>& I;
  Wv w;
  typename SSPtr<T, SSL>::type ss;
  MR_GLOBAL T* rc;
  MR_LDS T* lds;
  int N, ln;
  // wave-uniform iteration state
  int cur;
  T mu, sc, delta_last;
  T alpha_p, alpha_d;
  T theta_max, theta_min;
#if MR_DEVICE_BUILD
  // the filter is wave-uniform: one copy per workgroup in LDS (set by mr_wave_kernel), every
  // lane writing the same values, instead of one copy per lane in the solver object; the
  // watchdog / restoration state (WaveCold) follows it in the same LDS block (WaveShared)
  MR_LDS T* filt;
  MR_HD MR_LDS WaveCold<T>* cw() const { return &((MR_LDS WaveShared<T>*)filt)->cold; }
#else
  WaveShared<T> sh_store;
  T* filt = sh_store.filt;
  MR_HD WaveCold<T>* cw() { return &sh_store.cold; }
#endif
  int nfilt;
  T stat_max, pr_max, theta, slam_max, slam_min, nu1, lam1, fval, logs;
  int me, mi;
  // out-parameters of the non-inlined sweeps: members, so they land in the object's LDS slot
  // rather than in the caller's private stack (a scratch round trip after every call)
  T res_ap, res_ad, res_gphi, res_alpha;
  int res_flags, res_nls, res_ntr, res_nsoc;
  double* trace = nullptr;
  int trace_cap = 0;
#if MR_PHASE_CYCLES
  unsigned long long tsub[6] = {0, 0, 0, 0, 0, 0};  // diagnostics: sub-phase cycles of the trace instance
#endif

  MR_HD WaveSolver(const MR_CONST ProbParams<T>& P_, const Inst<T>& I_, Wv w_, MR_GLOBAL T* ws, MR_LDS T* lds_,
                   typename SSPtr<T, SSL>::type ss_)
      : P(P_), I(I_), w(w_), ss(ss_), rc(ws + (int64_t)SSF::NF * WL), lds(lds_), N(P_.N), ln(w_.lane) {}

  MR_HD auto& S(int f) const { return ss[f * WL + ln]; }
  MR_HD MR_GLOBAL T& Cf(int f) const { return rc[(int64_t)RC_STRIDE * WL + f * WL + ln]; }  // cold field
  // fp64 multiplier nu_k[i] of stage k = lane (x_k = F(x_{k-1}, u_{k-1}), k >= 1), its watchdog copy
  MR_HD MR_GLOBAL double* nub() const { return (MR_GLOBAL double*)(rc + (int64_t)(RC_STRIDE + CSF::NF) * WL); }
  MR_HD MR_GLOBAL double& NUd(int i) const { return nub()[i * WL + ln]; }
  MR_HD MR_GLOBAL double& WNUd(int i) const { return nub()[(NX + i) * WL + ln]; }
  MR_HD auto& fth(int i) const { return filt[i]; }
  MR_HD auto& fph(int i) const { return filt[FMAX + i]; }
  MR_HD MR_GLOBAL T* R(int k) const { return rc + (int64_t)k * RC_STRIDE; }
  MR_HD bool own() const { return ln <= N; }

  MR_HD int zf(int b) const { return b ? SSF::Z1 : SSF::Z0; }
  MR_HD int sf(int b) const { return b ? SSF::S1 : SSF::S0; }
  MR_HD int nxt() const { return (ln + 1) & (WL - 1); }

  MR_HD void load_z(int b, T* z) const {
    for (int i = 0; i < NZS; ++i) z[i] = own() ? S(zf(b) + i) : T(0);
    if (ln >= N) { z[11] = T(0); z[12] = T(0); z[13] = T(0); }
  }

  MR_HD void row_values(int k, const T* z, const Err<T>& e, T* d, int* act) const {
    MR_UNIFORM_P();
#pragma unroll
    for (int r = 0; r < NROW; ++r) {
      int a;
      T lo, hi;
      row_bounds(P, I, k, r, a, lo, hi);
      const T c = row_c(r, z);
      act[2 * r] = act[2 * r + 1] = a;
      d[2 * r] = c - lo;
      d[2 * r + 1] = hi - c;
    }
    const int la = lane_active(P, k) ? 1 : 0;
    act[JL] = act[JL + 1] = la;  // the hard lane rows e_C + m >= 0, m - e_C >= 0 (slot JL + 2 unused)
    act[JL + 2] = 0;
    lane_d(I, e.eC, T(0), d + JL);
  }

  // ---------------- initialisation (MPC.py:100-131) ----------------
  MR_SWEEP void init(const double* u_init, int64_t ustride) {
    MR_UNIFORM_P();
    cur = 0;
    T z[NZS], zn[NX], my[NZS];
    for (int i = 0; i < NZS; ++i) { z[i] = T(0); my[i] = T(0); }
    for (int i = 0; i < 6; ++i) z[i] = I.x0[i];
    z[7] = I.has_thr0 ? I.thr0 : T(0);
    z[8] = I.has_steer0 ? I.steer0 : T(0);
    // initial-guess rollout (sequential, wave-uniform); lane k keeps stage k
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
      z[14] = T(0);  // (the stage vector's slot 14 is unused)
      if (ln == k)
        for (int i = 0; i < NZS; ++i) my[i] = z[i];
      if (k < N) {
        faug<T, MODEL>(P, k, z, zn);
        for (int i = 0; i < NX; ++i) z[i] = zn[i];
      }
    }
    T gmax = T(0), th = T(0);
    if (own()) {
      const int k = ln;
      for (int i = 0; i < NZS; ++i) S(SSF::Z0 + i) = my[i];
      Err<T> e;
      errors(I, my[0], my[1], my[6], e, false);
      T g[NZ];
      for (int i = 0; i < NZ; ++i) g[i] = T(0);
      stage_cost(P, I, k, my, e, T(1), g, (T*)nullptr);
      for (int i = 0; i < NZ; ++i) gmax = mr_max(gmax, mr_abs(g[i]));
      T d[NI];
      int act[NI];
      row_values(k, my, e, d, act);
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        T push;
        if (j < JL) {
          int ra;
          T lo, hi;
          row_bounds(P, I, k, j / 2, ra, lo, hi);
          T bnd = (j & 1) ? mr_abs(hi) : mr_abs(lo);
          push = mr_min(T(1e-2) * mr_max(T(1), bnd), T(1e-2) * (hi - lo));
        } else {
          push = j < JL + 2 ? T(1e-2) * mr_max(T(1), I.max_err) : T(1e-2);
        }
        T s = act[j] ? mr_max(d[j], push) : T(1);
        S(SSF::S0 + j) = s;
        S(SSF::LAM + j) = act[j] ? T(1) : T(0);
        S(SSF::DLAM + j) = T(0);
        if (act[j]) th += mr_abs(d[j] - s);
      }
      for (int i = 0; i < NX; ++i) { NUd(i) = 0.0; S(SSF::DNU + i) = T(0); }
      MR_GLOBAL T* Rk = R(k);  // constant slots of the Riccati gather plan (frag_plan)
      Rk[RCF::CONE] = T(1);
      Rk[RCF::CZERO] = T(0);
      Rk[RCF::SELP] = k > 0 ? T(1) : T(0);
      Rk[RCF::SEL0] = k > 0 ? T(0) : T(1);
      if (k == N) {
        // stage N has no dynamics and no gains: the evaluation and Riccati sweeps never write its
        // Jacobian / defect / K / k slots, yet the forward recursion's last step (k = N) gathers
        // them in its lane groups 0 and 2 (whose results go only to the unused LDX row N + 1 and
        // du_N); zeros keep that step on defined values
        for (int q = 0; q < 48; ++q) Rk[RCF::J + q] = T(0);
        for (int q = 0; q < NX; ++q) Rk[RCF::C + q] = T(0);
        for (int q = 0; q < NU * NX; ++q) Rk[RCF::K + q] = T(0);
        for (int q = 0; q < NU; ++q) Rk[RCF::K0 + q] = T(0);
      }
    }
    gmax = wmax(w, gmax);
    th = wsum(w, th);
    sc = gmax > T(0) ? mr_min(T(1), T(100) / gmax) : T(1);
    mu = T(0.1);
    delta_last = T(0);
    alpha_p = alpha_d = T(0);
    theta_max = T(1e4) * mr_max(T(1), th);
    theta_min = T(1e-4) * mr_max(T(1), th);
    nfilt = 0;
    auto* C = cw();
    C->resto = 0;
    C->in_wd = 0;
    C->wd_short = 0;
    C->wd_trial = 0;
  }

  // ---------------- sweep 1: evaluation, KKT error terms, stage QP data (lane = stage) ----------------
  // RESTO: the restoration phase's NLP (mr_solver.h Solver::eval_sweep with resto set): relaxed vehicle
  // dynamics and rows, the proximity term instead of the objective
  template <bool RESTO>
  MR_SWEEP void eval_sweep(T mu_prev) {
    MR_ASSUME_LDS_STATE();
    MR_UNIFORM_P();
    const T kappa_sigma = T(1e10);
    T rho = T(0), zeta = T(0);
    if constexpr (RESTO) {
      rho = cw()->rho;
      zeta = mr_sqrt(mu_prev);  // IPOPT: resto_proximity_weight sqrt(mu)
      cw()->zeta = zeta;
    }
    auto clip = [&](T v, T x) { return mr_min(mr_max(v, mu_prev / (kappa_sigma * x)), kappa_sigma * mu_prev / x); };
    const int k = ln;
    T st_l = T(0), pr_l = T(0), th_l = T(0), smax_l = T(0), smin_l = T(1e30), nu1_l = T(0), lam1_l = T(0),
      f_l = T(0), lg_l = T(0);
    int mi_l = 0;
    // lazy multiplier update nu_k += alpha_p * dnu_k (stages 1..N), in fp64; T copies weight the
    // dynamics Hessian
    // refk: the optimality error on the reference's NLP (mr_solver.h MR_KKT_RESTATED); nu_0[0..6] = the
    // multipliers of the initial-state rows X_0 = state0, S_0 = s0 (stepped by the stage-0 costate)
    constexpr bool refk = !MR_KKT_RESTATED && !RESTO;
    T nuk[NX];
    for (int i = 0; i < NX; ++i) nuk[i] = T(0);
    if (own() && k >= 1) {
      for (int i = 0; i < NX; ++i) {
        const double v = NUd(i) + (double)alpha_p * (double)S(SSF::DNU + i);
        NUd(i) = v;
        nuk[i] = T(v);
        if (!refk || i < 6) nu1_l += mr_abs(nuk[i]);
      }
    } else if (refk && k == 0) {
      for (int i = 0; i <= 6; ++i) {
        const double v = NUd(i) + (double)alpha_p * (double)S(SSF::DNU + i);
        NUd(i) = v;
        nu1_l += mr_abs(T(v));
      }
    }
    T z[NZS];
    load_z(cur, z);
    T nun[NX], znext[NX];
    for (int i = 0; i < NX; ++i) {
      nun[i] = wnext(w, nuk[i]);
      znext[i] = wnext(w, z[i]);
    }
#if MR_PHASE_CYCLES
    const unsigned long long te0 = trace ? MR_CLOCK() : 0ull;
#endif
    // the stage record through a buffer resource: its stores do not order this sweep's later
    // stage-field loads (different memory objects to the compiler), so those issue early
    const WBuf<T> rbe(rc, (unsigned)WL * (unsigned)RC_STRIDE);
    const unsigned Rk = (unsigned)k * (unsigned)RC_STRIDE;
    T H[NH], g0[NZ], g1[NZ], gl[NZ], st[NZ], J[48];
    T rs_a = T(0), rs_b = T(0), rs_u[2] = {T(0), T(0)}, rs_p[2] = {T(0), T(0)}, rs_w[2] = {T(0), T(0)};
    if (own()) {
      for (int i = 0; i < NH; ++i) H[i] = T(0);
      for (int i = 0; i < NZ; ++i) { g0[i] = g1[i] = gl[i] = st[i] = T(0); }
      if (k < N) {
        T Hd[36], fx[6];
        Dyn<T, MODEL>::fjh(P, z, z + NX, nun, fx, J, Hd);
        const int map[8] = {0, 1, 2, 3, 4, 5, 11, 12};
        int q = 0;
        for (int a = 0; a < 8; ++a)
          for (int bb = a; bb < 8; ++bb, ++q) H[hidx(map[a], map[bb])] += Hd[q];
        T c[NX];
        for (int i = 0; i < 6; ++i) c[i] = fx[i] - znext[i];
        c[6] = z[6] + z[13] - znext[6];
        c[7] = z[11] - znext[7];
        c[8] = z[12] - znext[8];
        c[9] = (k == 0 ? z[11] : z[9]) - znext[9];
        c[10] = (k == 0 ? z[12] : z[10]) - znext[10];
        if constexpr (RESTO) {  // relaxed vehicle rows F - x' - p + n (the S / previous-control rows are definitions)
          for (int i = 0; i < 6; ++i) {
            const T p = Cf(CSF::CP + i), n = Cf(CSF::CN + i);
            const T vp = clip(Cf(CSF::CVP + i) + alpha_d * Cf(CSF::CDVP + i), p);
            const T vn = clip(Cf(CSF::CVN + i) + alpha_d * Cf(CSF::CDVN + i), n);
            Cf(CSF::CVP + i) = vp;
            Cf(CSF::CVN + i) = vn;
            c[i] += n - p;
            const T ip = p / vp, in = n / vn, sw = T(1) / (ip + in);
            Cf(CSF::CSW + i) = sw;
            // + nu_{k+1}: the Riccati right-hand side is in correction form (below), the disturbance's is not
            Cf(CSF::CGW0 + i) = sw * rho * (in - ip) + nun[i];
            Cf(CSF::CGW1 + i) = sw * (T(1) / vp - T(1) / vn);
            smax_l = mr_max(smax_l, mr_max(p * vp, n * vn));
            smin_l = mr_min(smin_l, mr_min(p * vp, n * vn));
            lam1_l += mr_abs(vp) + mr_abs(vn);
            lg_l += mr_log(p) + mr_log(n);
            mi_l += 2;
            f_l += rho * (p + n);
            st_l = mr_max(st_l, mr_max(mr_abs(rho - nun[i] - vp), mr_abs(rho + nun[i] - vn)));
          }
        }
        for (int i = 0; i < NX; ++i) {
          rbe.st(c[i], 0u, Rk + RCF::C + i);
          pr_l = mr_max(pr_l, mr_abs(c[i]));
          th_l += mr_abs(c[i]);
        }
        for (int i = 0; i < 48; ++i) rbe.st(J[i], 0u, Rk + RCF::J + i);
      }
    }
    // The dynamics rows' terms of the Lagrangian gradient, dd = [A^T nu_{k+1} - nu_k ; B^T nu_{k+1}], in
    // fp64 from the fp64 multipliers (nu_{k+1} from the neighbour lane, after the Hessian so the fp64
    // copies are not live across it).  Correction form: the Riccati right-hand side is g0 + dd, so the
    // sweeps solve for the multipliers' step dnu directly (forward: dnu = P dx + p), and g0 + dd and the
    // stationarity residual are small near a solution and carry full relative precision.  In fp32 the
    // absolute form (nu_new = P dx + p with p ~ nu ~ 1e3) cannot resolve the stationarity below the
    // fp32 ulp of the costates (1.2e-4 at 1e3), above a 1e-4 tolerance.
    double nnd[NX];
    for (int i = 0; i < NX; ++i) nnd[i] = wnext(w, (own() && k >= 1) ? NUd(i) : 0.0);
    if (own()) {
      double dd[NZ];
      for (int i = 0; i < NZ; ++i) dd[i] = 0.0;
      if (k < N) {
        apply_At(J, k, nnd, dd);
        apply_Bt(J, k, nnd, dd + NX);
      }
      if (k >= 1 || refk)  // (k = 0: nu_0 of the initial-state rows, zero unless refk)
        for (int i = 0; i < NX; ++i) dd[i] -= NUd(i);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, true);
      if constexpr (RESTO) {
        T zr[NZS];
        for (int i = 0; i < NZS; ++i) zr[i] = Cf(CSF::RZ + i);
        f_l += prox_term(I, k, N, z, zr, zeta, gl, H);
      } else {
        f_l += stage_cost(P, I, k, z, e, sc, gl, H);
      }
      for (int i = 0; i < NZ; ++i) { g0[i] += gl[i]; st[i] += gl[i]; S(SSF::GL + i) = gl[i]; }
      T d[NI];
      int act[NI];
      row_values(k, z, e, d, act);
      T lam_j[NI], s_j[NI];
      T sg_j[NI], c0_j[NI], c1_j[NI], y_j[NI];  // restoration: condensed row data (row_cond_r), multipliers y
      for (int j = 0; j < NI; ++j) {
        lam_j[j] = T(0);
        s_j[j] = T(1);
        sg_j[j] = c0_j[j] = c1_j[j] = y_j[j] = T(0);
        if (!act[j]) continue;
        T s = S(sf(cur) + j);
        T lam = S(SSF::LAM + j) + alpha_d * S(SSF::DLAM + j);
        lam = mr_min(mr_max(lam, mu_prev / (kappa_sigma * s)), kappa_sigma * mu_prev / s);
        S(SSF::LAM + j) = lam;
        lam_j[j] = lam;
        s_j[j] = s;
        T rd = d[j] - s;
        T sl = s * lam;
        smax_l = mr_max(smax_l, sl);
        smin_l = mr_min(smin_l, sl);
        lam1_l += mr_abs(lam);
        lg_l += mr_log(s);
        mi_l += 1;
        if constexpr (RESTO) {  // relaxed row d - s - p + n; its multiplier y is its own variable (IPOPT's y_d)
          const T p = Cf(CSF::RP + j), n = Cf(CSF::RN + j);
          const T vp = clip(Cf(CSF::RVP + j) + alpha_d * Cf(CSF::RDVP + j), p);
          const T vn = clip(Cf(CSF::RVN + j) + alpha_d * Cf(CSF::RDVN + j), n);
          Cf(CSF::RVP + j) = vp;
          Cf(CSF::RVN + j) = vn;
          const T y = Cf(CSF::RY + j) + alpha_p * Cf(CSF::RDY + j);
          Cf(CSF::RY + j) = y;
          y_j[j] = y;
          st_l = mr_max(st_l, mr_abs(y - lam));
          rd = rd - p + n;
          smax_l = mr_max(smax_l, mr_max(p * vp, n * vn));
          smin_l = mr_min(smin_l, mr_min(p * vp, n * vn));
          lam1_l += mr_abs(vp) + mr_abs(vn);
          lg_l += mr_log(p) + mr_log(n);
          mi_l += 2;
          f_l += rho * (p + n);
          st_l = mr_max(st_l, mr_max(mr_abs(rho + y - vp), mr_abs(rho - y - vn)));
          row_cond_r(d[j], s, lam, p, n, vp, vn, rho, sg_j[j], c0_j[j], c1_j[j]);
        }
        pr_l = mr_max(pr_l, mr_abs(rd));
        th_l += mr_abs(rd);
      }
#pragma unroll
      for (int r = 0; r < NROW; ++r) {
        if (!act[2 * r]) continue;
        T sig_sum = T(0), gsc0 = T(0), gsc1 = T(0), lamdiff = T(0);
#pragma unroll
        for (int sd = 0; sd < 2; ++sd) {
          int j = 2 * r + sd;
          T sgn = sd == 0 ? T(1) : T(-1);
          if constexpr (RESTO) {
            sig_sum += sg_j[j];
            gsc0 += sgn * c0_j[j];
            gsc1 += sgn * c1_j[j];
            lamdiff += sgn * y_j[j];
          } else {
            T sig = lam_j[j] / s_j[j];
            sig_sum += sig;
            gsc0 += sgn * sig * (d[j] - s_j[j]);
            gsc1 += -sgn / s_j[j];
            lamdiff += sgn * lam_j[j];
          }
        }
#pragma unroll
        for (int a = 0; a < RN(r); ++a) {
          const T sa = T(RS(a));
          g0[RI(r, a)] += sa * gsc0;
          g1[RI(r, a)] += sa * gsc1;
          st[RI(r, a)] -= lamdiff * sa;
#pragma unroll
          for (int bb = a; bb < RN(r); ++bb) H[hidx(RI(r, a), RI(r, bb))] += sig_sum * sa * T(RS(bb));
        }
      }
      if (lane_active(P, k)) {
        // hard lane rows e_C + m >= 0 (slot JL) and m - e_C >= 0 (JL + 1), nonlinear in (X, Y, S)
        const int id3[3] = {0, 1, 6};
        T s0 = s_j[JL], s1 = s_j[JL + 1];
        T sig0 = lam_j[JL] / s0, sig1 = lam_j[JL + 1] / s1;
        T lamdiff = lam_j[JL] - lam_j[JL + 1];
        T gz0 = sig0 * (d[JL] - s0) - sig1 * (d[JL + 1] - s1);
        T gz1 = -T(1) / s0 + T(1) / s1;
        if constexpr (RESTO) {
          sig0 = sg_j[JL];
          sig1 = sg_j[JL + 1];
          lamdiff = y_j[JL] - y_j[JL + 1];
          gz0 = c0_j[JL] - c0_j[JL + 1];
          gz1 = c1_j[JL] - c1_j[JL + 1];
        }
        int q = 0;
        for (int a = 0; a < 3; ++a) {
          g0[id3[a]] += e.gC[a] * gz0;
          g1[id3[a]] += e.gC[a] * gz1;
          st[id3[a]] -= lamdiff * e.gC[a];
          for (int bb = a; bb < 3; ++bb, ++q)
            H[hidx(id3[a], id3[bb])] += (sig0 + sig1) * e.gC[a] * e.gC[bb] - lamdiff * e.hC[q];
        }
      }
      if constexpr (refk) {  // the reference's variables: X_k here, S_k and U_k with their copies below
        T sti[NZ];
        for (int i = 0; i < NZ; ++i) sti[i] = T((double)st[i] + dd[i]);
        for (int i = 0; i < 6; ++i) st_l = mr_max(st_l, mr_abs(sti[i]));
        rs_a = sti[6];
        rs_b = k < N ? sti[13] : T(0);
        if (k < N) { rs_u[0] = sti[11]; rs_u[1] = sti[12]; }
        if (k >= 1) { rs_p[0] = sti[7]; rs_p[1] = sti[8]; rs_w[0] = sti[9]; rs_w[1] = sti[10]; }
      } else {
        for (int i = 0; i < NZ; ++i) {
          const T sti = T((double)st[i] + dd[i]);
          if (i < NX ? k >= 1 : k < N) st_l = mr_max(st_l, mr_abs(sti));
        }
      }
      for (int i = 0; i < NH; ++i) rbe.st(H[i], 0u, Rk + RCF::H + i);
      for (int i = 0; i < NZ; ++i) {
        rbe.st(T((double)g0[i] + dd[i]), 0u, Rk + RCF::G0 + i);
        rbe.st(g1[i], 0u, Rk + RCF::G1 + i);
      }
    }
    if constexpr (refk) {
      // S_k = S_k + Delta-S_{k-1} - Delta-S_k; U_k = u_k + p_{k+1} (U_0: + every w_j); lanes > N hold zeros
      const T bprev = wprev(w, rs_b), pn0 = wnext(w, rs_p[0]), pn1 = wnext(w, rs_p[1]);
      const T ws0 = wsum(w, rs_w[0]), ws1 = wsum(w, rs_w[1]);
      if (own()) {
        st_l = mr_max(st_l, mr_abs(rs_a + (k >= 1 ? bprev : T(0)) - rs_b));
        if (k < N) {
          st_l = mr_max(st_l, mr_abs(rs_u[0] + pn0 + (k == 0 ? ws0 : T(0))));
          st_l = mr_max(st_l, mr_abs(rs_u[1] + pn1 + (k == 0 ? ws1 : T(0))));
        }
      }
    }
#if MR_PHASE_CYCLES
    const unsigned long long te1 = trace ? MR_CLOCK() : 0ull;
#endif
    stat_max = wmax(w, st_l);
    pr_max = wmax(w, pr_l);
    theta = wsum(w, th_l);
    slam_max = wmax(w, smax_l);
    slam_min = wmin(w, smin_l);
    nu1 = wsum(w, nu1_l);
    lam1 = wsum(w, lam1_l);
    fval = wsum(w, f_l);
    logs = wsum(w, lg_l);
    mi = wsum(w, mi_l);
    me = refk ? 6 * N + 7 : NX * (N + 1);
    wsync(w);  // stage records visible to every lane before the Riccati sweep
#if MR_PHASE_CYCLES
    if (trace) { tsub[2] += te1 - te0; tsub[3] += MR_CLOCK() - te1; }
#endif
  }

  MR_HD T kkt_error(T m) const {
    const T smax = T(100);
    T sd = mr_max(smax, (nu1 + lam1) / T(me + (mi > 0 ? mi : 1))) / smax;
    T scm = mr_max(smax, lam1 / T(mi > 0 ? mi : 1)) / smax;
    T cerr = mr_max(mr_abs(slam_max - m), mr_abs(m - slam_min));
    if (mi == 0) cerr = T(0);
    return mr_max(mr_max(stat_max / sd, pr_max), cerr / scm);
  }

  // D-register row map of the 16x16x4 MFMA (mr_wave_prims.h) and its inverse
  static MR_HD constexpr int drow(int g, int v) { return sizeof(T) == 8 ? g + 4 * v : 4 * g + v; }
  static MR_HD constexpr int dgrp(int a) { return sizeof(T) == 8 ? (a & 3) : (a >> 2); }
  static MR_HD constexpr int dreg(int a) { return sizeof(T) == 8 ? (a >> 2) : (a & 3); }

  // Entry (i, j) of the 16 x 16 stage map E^ of stage k:
  //   rows 0..10 = [A | B | 0 | c] of x_{k+1} = A x + B u + c (columns 0..10 x, 11..13 u, 14 c);
  //   row 11 routes p0 into column 14, row 12 routes p1 into column 15.
  // Entry (i, j) of E^: record index (data entries: Jacobian or defect) or constant 0/1
  static MR_HD void ehat_src(int k, int i, int j, int& idx, bool& data, T& cst) {
    const int jj = j < 6 ? j : (j == 11 ? 6 : (j == 12 ? 7 : -1));
    const bool cdef = (i < NX) & (j == 14);
    const bool jac = (i < 6) & (jj >= 0);
    idx = cdef ? RCF::C + i : (jac ? RCF::J + i * 8 + jj : 0);
    data = cdef | jac;
    const bool one = ((i == 6) & ((j == 6) | (j == 13))) | ((i == 7) & (j == 11)) | ((i == 8) & (j == 12)) |
                     ((i == 9) & (j == (k > 0 ? 9 : 11))) | ((i == 10) & (j == (k > 0 ? 10 : 12))) |
                     ((i == 11) & (j == 14)) | ((i == 12) & (j == 15));
    cst = one ? T(1) : T(0);
  }

  // Per-lane MFMA operands of stage k (lane = (g, c) = (lane >> 4, lane & 15)):
  //   eb[s] = E^[4s+g][c]                           B fragment of X = P^ E^ and A fragment of E^T X
  //   hc[v] = (H + delta I | g0 | g1)[drow(g,v)][c]  C input of Q
  // The gather plan (record offsets, data/constant/diagonal bits, output targets) depends on
  // the lane only (k == 0 differs in two constants) and is built once per factorisation;
  // frag_load issues the 8 gathers unconditionally two stages ahead, frag_finish applies the
  // selects when the stage is factorised, so no load is sunk into a lane-divergent branch.
  static constexpr int NGATHER = 8;
  struct FragPlan {
    int off[NGATHER];  // record offsets: data entries, or the record's constant slots (CONE, CZERO, SELP, SEL0)
    unsigned dlt;  // D registers on the diagonal of H (+ delta)
    int st_p[4], lp[4];  // per D register: record / LDS targets (discard slots if none)
  };
  // record slot of entry (i, j) of E^ (either stage class k = 0 / k > 0): its data word, or the
  // constant slot holding its value; CZERO when !keep
  static MR_HD int ehat_slot(int i, int j, bool keep) {
    int idx;
    bool data;
    T cst;
    if (!keep) return RCF::CZERO;
    ehat_src(1, i, j, idx, data, cst);
    if (data) return idx;
    const bool one_pos = cst != T(0);
    ehat_src(0, i, j, idx, data, cst);
    const bool one_k0 = cst != T(0);
    return one_pos ? (one_k0 ? RCF::CONE : RCF::SELP) : (one_k0 ? RCF::SEL0 : RCF::CZERO);
  }
  static MR_HD void frag_plan(int lane, FragPlan& fp) {
    const int g = lane >> 4, c = lane & 15;
    fp.dlt = 0u;
#pragma unroll
    for (int s = 0; s < 4; ++s) fp.off[s] = ehat_slot(4 * s + g, c, true);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int a = drow(g, v);
      const int a_ = a < NZ ? a : 0;
      fp.off[4 + v] = a < NZ ? (c < NZ ? RCF::H + hidx(a_, c) : (c == 14 ? RCF::G0 + a_ : RCF::G1 + a_)) : RCF::CZERO;
      if (a < NZ && a == c && delta_var(a)) fp.dlt |= 1u << v;
      // outputs of D register v: packed-upper P | p (column 14) to the record; the whole tile of P^
      // (both triangles as the product computes them, one LDS write per register) to LDS
      const int junk_r = RCF::JUNK, junk_l = LJUNK_OFF - LP_OFF + lane;  // lp index from LP
      const bool ax = a < NX, sq = ax & (c < NX), up = sq & (a <= c);
      const bool c14 = ax & (c == 14);
      fp.st_p[v] = up ? RCF::P + pidx(a, c) : (c14 ? RCF::PV0 + a : junk_r);
      fp.lp[v] = sq ? a * LDS_LD + c : (c14 ? a * LDS_LD + 11 : junk_l);
    }
  }
  static MR_HD void frag_load(const WBuf<T>& rb, unsigned ro, const FragPlan& fp, T* raw) {
#pragma unroll
    for (int q = 0; q < NGATHER; ++q) raw[q] = rb.ld(ro, (unsigned)fp.off[q]);
  }
  // operands straight from the gathered words (constants come from the record's constant slots)
  static MR_HD void frag_finish(const T* dd, const T* raw, T* eb, T* hc) {
#pragma unroll
    for (int s = 0; s < 4; ++s) eb[s] = raw[s];
#pragma unroll
    for (int v = 0; v < 4; ++v) hc[v] = raw[4 + v] + dd[v];
  }

  // ---------------- sweep 2: Riccati factorisation on the matrix cores ----------------
  // Backward over stages, with P^ = [P' | p'] (cost-to-go of stage k+1) kept in LDS:
  //   X    = P^ E^                        3 x v_mfma 16x16x4  (= [P'A  P'B | P'c + p'])
  //   Q    = (H + dI | g) + E^T X         3 x v_mfma          (E^'s B fragment is E^T's A fragment)
  //   Q_uu = L L^T (3x3, wave-uniform),   W = L^{-1} Q_u.     (one column per lane)
  //   P^   = Q_x. - W^T W                 1 x v_mfma
  //   K = -L^{-T} W_x,  k = -L^{-T} w
  // The right-hand side is the iteration's: g = g0 + mu g1 (the evaluation sweep stores the barrier
  // gradient's mu-free and mu parts because mu is updated after it; the gathered g1 column is folded into
  // the g0 column by a DPP row shift), so P^ has one vector column and E^'s contraction index one row less:
  // the fourth K-chunk of both products is zero and skipped (7 MFMAs per stage instead of 9).
  // Stage k-2's record is gathered (8 loads per lane) while stage k is factorised.  The record gets
  // P, p, K, k of stage k; the forward recursion forms A dx + B du + c from the stage's
  // Jacobian itself (no closed-loop map is stored: 132 fewer words written per stage and
  // factorisation, and a smaller record).
  // Restoration phase: the cost-to-go tile P^ of stage k+1 (LP) minimised over the disturbance of
  // stage k's relaxed vehicle rows (mr_solver.h noise_cond): M = P_vv + diag(sw) = L L^T (every lane,
  // registers), Y = L^-1 [P_v. | p0_v + gw0 | p1_v + gw1] (lane c < 13: column c, to the LX scratch
  // tile), then P^ -= Y^T Y entry-wise.  False if M is not positive definite.
  // In fp64 whatever T (mr_solver.h noise_cond: the vehicle block of P^ is otherwise fp32 rounding noise
  // where a relaxation is active); the L^-1 columns go through the LX scratch tile as doubles.
  MR_HD bool noise_tile(int k, MR_LDS T* LP, T mu) const {
    typedef double D;
    static_assert(6 * 16 * sizeof(D) <= 16 * LDS_LD * sizeof(T), "LX scratch holds 6 x 16 doubles");
    MR_LDS D* const LX = (MR_LDS D*)(lds + LX_OFF);
    const MR_GLOBAL T* cb = rc + (int64_t)RC_STRIDE * WL;
    const int l = ln;
    D sw[6], gw0[6], gw1[6], M[36], L[36];
    for (int i = 0; i < 6; ++i) {
      sw[i] = (D)cb[(CSF::CSW + i) * WL + k];
      gw0[i] = (D)cb[(CSF::CGW0 + i) * WL + k];
      gw1[i] = (D)cb[(CSF::CGW1 + i) * WL + k];
    }
    for (int i = 0; i < 6; ++i)
      for (int j = 0; j < 6; ++j) M[i * 6 + j] = (D)LP[i * LDS_LD + j] + (i == j ? sw[i] : 0.0);
    const bool ok = chol6(M, L);
    if (!wuni(w, ok)) return false;
    const int c = l < 13 ? l : 0;
    D col[6];
    for (int i = 0; i < 6; ++i) col[i] = (D)LP[i * LDS_LD + c] + (c == 11 ? gw0[i] + (D)mu * gw1[i] : 0.0);
    lsolve6(L, col);
    if (l < 13)
      for (int a = 0; a < 6; ++a) LX[a * 16 + l] = col[a];
    wsync_lds(w);
    for (int e = l; e < NX * 13; e += WL) {
      const int i = e / 13, j = e - 13 * (e / 13);
      D v = (D)LP[i * LDS_LD + j];
      for (int a = 0; a < 6; ++a) v -= LX[a * 16 + i] * LX[a * 16 + j];
      LP[i * LDS_LD + j] = (T)v;
    }
    wsync_lds(w);
    return true;
  }

  template <bool RESTO>
  MR_SWEEP bool riccati(T delta, T mu) {
    MR_ASSUME_LDS_STATE();
    const int l = ln, N = wu(w, this->N), g = l >> 4, c = l & 15;
    const Wv w = this->w;
    // the instance's records as a wave-uniform buffer: gathers and stores are (uniform stage offset,
    // 32-bit lane offset) buffer operations
    const WBuf<T> rb(rc, (unsigned)WL * (unsigned)RC_STRIDE);
    MR_LDS T* const LP = lds + LP_OFF;
    auto R = [](int k) { return (unsigned)k * (unsigned)RC_STRIDE; };  // word offset of stage k's record
    for (int q = l; q < 16 * LDS_LD; q += WL) LP[q] = T(0);
    wsync_lds(w);
    FragPlan fp;
    frag_plan(l, fp);
    T dd[4];
#pragma unroll
    for (int v = 0; v < 4; ++v) dd[v] = ((fp.dlt >> v) & 1u) ? delta : T(0);
    // lane-constant 0/1 selectors: per-lane picks as products (exact for finite values), so the
    // step has no lane-divergent branches
    const T sg[3] = {g == 0 ? T(1) : T(0), g == 1 ? T(1) : T(0), g == 2 ? T(1) : T(0)};
    const T s14 = c == 14 ? mu : T(0), k15 = c == 15 ? T(0) : T(1);  // g = g0 + mu g1 into column 14
    // operand gathers run two stages ahead of the factorisation (three rotating buffers): a record
    // gather is an Infinity-Cache / HBM round trip (the 8 192 instances' records do not fit the L2),
    // longer than one stage's arithmetic
    T raw_a[NGATHER], raw_b[NGATHER], raw_c[NGATHER];
    frag_load(rb, R(N - 1), fp, raw_a);
    frag_load(rb, R(N >= 2 ? N - 2 : 0), fp, raw_b);
#if MR_RIC_AHEAD == 3
    T raw_d[NGATHER];
    frag_load(rb, R(N >= 3 ? N - 3 : 0), fp, raw_c);
#endif
    {  // terminal cost-to-go: P_N = H_N,xx + delta I, p_N = g_N.  Branch-free (lanes >= NX write
       // discard slots), so at least as many memory ops follow the first prefetch on this path as
       // on the loop back-edge and the wait at the loop head stays exact.
      const unsigned Rn = R(N);
      const bool row = l < NX;
      const int lr = row ? l : 0, jl = RCF::JUNK, jd = LJUNK_OFF - LP_OFF + l;
      T hv[NX];  // all loads ahead of the stores (the compiler cannot disambiguate H from P)
#pragma unroll
      for (int j = 0; j < NX; ++j) hv[j] = rb.ld(Rn, RCF::H + hidx(lr, j));
      const T p0 = rb.ld(Rn, RCF::G0 + lr), p1 = rb.ld(Rn, RCF::G1 + lr);
#pragma unroll
      for (int j = 0; j < NX; ++j) {
        const T v = hv[j] + (l == j && delta_var(j) ? delta : T(0));
        LP[row ? l * LDS_LD + j : jd] = v;
        rb.st(v, Rn, (row && j >= l) ? RCF::P + pidx(lr, j) : jl);
      }
      const T pN = p0 + mu * p1;
      LP[row ? l * LDS_LD + 11 : jd] = pN;
      rb.st(pN, Rn, row ? RCF::PV0 + l : jl);
    }
    wsync_lds(w);
    // one stage; the loop below is unrolled by three so the prefetch buffers rotate roles
    // (no register copies of in-flight loads, hence exact vmcnt waits instead of vmcnt(0))
    auto step = [&](int k, const T* raw_use, T* raw_fill) -> bool {
      bool noise_ok = true;
      if constexpr (RESTO) noise_ok = noise_tile(k, LP, mu);  // P^ of stage k+1 minimised over the disturbance
      // stage offsets as visibly wave-uniform values (SGPR soffsets, not per-lane waterfall loops)
      const unsigned Rk = (unsigned)wu(w, (int)R(k));
      T eb[4], dq[4];
      frag_finish(dd, raw_use, eb, dq);
#pragma unroll
      for (int v = 0; v < 4; ++v) dq[v] = (dq[v] + s14 * wrow_next(w, dq[v])) * k15;  // g0 + mu g1 | 0
      frag_load(rb, (unsigned)wu(w, (int)R(k >= MR_RIC_AHEAD ? k - MR_RIC_AHEAD : 0)), fp, raw_fill);  // unconditional: k < AHEAD re-read stage 0's record
      // X = P^ E^  (A fragment s: P^[c][4s+g])
      // two independent 2-MFMA accumulation chains (k = 0..7 | 8..15) instead of one 4-long
      // dependent chain: half the MFMA latency on the stage's critical path
      T dx[4] = {T(0), T(0), T(0), T(0)}, dx2[4] = {T(0), T(0), T(0), T(0)};
      wmfma(w, LP[c * LDS_LD + g], eb[0], dx);
      wmfma(w, LP[c * LDS_LD + 8 + g], eb[2], dx2);
      wmfma(w, LP[c * LDS_LD + 4 + g], eb[1], dx);  // (K-chunk 12..15 is zero)
#pragma unroll
      for (int v = 0; v < 4; ++v) dx[v] += dx2[v];
      // B fragments X[4s+g][c]
      T xb[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) xb[s] = dx[s];  // f64: register s already holds row g + 4s
      if constexpr (sizeof(T) == 4) wtranspose4(w, xb);  // f32: D rows 4g+v -> B rows 4s+g, in registers
      // Q = (H + delta I | g0 | g1) + E^T X
      {
        T dq2[4] = {T(0), T(0), T(0), T(0)};
        wmfma(w, eb[0], xb[0], dq);
        wmfma(w, eb[2], xb[2], dq2);
        wmfma(w, eb[1], xb[1], dq);  // (K-chunk 12..15 is zero)
#pragma unroll
        for (int v = 0; v < 4; ++v) dq[v] += dq2[v];
      }
      auto qat = [&](int a, int b) { return wbcast(w, dq[dreg(a)], dgrp(a) * 16 + b); };
      T Rh[6] = {qat(11, 11), qat(11, 12), qat(11, 13), qat(12, 12), qat(12, 13), qat(13, 13)};
      T L[6], iv[3];
      const bool piv_ok = chol3r(Rh, L, iv);  // checked every second stage (below)
      T w0[3] = {qat(11, 14), qat(12, 14), qat(13, 14)};
      lsolve3r(L, iv, w0);
      T wc[3] = {wshfl(w, dq[dreg(11)], dgrp(11) * 16 + c), wshfl(w, dq[dreg(12)], dgrp(12) * 16 + c),
                 wshfl(w, dq[dreg(13)], dgrp(13) * 16 + c)};
      lsolve3r(L, iv, wc);  // W[:, c]
      const T wv = wc[0] * sg[0] + wc[1] * sg[1] + wc[2] * sg[2];  // W[g][c] (0 for g = 3)
      T dw[4] = {T(0), T(0), T(0), T(0)};
      wmfma(w, wv, wv, dw);  // W^T W
      // gains: K[:, c] = -L^{-T} W[:, c], feed-forward k
      T kc[3] = {wc[0], wc[1], wc[2]}, k0[3] = {w0[0], w0[1], w0[2]};
      ltsolve3r(L, iv, kc);
      ltsolve3r(L, iv, k0);
      {  // branch-free gain stores (other lanes hit the discard slot): a loop free of divergent
         // branches keeps the waits for the prefetched operands exact across the back-edge
        // row a of K by lanes (0, c < 11), k[a] by lane (0, 11): one store per a
        const bool kcol = (g == 0) & (c < NX), kf0 = (g == 0) & (c == NX);
#pragma unroll
        for (int a = 0; a < NU; ++a) {
          const unsigned idx = kcol ? RCF::K + a * NX + c : (kf0 ? RCF::K0 + a : RCF::JUNK);
          rb.st(kcol ? -kc[a] : -k0[a], Rk, idx);
        }
      }
#pragma unroll
      for (int v = 0; v < 4; ++v) {  // branch-free: lanes without a target write their discard slot
        const T pv = dq[v] - dw[v];
        rb.st(pv, Rk, (unsigned)fp.st_p[v]);
        LP[fp.lp[v]] = pv;
      }
      wsync_lds(w);
      return piv_ok & noise_ok;
    };
    // Pivots are tested once per three stages, at the loop latch: a failed stage only costs the
    // next two, and the loop keeps one back-edge block (exact prefetch waits at the loop head).
    // Buffer roles rotate a -> c -> b -> a over the three unrolled steps.
    bool ok = true;
#if MR_RIC_AHEAD == 3
    // A/B option: gathers three stages ahead, four rotating buffers (a -> d -> c -> b -> a)
    for (int k = N - 1;; k -= 4) {
      ok = step(k, raw_a, raw_d) & ok;
      if (k == 0) break;
      ok = step(k - 1, raw_b, raw_a) & ok;
      if (k == 1) break;
      ok = step(k - 2, raw_c, raw_b) & ok;
      if (k == 2) break;
      ok = step(k - 3, raw_d, raw_c) & ok;
      if (k == 3) break;
      if (!wuni(w, ok)) return false;
    }
#else
    for (int k = N - 1;; k -= 3) {
      ok = step(k, raw_a, raw_c) & ok;
      if (k == 0) break;
      ok = step(k - 1, raw_b, raw_a) & ok;
      if (k == 1) break;
      ok = step(k - 2, raw_c, raw_b) & ok;
      if (k == 2) break;
      if (!wuni(w, ok)) return false;
    }
#endif
    if (!wuni(w, ok)) return false;
    wsync(w);  // records (P, p, K, k) visible to every lane
    return true;
  }


  // ---------------- sweep 3: forward substitution, slack/dual steps ----------------
  //   Sequential part: per stage, three lane groups share one 11-term dot with dx_k (gathered from
  //   lanes 0..10): [A | c] rows -> A dx_k + c, P_k rows -> the costate step, K_k rows -> du_k =
  //   K_k dx_k + k; then dx_{k+1} = A dx_k + c + B du_k (stage Jacobian from the record,
  //   no closed-loop map).  Then stage-parallel: slack / multiplier steps and the step limits.
  MR_SWEEP void forward(T& ap, T& ad, T& gphi) {
    MR_UNIFORM_P();
    MR_ASSUME_LDS_STATE();
#if MR_PHASE_CYCLES
    const unsigned long long tf0 = trace ? MR_CLOCK() : 0ull;
#endif
    const T mu = this->mu;
    const T tau = mr_max(T(0.99), T(1) - mu);
    T dz[NZS];
    for (int i = 0; i < NZS; ++i) dz[i] = T(0);
    {
      const int N = wu(this->w, this->N), ln = this->ln;  // N wave-uniform: the stage offsets are soffsets
      const Wv w = this->w;
      // the instance's workspace (stage fields, then the records) as one wave-uniform buffer
      const WBuf<T> wb(rc - (int64_t)SSF::NF * WL, (unsigned)WS_NU_OFF);
      auto R = [](int k) { return (unsigned)(SSF::NF * WL) + (unsigned)k * (unsigned)RC_STRIDE; };
      MR_LDS T* const LDX = lds + LDX_OFF;
      // One recursion step per stage k = 0..N with three lane groups sharing the same dot product
      // row . dx_k (dx_k gathered from lanes 0..10): group 0 (lanes 0..10) row i of [A | c] of the
      // stage map E^ -> (A dx_k + c)[i]; group 1 (lanes 16..26) row i of P_k -> the costate step
      // dnu_k[i] = P_k dx_k + p_k - nu_k (k >= 1); group 2 (lanes 32..34) row a of K_k ->
      // du_k[a] = K_k dx_k + k.  Then group 0 adds B du_k (du_k read from group 2):
      // dx_{k+1} = A dx_k + B du_k + c.  Every lane gathers its row from stage k's record (one
      // record, a few cache lines per load), instead of each lane reading its own stage's P and K
      // afterwards (a different cache line per lane and load).  Lanes without a row read the
      // record's zero slot; E^'s structural entries come from the record's constant slots.
      const int grp = ln >> 4, r = ln & 15;
      const bool g0r = (grp == 0) & (r < NX), g1r = (grp == 1) & (r < NX), g2r = (grp == 2) & (r < NU);
      const int r0 = g0r ? r : 0;
      int roff[NX], boff[NU], c0off;
#pragma unroll
      for (int j = 0; j < NX; ++j)
        roff[j] = g0r ? ehat_slot(r0, j, true)
                      : (g1r ? RCF::P + pidx(r, j) : (g2r ? RCF::K + r * NX + j : RCF::CZERO));
#pragma unroll
      for (int a = 0; a < NU; ++a) boff[a] = ehat_slot(r0, NX + a, g0r);
      c0off = g0r ? ehat_slot(r0, 14, true) : (g1r ? RCF::PV0 + r : (g2r ? RCF::K0 + r : RCF::CZERO));
      static_assert(3 * WL <= LP_OFF + 16 * LDS_LD, "du staging");
      // LDS target of each lane's step result (branch-free, one store): group 0 dx_{k+1}[r] at
      // LDX[(k + 1) 12 + r] (row N + 1 <= 64; N = 63: the discard slots), group 2 du_k[r] at
      // [LX_OFF + 3 k + r] (the Riccati tiles are dead here), the others their discard slot
      const int lbase = g0r ? LDX_OFF + 12 + r : (g2r ? LX_OFF + r : LJUNK_OFF + ln);
      const int lstep = g0r ? 12 : (g2r ? 3 : 0);
      T dxi = T(0);
      if (ln < NX) LDX[ln] = T(0);
      // Row gathers run two stages ahead in three rotating register sets, the loop unrolled by three
      // with one exit test per step at its end (uniform control, no copies of in-flight loads): the
      // waits for a set are exact vmcnt counts, not drains at the loop head.
      struct FwdRow {
        T rw[NX], bw[NU], c0;  // (the Riccati's p and k already carry mu)
      };
      auto fload = [&](int kk, FwdRow& f) {
        kk = kk < N ? kk : N;
        const unsigned ro = (unsigned)wu(w, (int)R(kk));
#pragma unroll
        for (int j = 0; j < NX; ++j) f.rw[j] = wb.ld(ro, (unsigned)roff[j]);
#pragma unroll
        for (int a = 0; a < NU; ++a) f.bw[a] = wb.ld(ro, (unsigned)boff[a]);
        f.c0 = wb.ld(ro, (unsigned)c0off);
      };
      auto fstep = [&](int k, const FwdRow& f) {
        T dxv[NX];
        wgather<T, NX>(w, dxi, dxv);
#if MR_FWD_TREE
        // the 11-term dot as three interleaved chains (critical path 4 FMAs + 2 adds, not 11)
        T a0 = f.c0, a1 = f.rw[1] * dxv[1], a2 = f.rw[2] * dxv[2];
        a0 += f.rw[0] * dxv[0];
#pragma unroll
        for (int j = 3; j < NX; j += 3) {
          a0 += f.rw[j] * dxv[j];
          if (j + 1 < NX) a1 += f.rw[j + 1] * dxv[j + 1];
          if (j + 2 < NX) a2 += f.rw[j + 2] * dxv[j + 2];
        }
        const T acc = (a0 + a1) + a2;
#else
        T acc = f.c0;
        for (int j = 0; j < NX; ++j) acc += f.rw[j] * dxv[j];
#endif
        // dx_{k+1} = (A dx_k + c) + B du_k on group 0, du_k from group 2 (lanes 32..34)
        T accx = acc;
#pragma unroll
        for (int a = 0; a < NU; ++a) accx += f.bw[a] * wbcast(w, acc, 32 + a);
        dxi = g0r ? accx : T(0);
        lds[lbase + lstep * k] = g0r ? accx : acc;
        const bool dn = g1r & (k >= 1 || !MR_KKT_RESTATED);  // k = 0: the initial-state rows' multiplier step
        if constexpr (SSL) {
          if (dn) ss[(SSF::DNU + r) * WL + k] = acc;
        } else {  // branch-free: other lanes write stage k's record discard slot
          wb.st(acc, (unsigned)k, dn ? (unsigned)(SSF::DNU + r) * WL : R(k) + RCF::JUNK - (unsigned)k);
        }
      };
      FwdRow fa, fb, fc;
      fload(0, fa);
      fload(1, fb);
      for (int k = 0;; k += 3) {
        fload(k + 2, fc);
        fstep(k, fa);
        if (k == N) break;
        fload(k + 3, fa);
        fstep(k + 1, fb);
        if (k + 1 == N) break;
        fload(k + 4, fb);
        fstep(k + 2, fc);
        if (k + 2 == N) break;
      }
      wsync_lds(w);
      if (ln <= N)
        for (int j = 0; j < NX; ++j) dz[j] = LDX[ln * 12 + j];
      if (ln < N)
        for (int a = 0; a < NU; ++a) dz[NX + a] = lds[LX_OFF + 3 * ln + a];
    }
#if MR_PHASE_CYCLES
    const unsigned long long tf1 = trace ? MR_CLOCK() : 0ull;
#endif
    // stage-parallel part
    T ap_l = T(1), ad_l = T(1), g_l = T(0);
    if (own()) {
      const int k = ln;
      MR_GLOBAL T* Rk = R(k);
      for (int i = 0; i < NZ; ++i) g_l += S(SSF::GL + i) * dz[i];
      T z[NZS];
      load_z(cur, z);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      row_values(k, z, e, d, act);
      T adz[NI];
#pragma unroll
      for (int r = 0; r < NROW; ++r) {
        const T v = row_c(r, dz);
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
      for (int i = 0; i < NZS; ++i) S(SSF::DZ + i) = dz[i];
      for (int j = 0; j < NI; ++j) {
        if (!act[j]) continue;
        T s = S(sf(cur) + j), lam = S(SSF::LAM + j);
        T ds = adz[j] + (d[j] - s);
        T dl = mu / s - lam - (lam / s) * ds;
        S(SSF::DS + j) = ds;
        S(SSF::DLAM + j) = dl;
        g_l -= mu * ds / s;
        if (ds < T(0)) ap_l = mr_min(ap_l, -tau * s / ds);
        if (dl < T(0)) ad_l = mr_min(ad_l, -tau * lam / dl);
      }
    }
    ap = wmin(w, ap_l);
    ad = wmin(w, ad_l);
    gphi = wsum(w, g_l);
#if MR_PHASE_CYCLES
    if (trace) { tsub[0] += tf1 - tf0; tsub[1] += MR_CLOCK() - tf1; }
#endif
  }

  // ---------------- sweep 3 of the restoration phase ----------------
  // The recursion is mr_solver.h Solver::forward with resto set, run wave-uniformly (every lane computes
  // the same dx, du, disturbance; lane k keeps stage k's), the record read with uniform addresses --
  // the restoration phase is entered by few instances for few iterations, so this sweep is written for
  // clarity rather than for the prefetch pipeline of forward().  Then stage-parallel: the relaxed rows'
  // and dynamics rows' steps (row_steps_r, dyn_steps_r), step limits, the directional derivative.
  MR_SWEEP void forward_resto(T& ap, T& ad, T& gphi) {
    MR_UNIFORM_P();
    MR_ASSUME_LDS_STATE();
    const T mu = this->mu, rho = cw()->rho;
    const T tau = mr_max(T(0.99), T(1) - mu);
    const int N = wu(w, this->N);
    const MR_GLOBAL T* cb = rc + (int64_t)RC_STRIDE * WL;
    T dx[NX], mydz[NZS], myw[6];
    for (int i = 0; i < NX; ++i) dx[i] = T(0);
    for (int i = 0; i < NZS; ++i) mydz[i] = T(0);
    for (int i = 0; i < 6; ++i) myw[i] = T(0);
    for (int k = 0; k <= N; ++k) {
      const MR_GLOBAL T* Rk = R(k);
      T du[NU] = {T(0), T(0), T(0)};
      if (k < N)
        for (int a = 0; a < NU; ++a) {
          T v = Rk[RCF::K0 + a];  // k (the Riccati's, mu already in)
          for (int j = 0; j < NX; ++j) v += Rk[RCF::K + a * NX + j] * dx[j];
          du[a] = v;
        }
      if (ln == k) {
        for (int i = 0; i < NX; ++i) mydz[i] = dx[i];
        for (int a = 0; a < NU; ++a) mydz[NX + a] = du[a];
      }
      if (k == N) break;
      T J[48], t[NX], tb[NX];
      for (int i = 0; i < 48; ++i) J[i] = Rk[RCF::J + i];
      apply_A(J, k, dx, t);
      apply_B(J, k, du, tb);
      for (int i = 0; i < NX; ++i) dx[i] = t[i] + tb[i] + Rk[RCF::C + i];
      // + the disturbance of the relaxed vehicle rows, w = -M^-1 (nu_y + gw)
      const MR_GLOBAL T* Rn = R(k + 1);
      T Pn[NP], sw[6], rhs[6], wv[6];
      for (int i = 0; i < NP; ++i) Pn[i] = Rn[RCF::P + i];
      for (int i = 0; i < 6; ++i) {
        T v = Rn[RCF::PV0 + i];  // p (the Riccati's, mu already in)
        for (int l = 0; l < NX; ++l) v += Pn[pidx(i, l)] * dx[l];
        rhs[i] = v + cb[(CSF::CGW0 + i) * WL + k] + mu * cb[(CSF::CGW1 + i) * WL + k];
        sw[i] = cb[(CSF::CSW + i) * WL + k];
      }
      noise_step(Pn, sw, rhs, wv);
      for (int i = 0; i < 6; ++i) dx[i] += wv[i];
      if (ln == k)
        for (int i = 0; i < 6; ++i) myw[i] = wv[i];
      // multiplier step dnu_{k+1} = P_{k+1} dx_{k+1} + p_{k+1} (correction form, eval_sweep)
      if (ln == k + 1)
        for (int i = 0; i < NX; ++i) {
          T v = Rn[RCF::PV0 + i];  // p (the Riccati's, mu already in)
          for (int l = 0; l < NX; ++l) v += Pn[pidx(i, l)] * dx[l];
          S(SSF::DNU + i) = v;  // correction form: the multiplier step itself
        }
    }
    T ap_l = T(1), ad_l = T(1), g_l = T(0);
    if (own()) {
      const int k = ln;
      T dz[NZS];
      for (int i = 0; i < NZS; ++i) dz[i] = mydz[i];
      for (int i = 0; i < NZ; ++i) g_l += S(SSF::GL + i) * dz[i];
      T z[NZS];
      load_z(cur, z);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      row_values(k, z, e, d, act);
      T adz[NI];
#pragma unroll
      for (int r = 0; r < NROW; ++r) {
        const T v = row_c(r, dz);
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
      for (int i = 0; i < NZS; ++i) S(SSF::DZ + i) = dz[i];
      for (int j = 0; j < NI; ++j) {
        if (!act[j]) continue;
        const T s = S(sf(cur) + j), lam = S(SSF::LAM + j);
        const T p = Cf(CSF::RP + j), n = Cf(CSF::RN + j), vp = Cf(CSF::RVP + j), vn = Cf(CSF::RVN + j);
        T ds, dl, dp, dn, dvp, dvn;
        row_steps_r(adz[j] + (d[j] - s - p + n), s, lam, p, n, vp, vn, rho, mu, ds, dp, dn, dl, dvp, dvn);
        Cf(CSF::RDP + j) = dp;
        Cf(CSF::RDN + j) = dn;
        Cf(CSF::RDVP + j) = dvp;
        Cf(CSF::RDVN + j) = dvn;
        Cf(CSF::RDY + j) = lam + dl - Cf(CSF::RY + j);  // eta - y
        S(SSF::DS + j) = ds;
        S(SSF::DLAM + j) = dl;
        g_l += (rho - mu / p) * dp + (rho - mu / n) * dn - mu * ds / s;
        if (ds < T(0)) ap_l = mr_min(ap_l, -tau * s / ds);
        if (dp < T(0)) ap_l = mr_min(ap_l, -tau * p / dp);
        if (dn < T(0)) ap_l = mr_min(ap_l, -tau * n / dn);
        if (dl < T(0)) ad_l = mr_min(ad_l, -tau * lam / dl);
        if (dvp < T(0)) ad_l = mr_min(ad_l, -tau * vp / dvp);
        if (dvn < T(0)) ad_l = mr_min(ad_l, -tau * vn / dvn);
      }
      if (k < N)
        for (int i = 0; i < 6; ++i) {
          const T p = Cf(CSF::CP + i), n = Cf(CSF::CN + i), vp = Cf(CSF::CVP + i), vn = Cf(CSF::CVN + i);
          T dp, dn, dvp, dvn;
          dyn_steps_r(myw[i], p, n, vp, vn, rho, mu, dp, dn, dvp, dvn);
          Cf(CSF::CDP + i) = dp;
          Cf(CSF::CDN + i) = dn;
          Cf(CSF::CDVP + i) = dvp;
          Cf(CSF::CDVN + i) = dvn;
          g_l += (rho - mu / p) * dp + (rho - mu / n) * dn;
          if (dp < T(0)) ap_l = mr_min(ap_l, -tau * p / dp);
          if (dn < T(0)) ap_l = mr_min(ap_l, -tau * n / dn);
          if (dvp < T(0)) ad_l = mr_min(ad_l, -tau * vp / dvp);
          if (dvn < T(0)) ad_l = mr_min(ad_l, -tau * vn / dvn);
        }
    }
    ap = wmin(w, ap_l);
    ad = wmin(w, ad_l);
    gphi = wsum(w, g_l);
    wsync(w);  // costate steps of every lane written
  }

  // ---------------- sweep 4: the filter line search (IPOPT backtracking, one SOC) ----------------
  // The lane's stage iterate, step, slacks and slack steps are loaded once; every trial point is
  // formed and measured in registers (one pass per trial: the trial's stage values, its dynamics
  // defect against the neighbour's trial state, three wave sums), and only the accepted point --
  // or the fallback point when none is acceptable -- is written to iterate buffer 1-cur.
  // Backtracking (same rules and order as IPOPT's filter line search, Waechter & Biegler 2006):
  // alpha = ap, ap/2, ... down to a_min; a second-order correction only after the first trial
  // (nls = 0) when it did not decrease theta; acceptance = theta_max, then the switching /
  // Armijo or sufficient-decrease test, then the filter.
  // a0: the first trial step (ap, or ap/2 when the watchdog backtracks from its stored point, nls0 = 1:
  // the full step was tried); ap: the fraction-to-boundary step (the fallback point's upper clamp)
  // RESTO: the restoration phase's line search (mr_solver.h trial() with resto set): the relaxations
  // p, n of the rows and of the vehicle dynamics rows move with the step; theta and phi of the
  // restoration NLP decide, the point's original theta / barrier objective go to the WaveCold state
  // (the restoration exit test); no second-order correction.
  template <bool RESTO>
  MR_SWEEP void line_search(T th, T ph, T gphi, T a0, T ap, T a_min, T th_pow, int nls0) {
    MR_UNIFORM_P();
    MR_ASSUME_LDS_STATE();
    const T s_phi = T(2.3), delta_sw = T(1), eta = T(1e-4), g_th = T(1e-5), g_ph = T(1e-5);
    const int nb = 1 - cur;
    const int k = ln;
    const int N = wu(w, this->N);  // wave-uniform: the SOC re-roll's lane index must be an SGPR
    T z[NZS], dz[NZS], s_c[NI], ds[NI];
    load_z(cur, z);
    for (int i = 0; i < NZS; ++i) dz[i] = own() ? S(SSF::DZ + i) : T(0);
    unsigned actm = 0u;  // active rows of this stage (depend on the stage only, not on the point)
#pragma unroll
    for (int r = 0; r < NROW; ++r) {
      int a;
      T lo, hi;
      row_bounds(P, I, k, r, a, lo, hi);
      actm |= (own() && a) ? (3u << (2 * r)) : 0u;
    }
    actm |= (own() && lane_active(P, k)) ? (3u << JL) : 0u;
    for (int j = 0; j < NI; ++j) {
      const bool a = (actm >> j) & 1u;
      s_c[j] = a ? S(sf(cur) + j) : T(1);
      ds[j] = a ? S(SSF::DS + j) : T(0);
    }
    // restoration: the relaxations and their steps (rows of this stage; vehicle rows of x_{k+1})
    T rp[NI], rn[NI], rdp[NI], rdn[NI], cp[6], cn[6], cdp[6], cdn[6], zr[NZS];
    T rho = T(0), zeta = T(0), mu_o = T(0);
    if constexpr (RESTO) {
      rho = cw()->rho;
      zeta = cw()->zeta;
      mu_o = cw()->mu_o;
      for (int j = 0; j < NI; ++j) {
        const bool a = (actm >> j) & 1u;
        rp[j] = a ? Cf(CSF::RP + j) : T(1);
        rn[j] = a ? Cf(CSF::RN + j) : T(1);
        rdp[j] = a ? Cf(CSF::RDP + j) : T(0);
        rdn[j] = a ? Cf(CSF::RDN + j) : T(0);
      }
      const bool dk = own() && k < N;
      for (int i = 0; i < 6; ++i) {
        cp[i] = dk ? Cf(CSF::CP + i) : T(1);
        cn[i] = dk ? Cf(CSF::CN + i) : T(1);
        cdp[i] = dk ? Cf(CSF::CDP + i) : T(0);
        cdn[i] = dk ? Cf(CSF::CDN + i) : T(0);
      }
      for (int i = 0; i < NZS; ++i) zr[i] = own() ? Cf(CSF::RZ + i) : T(0);
    }
    T zt[NZS], st[NI];
    // one trial point: zt, st (registers), theta, phi; false if a slack is not positive or a value is
    // not finite
    auto eval = [&](T alpha, bool soc, T& th_t, T& ph_t) -> bool {
      for (int i = 0; i < NZS; ++i) zt[i] = z[i] + alpha * dz[i];
      if (k == 0)
        for (int i = 0; i < NX; ++i) zt[i] = z[i];  // x_0 fixed
      if (k >= N) { zt[11] = zt[12] = zt[13] = T(0); }
      T zpl[NZS];
      for (int i = 0; i < NZS; ++i) zpl[i] = zt[i];
      if (soc) {
        // second-order correction: re-roll the shooting states through the dynamics (sequential)
        T xr[NX], myx[NX];
        for (int i = 0; i < NX; ++i) { xr[i] = wbcast(w, z[i], 0); myx[i] = xr[i]; }
        for (int kk = 0; kk < N; ++kk) {
          T zz[NZS];
          for (int i = 0; i < NX; ++i) zz[i] = xr[i];
          zz[11] = wbcast(w, zpl[11], kk);
          zz[12] = wbcast(w, zpl[12], kk);
          zz[13] = wbcast(w, zpl[13], kk);
          zz[14] = T(0);
          T xn[NX];
          faug<T, MODEL>(P, kk, zz, xn);
          for (int i = 0; i < NX; ++i) xr[i] = xn[i];
          if (ln == kk + 1)
            for (int i = 0; i < NX; ++i) myx[i] = xr[i];
        }
        if (k >= 1)
          for (int i = 0; i < NX; ++i) zt[i] = myx[i];
      }
      T ztn[NX];
      for (int i = 0; i < NX; ++i) ztn[i] = wnext(w, zt[i]);
      T th_l = T(0), f_l = T(0), lg_l = T(0), lgr_l = T(0), tho_l = T(0), fo_l = T(0);
      int ok_l = 1;
      if (own()) {
        Err<T> e, ep;
        errors(I, zt[0], zt[1], zt[6], e, false);
        T d[NI], dp[NI];
        int act[NI];
        row_values(k, zt, e, d, act);
        if (soc) {
          errors(I, zpl[0], zpl[1], zpl[6], ep, false);
          int actp[NI];
          row_values(k, zpl, ep, dp, actp);
        }
        for (int j = 0; j < NI; ++j) {
          st[j] = s_c[j];
          if (!((actm >> j) & 1u)) continue;
          T sj = s_c[j] + alpha * ds[j];
          if (soc) sj += d[j] - dp[j];
          if (!(sj > T(0))) ok_l = 0;
          st[j] = sj;
          lg_l += mr_log(sj > T(0) ? sj : T(1));
          if constexpr (RESTO) {
            const T pt = rp[j] + alpha * rdp[j], nt = rn[j] + alpha * rdn[j];
            if (!(pt > T(0)) || !(nt > T(0))) ok_l = 0;
            th_l += mr_abs(d[j] - sj - pt + nt);
            tho_l += mr_abs(d[j] - sj);
            lgr_l += mr_log(pt > T(0) ? pt : T(1)) + mr_log(nt > T(0) ? nt : T(1));
            f_l += rho * (pt + nt);
          } else {
            th_l += mr_abs(d[j] - sj);
          }
        }
        if constexpr (RESTO) {
          f_l += prox_term(I, k, N, zt, zr, zeta, (T*)nullptr, (T*)nullptr);
          fo_l += stage_cost(P, I, k, zt, e, sc, (T*)nullptr, (T*)nullptr);
        } else {
          f_l += stage_cost(P, I, k, zt, e, sc, (T*)nullptr, (T*)nullptr);
        }
        if (k < N && !soc) {
          T xn[NX];
          faug<T, MODEL>(P, k, zt, xn);
          if constexpr (RESTO) {
            for (int i = 0; i < NX; ++i) {
              T r = xn[i] - ztn[i];
              tho_l += mr_abs(r);
              if (i < 6) {  // the relaxed vehicle rows
                const T pt = cp[i] + alpha * cdp[i], nt = cn[i] + alpha * cdn[i];
                if (!(pt > T(0)) || !(nt > T(0))) ok_l = 0;
                r += nt - pt;
                lgr_l += mr_log(pt > T(0) ? pt : T(1)) + mr_log(nt > T(0) ? nt : T(1));
                f_l += rho * (pt + nt);
              }
              th_l += mr_abs(r);
            }
          } else {
            for (int i = 0; i < NX; ++i) th_l += mr_abs(xn[i] - ztn[i]);
          }
        }
      }
      th_t = wsum(w, th_l);
      const T fv = wsum(w, f_l), lg = wsum(w, lg_l);
      int ok = wmin(w, ok_l);
      ph_t = fv - mu * lg;
      if constexpr (RESTO) {
        ph_t = fv - mu * (lg + wsum(w, lgr_l));
        cw()->tho = wsum(w, tho_l);  // the point as the original problem sees it (restoration exit test)
        cw()->pho = wsum(w, fo_l) - mu_o * lg;
      }
      if (!(th_t == th_t) || !(ph_t == ph_t)) ok = 0;
      return wuni(w, ok != 0);
    };
    T alpha = a0;
    int nls = nls0, pass = 0, ntr = 0, nsoc = 0;
    bool accepted = false, ftype = false, rej_filter = false;
    // backtracking ends below a_min, or below 1e-30: a_min is 0 when theta is (and may flush to 0 in
    // fp32), and halving alpha to 0 would never leave the loop.  No acceptable step: IPOPT would enter
    // its restoration phase; this solver takes the shortest tried step (never past the
    // fraction-to-boundary step, so the slacks stay positive) -- the fallback point.
    bool fallback = !(alpha >= a_min && alpha >= T(1e-30));
    if (fallback) alpha = mr_min(mr_max(alpha, a_min), ap);
    for (;;) {
      const bool soc = pass == 1;
      T th_t, ph_t;
      bool ok = eval(alpha, soc, th_t, ph_t);
      ntr++;
      nsoc += soc ? 1 : 0;
      if (fallback) { ftype = false; break; }
      if (ok) ok = th_t <= theta_max;
      if (ok) {
        const bool sw = gphi < T(0) && alpha * mr_exp(s_phi * mr_log(-gphi)) > delta_sw * th_pow;
        if (th <= theta_min && sw) {
          ok = ph_t <= ph + eta * alpha * gphi + T(1e-14) * mr_abs(ph);
          ftype = true;
        } else {
          ok = th_t <= (T(1) - g_th) * th || ph_t <= ph - g_ph * th + T(1e-14) * mr_abs(ph);
          ftype = false;
        }
      }
      // the filter last (IPOPT's order), so a rejection by the filter itself is known for the reset
      // heuristic
      if (ok && !filter_ok(th_t, ph_t)) { ok = false; rej_filter = true; }
      if (wuni(w, ok)) { accepted = true; break; }
      if (!RESTO && pass == 0 && nls == 0 && th_t >= th) { pass = 1; continue; }  // second-order correction
      pass = 0;
      alpha *= T(0.5);
      nls++;
      if (!(alpha >= a_min && alpha >= T(1e-30))) {
        fallback = true;
        alpha = mr_min(mr_max(alpha, a_min), ap);
      }
    }
    if (own()) {  // the chosen point
      for (int j = 0; j < NI; ++j)
        if ((actm >> j) & 1u) S(sf(nb) + j) = st[j];
      for (int i = 0; i < NZS; ++i) S(zf(nb) + i) = zt[i];
      if constexpr (RESTO) {  // the relaxations move in place (their step is applied once, here)
        if (accepted) {
          for (int j = 0; j < NI; ++j)
            if ((actm >> j) & 1u) {
              Cf(CSF::RP + j) = rp[j] + alpha * rdp[j];
              Cf(CSF::RN + j) = rn[j] + alpha * rdn[j];
            }
          if (k < N)
            for (int i = 0; i < 6; ++i) {
              Cf(CSF::CP + i) = cp[i] + alpha * cdp[i];
              Cf(CSF::CN + i) = cn[i] + alpha * cdn[i];
            }
        }
      }
    }
    res_alpha = alpha;
    res_flags = (accepted ? 1 : 0) | (ftype ? 2 : 0) | (rej_filter ? 4 : 0);
    res_nls = nls;
    res_ntr = ntr;
    res_nsoc = nsoc;
  }

  MR_HD bool filter_ok(T th, T ph) const {
    for (int i = 0; i < FMAX; ++i)
      if (i < nfilt && th >= fth(i) && ph >= fph(i)) return false;
    return true;
  }
  MR_HD void filter_add(T th, T ph) {
    if (nfilt < FMAX) {
      for (int i = 0; i < FMAX; ++i)
        if (i == nfilt) { fth(i) = th; fph(i) = ph; }
      nfilt++;
    } else {
      for (int i = 0; i < FMAX - 1; ++i) { fth(i) = fth(i + 1); fph(i) = fph(i + 1); }
      fth(FMAX - 1) = th;
      fph(FMAX - 1) = ph;
    }
  }

  MR_HD T lane_violation() const {
    MR_UNIFORM_P();
    T v = T(0);
    if (P.lane && own() && ln >= 1) v = S(zf(cur) + 14);
    return wmax(w, v);
  }

  // ---------------- watchdog snapshot (lane = stage) ----------------
  MR_SWEEP void wd_save() {
    MR_ASSUME_LDS_STATE();
    if (own()) {
      for (int i = 0; i < NZS; ++i) { Cf(CSF::WZ + i) = S(zf(cur) + i); Cf(CSF::WDZ + i) = S(SSF::DZ + i); }
      for (int j = 0; j < NI; ++j) {
        Cf(CSF::WSL + j) = S(sf(cur) + j); Cf(CSF::WLAM + j) = S(SSF::LAM + j);
        Cf(CSF::WDS + j) = S(SSF::DS + j); Cf(CSF::WDLAM + j) = S(SSF::DLAM + j);
      }
      for (int i = 0; i < NX; ++i) { WNUd(i) = NUd(i); Cf(CSF::WDNU + i) = S(SSF::DNU + i); }
    }
    wsync(w);
  }
  MR_SWEEP void wd_restore() {
    MR_ASSUME_LDS_STATE();
    if (own()) {
      for (int i = 0; i < NZS; ++i) { S(zf(cur) + i) = Cf(CSF::WZ + i); S(SSF::DZ + i) = Cf(CSF::WDZ + i); }
      for (int j = 0; j < NI; ++j) {
        S(sf(cur) + j) = Cf(CSF::WSL + j); S(SSF::LAM + j) = Cf(CSF::WLAM + j);
        S(SSF::DS + j) = Cf(CSF::WDS + j); S(SSF::DLAM + j) = Cf(CSF::WDLAM + j);
      }
      for (int i = 0; i < NX; ++i) { NUd(i) = WNUd(i); S(SSF::DNU + i) = Cf(CSF::WDNU + i); }
    }
    wsync(w);
  }

  // ---------------- the restoration phase (mr_solver.h Solver::resto_enter / resto_done / resto_exit) ----------------
  MR_SWEEP void resto_enter(T th, T ph) {
    MR_UNIFORM_P();
    MR_ASSUME_LDS_STATE();
    const T g_th = T(1e-5), g_ph = T(1e-5), rho = T(RESTO_RHO);
    auto* C = cw();
    filter_add((T(1) - g_th) * th, ph - g_ph * th);
    C->onfilt = nfilt;
    for (int i = 0; i < 2 * FMAX; ++i) C->ofilt[i] = filt[i];
    C->mu_o = mu;
    C->th_entry = th;
    C->delta_last_o = delta_last;
    C->theta_max_o = theta_max;
    C->theta_min_o = theta_min;
    C->rho = rho;
    const T mu_r = mr_max(mu, pr_max);
    T th_rows_l = T(0);
    if (own()) {
      const int k = ln;
      T z[NZS];
      load_z(cur, z);
      for (int i = 0; i < NZS; ++i) Cf(CSF::RZ + i) = z[i];
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      row_values(k, z, e, d, act);
      for (int j = 0; j < NI; ++j) {
        T p = T(1), n = T(1);
        if (act[j]) {
          const T s = S(sf(cur) + j), c = d[j] - s;
          th_rows_l += mr_abs(c);
          resto_pn(c, mu_r, rho, p, n);
          S(SSF::LAM + j) = mu_r / s;  // the slacks' bound duals restart at complementarity with mu_R
        }
        Cf(CSF::RP + j) = p;
        Cf(CSF::RN + j) = n;
        Cf(CSF::RVP + j) = mu_r / p;
        Cf(CSF::RVN + j) = mu_r / n;
        Cf(CSF::RDP + j) = T(0); Cf(CSF::RDN + j) = T(0); Cf(CSF::RDVP + j) = T(0); Cf(CSF::RDVN + j) = T(0);
        Cf(CSF::RY + j) = T(0);  // the rows' equality multipliers start at 0
        Cf(CSF::RDY + j) = T(0);
        S(SSF::DLAM + j) = T(0);
      }
      for (int i = 0; i < NX; ++i) { NUd(i) = 0.0; S(SSF::DNU + i) = T(0); }
      if (k < N)
        for (int i = 0; i < 6; ++i) {  // the vehicle rows start satisfied too (p - n = F - x')
          T p, n;
          const T c = R(k)[RCF::C + i];
          th_rows_l += mr_abs(c);
          resto_pn(c, mu_r, rho, p, n);
          Cf(CSF::CP + i) = p;
          Cf(CSF::CN + i) = n;
          Cf(CSF::CVP + i) = mu_r / p;
          Cf(CSF::CVN + i) = mu_r / n;
          Cf(CSF::CDP + i) = T(0); Cf(CSF::CDN + i) = T(0); Cf(CSF::CDVP + i) = T(0); Cf(CSF::CDVN + i) = T(0);
        }
    }
    const T th_rows = wsum(w, th_rows_l);
    alpha_p = alpha_d = T(0);
    mu = mu_r;
    C->resto = 1;
    nfilt = 0;
    delta_last = T(0);
    const T th_r = mr_max(theta - th_rows, T(0));  // relaxed rows start satisfied: the definitional rows only
    theta_max = T(1e4) * mr_max(T(1), th_r);
    theta_min = T(1e-4) * mr_max(T(1), th_r);
    wsync(w);
  }
  MR_HD bool resto_done() {  // the accepted restoration step's point, seen by the original problem
    auto* C = cw();
    const T tho = C->tho, pho = C->pho;
    bool ok = tho <= T(RESTO_KAPPA) * C->th_entry;
    for (int i = 0; i < FMAX; ++i)
      if (i < C->onfilt && tho >= C->ofilt[i] && pho >= C->ofilt[FMAX + i]) ok = false;
    return wuni(w, ok);
  }
  MR_SWEEP void resto_exit() {
    MR_ASSUME_LDS_STATE();
    auto* C = cw();
    const T mu_o = C->mu_o;
    if (own()) {
      for (int j = 0; j < NI; ++j) {
        const T s = S(sf(cur) + j), lam0 = S(SSF::LAM + j), lam = lam0 + alpha_d * S(SSF::DLAM + j);
        T lnew = mu_o / s;
        if (mr_abs(lnew - lam) > T(RESTO_MULT_RESET)) lnew = T(1);
        S(SSF::LAM + j) = lam0 == T(0) ? T(0) : lnew;  // inactive slots stay 0
        S(SSF::DLAM + j) = T(0);
      }
      for (int i = 0; i < NX; ++i) { NUd(i) = 0.0; S(SSF::DNU + i) = T(0); }
    }
    alpha_p = alpha_d = T(0);
    mu = mu_o;
    nfilt = C->onfilt;
    for (int i = 0; i < 2 * FMAX; ++i) filt[i] = C->ofilt[i];
    theta_max = C->theta_max_o;
    theta_min = C->theta_min_o;
    delta_last = C->delta_last_o;
    C->resto = 0;
    wsync(w);
  }

  // ---------------- the IPM loop (wave-uniform control) ----------------
  MR_HD SolveOut solve() {
    MR_UNIFORM_P();
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
    int it = 0;
    // diagnostics of the trace instance: shader cycles per phase and call counts (MR_PHASE_CYCLES
    // builds only -- the counters stay live across every sweep call, so the product build has none)
#if MR_PHASE_CYCLES
    unsigned long long cyc[8] = {0, 0, 0, 0, 0, 0, 0, 0}, t0 = 0, tstart = trace ? MR_CLOCK() : 0ull;
#define MR_T0() (t0 = trace ? MR_CLOCK() : 0ull)
#define MR_T1(slot) (cyc[slot] += trace ? MR_CLOCK() - t0 : 0ull)
#define MR_CNT(slot) (cyc[slot]++)
#else
#define MR_T0() ((void)0)
#define MR_T1(slot) ((void)0)
#define MR_CNT(slot) ((void)0)
#endif
    for (it = 0;; ++it) {
#if MR_DEVICE_BUILD && MR_PRIO_ITER > 0
      // long solves: raise the wave's issue priority over the partner wave on its SIMD, so the
      // batch's slowest instances (which set its makespan) are not slowed by the short ones
      if (it == MR_PRIO_ITER) __builtin_amdgcn_s_setprio(3);
#endif
      // wave-uniform mode of this iteration: the original problem, or its restoration phase
      const bool rs = wuni(w, cw()->resto != 0);
      MR_T0();
      if (rs) eval_sweep<true>(mu_prev); else eval_sweep<false>(mu_prev);
      MR_T1(0);
      T kkt = kkt_error(T(0));
      if (!(kkt == kkt) || !(fval == fval)) { out.status = 3; break; }
      if (rs) {
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
        cw()->in_wd = 0;
        cw()->wd_short = 0;
      }
      T delta = T(0);
      bool first = true, fact_ok = false;
      MR_T0();
      for (int tries = 0; tries < 60; ++tries) {
        MR_CNT(6);
#if MR_PHASE_CYCLES
        const unsigned long long tr0 = trace ? MR_CLOCK() : 0ull;
        const bool rok = rs ? riccati<true>(delta, mu) : riccati<false>(delta, mu);
        if (trace && !rok) { tsub[4] += MR_CLOCK() - tr0; tsub[5] += 1; }
        if (rok) { fact_ok = true; break; }
#else
        if (rs ? riccati<true>(delta, mu) : riccati<false>(delta, mu)) { fact_ok = true; break; }
#endif
        if (first) {
          delta = delta_last == T(0) ? T(1e-4) : mr_max(T(1e-20), delta_last / T(3));
          first = false;
        } else {
          delta *= (delta_last == T(0) ? T(100) : T(8));
        }
        if (delta > T(1e40)) break;
      }
      MR_T1(1);
      if (!fact_ok) { out.status = 3; break; }
      if (delta > T(0)) delta_last = delta;
      T &ap = res_ap, &ad = res_ad, &gphi = res_gphi;
      MR_T0();
      if (rs) forward_resto(ap, ad, gphi); else forward(ap, ad, gphi);
      MR_T1(2);
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
      if (rs) {  // a restoration-phase step: its own filter, no watchdog, no second-order correction
        MR_T0();
        line_search<true>(th, ph, gphi, ap, ap, a_min, th_pow, 0);
        MR_T1(3);
        if (!(res_flags & 1)) { out.status = 3; break; }  // IPOPT: restoration failed
        if (!(res_flags & 2)) filter_add((T(1) - g_th) * th, ph - g_ph * th);
        if (trace && ln == 0 && it < trace_cap - 2) {
          double* tr = trace + 8 * it;
          tr[0] = (double)kkt; tr[1] = (double)mu; tr[2] = (double)res_alpha; tr[3] = (double)ad;
          tr[4] = (double)delta; tr[5] = (double)th; tr[6] = (double)cw()->tho; tr[7] = -200.0 - res_nls;
        }
        alpha_p = res_alpha;
        alpha_d = ad;
        mu_prev = mu;
        cur = 1 - cur;
        wsync(w);
        if (resto_done()) {
          resto_exit();
          mu_prev = mu;
          cw()->in_wd = 0;
          cw()->wd_short = 0;
          acc_count = 0;
          filt_rej_iters = 0;
        }
        continue;
      }
#if MR_WD_TRIGGER > 0
      // IPOPT's watchdog (mr_solver.h, same rule): after watchdog_shortened_iter_trigger successive
      // shortened steps store the iterate and direction, take full steps tentatively, judged against the
      // stored point; after watchdog_trial_iter_max without an acceptable one, back to the stored point
      if (!cw()->in_wd && cw()->wd_short >= MR_WD_TRIGGER) {
        wd_save();
        auto* C = cw();
        C->wd_th = th; C->wd_ph = ph; C->wd_gphi = gphi; C->wd_ap = ap; C->wd_ad = ad; C->wd_amin = a_min;
        C->wd_thpow = th_pow;
        C->in_wd = 1;
        C->wd_trial = 0;
      }
#endif
      bool take_anyway = false;
      MR_T0();
      if (wuni(w, cw()->in_wd != 0)) {
        auto* C = cw();
        line_search<false>(C->wd_th, C->wd_ph, C->wd_gphi, ap, ap, ap, C->wd_thpow, 0);
        if (res_flags & 1) {
          C->in_wd = 0;
          C->wd_short = 0;
          th = C->wd_th;  // the filter entry is the watchdog point's (the acceptor's reference)
          ph = C->wd_ph;
        } else if (++C->wd_trial <= MR_WD_TRIAL_MAX) {
          take_anyway = true;  // the line search stored the plain full step (its fallback point at ap)
        } else {
          // back to the watchdog point: its iterate and direction, a regular backtracking line search
          // that skips the full step
          wd_restore();
          C->in_wd = 0;
          C->wd_short = 0;
          th = C->wd_th; ph = C->wd_ph; gphi = C->wd_gphi; ap = C->wd_ap; ad = C->wd_ad; a_min = C->wd_amin;
          th_pow = C->wd_thpow;
          line_search<false>(th, ph, gphi, T(0.5) * ap, ap, a_min, th_pow, 1);
        }
      } else {
        line_search<false>(th, ph, gphi, ap, ap, a_min, th_pow, 0);
      }
      MR_T1(3);
#if MR_PHASE_CYCLES
      cyc[4] += res_ntr;
      cyc[5] += res_nsoc;
#endif
      const T alpha = res_alpha;
      const bool accepted = (res_flags & 1) && !take_anyway, ftype = res_flags & 2, rej_filter = res_flags & 4;
      const int nls = res_nls;
      // no acceptable step at an infeasible point: the restoration phase (from the next iteration on)
      if (!accepted && !take_anyway && pr_max > P.tol) {
        resto_enter(th, ph);
        mu_prev = mu;
        cw()->in_wd = 0;
        cw()->wd_short = 0;
        acc_count = 0;
        if (trace && ln == 0 && it < trace_cap - 2) {
          double* tr = trace + 8 * it;
          tr[0] = (double)kkt; tr[1] = (double)mu; tr[2] = 0.0; tr[3] = 0.0;
          tr[4] = (double)delta; tr[5] = (double)th; tr[6] = (double)ph; tr[7] = -300.0;
        }
        continue;
      }
      // no acceptable step at a point feasible to the tolerance: the shortest tried step (the line
      // search's fallback point); after MR_LS_FAIL_MAX such iterations in a row the solve stops
      ls_fail = (accepted || take_anyway) ? 0 : ls_fail + 1;
      if (ls_fail >= MR_LS_FAIL_MAX) { out.status = 3; break; }
      if (!take_anyway) cw()->wd_short = (accepted && alpha < ap) ? cw()->wd_short + 1 : 0;
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
      if (!(ftype && accepted) && !take_anyway) filter_add((T(1) - g_th) * th, ph - g_ph * th);
      if (trace && ln == 0 && it < trace_cap - 2) {
        double* tr = trace + 8 * it;
        tr[0] = (double)kkt; tr[1] = (double)mu; tr[2] = (double)alpha; tr[3] = (double)ad;
        tr[4] = (double)delta; tr[5] = (double)th; tr[6] = (double)ph;
        tr[7] = (double)(take_anyway ? -100 - cw()->wd_trial : (accepted ? nls : -1));
      }
      alpha_p = alpha;
      alpha_d = ad;
      mu_prev = mu;
      cur = 1 - cur;
      wsync(w);  // new iterate buffer written by every lane before the next evaluation
    }
    out.iters = it;
#undef MR_T0
#undef MR_T1
#undef MR_CNT
#if MR_PHASE_CYCLES
    if (trace && ln == 0 && trace_cap >= 2) {  // last row: cycles eval, riccati, forward, trial, #trials, #soc, #factorisations, total
      double* tr = trace + 8 * (trace_cap - 1);
      for (int q = 0; q < 7; ++q) tr[q] = (double)cyc[q];
      tr[7] = (double)(trace ? MR_CLOCK() - tstart : 0ull);
      double* tr2 = trace + 8 * (trace_cap - 2);  // sub-phases: forward seq/par, eval stage/reduce, failed factorisations (cycles, count)
      for (int q = 0; q < 6; ++q) tr2[q] = (double)tsub[q];
    }
#endif
    if (trace && ln == 0 && it < trace_cap - 2) {
      double* tr = trace + 8 * it;
      tr[0] = (double)out.kkt; tr[1] = (double)fval; tr[2] = (double)theta; tr[3] = (double)stat_max;
      tr[4] = (double)pr_max; tr[5] = (double)sc; tr[6] = (double)mu; tr[7] = 1000.0 + out.status;
    }
    return out;
  }
};

// Per-instance driver: lane `w.lane` of the wave that solves instance i of the batch.
// Ish: where the instance constants live -- the workgroup's LDS on the device (every lane writes
// the same values), so the sweeps read them with LDS latency instead of private-stack latency;
// nullptr = a local (host build).
template <typename Solver>
MR_HD void run_instance(Solver& S, const mr_inputs& in, const mr_outputs& out, int64_t B, int64_t i, int N,
                        double X0, double Y0, double s0, Wv w);

template <typename T, int MODEL, bool SSL = false, bool OBJ_LDS = false>
MR_HD void solve_instance_wave(const MR_CONST ProbParams<T>& P, const mr_inputs& in, const mr_outputs& out, int64_t B,
                               int64_t i, MR_GLOBAL T* ws, MR_LDS T* lds, Wv w,
                               typename SSPtr<T, SSL>::type ssp = nullptr, Inst<T>* Ish = nullptr,
                               void* solver_slots = nullptr, MR_LDS T* filt_sh = nullptr) {
  const int N = P.N;
  Inst<T> Iloc;
  Inst<T>& I = Ish ? *Ish : Iloc;
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
#if MR_DEVICE_BUILD
  __builtin_amdgcn_s_waitcnt(0xc07f);  // lgkmcnt(0): the LDS copy is written before any lane reads it
  __builtin_amdgcn_wave_barrier();
#endif
  typedef WaveSolver<T, MODEL, SSL> Solver;
  const typename SSPtr<T, SSL>::type ssv = SSL ? ssp : (typename SSPtr<T, SSL>::type)ws;
  if constexpr (OBJ_LDS) {
    // the solver object (a per-lane copy of the wave-uniform iteration state) in the caller's LDS
    // slots: the non-inlined sweeps reach it through `this`, which would otherwise point into the
    // private stack, whose loads take Infinity-Cache / HBM latency
    Solver* Sp = new ((char*)solver_slots + (size_t)w.lane * sizeof(Solver)) Solver(P, I, w, ws, lds, ssv);
#if MR_DEVICE_BUILD
    Sp->filt = filt_sh;
#endif
    run_instance(*Sp, in, out, B, i, N, X0, Y0, s0, w);
  } else {
    Solver S(P, I, w, ws, lds, ssv);
    run_instance(S, in, out, B, i, N, X0, Y0, s0, w);
  }
}

// The reference's dual (control/MPC.py:171: sol.value(opti.lam_g)) from the stage-wise multipliers, in
// Opti row order (include/mpcracing.h lam_g).  Derivation: the solver's Lagrangian is
// sc*f + sum nu_{k+1}.(F(x_k, u_k) - x_{k+1}) - sum lam.d, Opti's is f + lam_g.g with g = X_i - f(X_{i-1},
// U_{i-1}), so the dynamics rows are -nu/sc; every inequality row of the reference is a row of the
// restatement (Delta-S = the u[2] box, rate rows via the previous-control state p, the i = 0 wrap rows via
// the frozen copy w at k = N-1), lam_g = (lam_upper - lam_lower)/sc; S_0 and X_{:,0} follow from the
// reference's stationarity in those variables: lam_S0 = lam_ds(1), lam_X0 = A_0^T lam_dyn(1).
template <typename Solver>
MR_HD void write_lam_g(Solver& S, const mr_outputs& out, int64_t B, int64_t i, int N, Wv w) {
  typedef decltype(S.mu) T;
  const int k = w.lane;
  const double isc = 1.0 / (double)S.sc;
  const int rows = 13 * N + 9;
  auto put = [&](int row, double v) { out.lam_g[(int64_t)row * B + i] = v; };
  auto lam = [&](int j) { return (double)S.S(SSF::LAM + j); };
  double nu1[NX];
  for (int q = 0; q < NX; ++q) nu1[q] = wshfl(w, S.own() ? S.NUd(q) : 0.0, 1);
  const double ds1 = wshfl(w, S.own() && k < N ? (lam(5) - lam(4)) * isc : 0.0, 0);
  if (k >= 1 && k <= N)
    for (int q = 0; q < 6; ++q) put(7 + 7 * (k - 1) + q, -S.NUd(q) * isc);
  if (k < N) {
    put(7 + 7 * k + 6, (lam(5) - lam(4)) * isc);  // Delta-S row of i = k + 1 (u[2] box of stage k)
    const int b = 7 + 7 * N + 6 * k;
    put(b + 0, lam(1) * isc);    // U[0,k] < d_max
    put(b + 1, -lam(0) * isc);   // U[0,k] > min_throttle
    put(b + 2, lam(3) * isc);    // U[1,k] < max_steer
    put(b + 3, -lam(2) * isc);   // U[1,k] > min_steer
    if (k >= 1) {
      put(b + 4, (lam(7) - lam(6)) * isc);
      put(b + 5, (lam(9) - lam(8)) * isc);
    }
    if (k == N - 1) {  // i = 0 rate rows U[:,0] - U[:,N-1]: the frozen-copy rows at stage N-1
      const int b0 = 7 + 7 * N;
      put(b0 + 4, N >= 2 ? (lam(11) - lam(10)) * isc : 0.0);
      put(b0 + 5, N >= 2 ? (lam(13) - lam(12)) * isc : 0.0);
    }
  }
  if (k == 0) {
    put(0, ds1);  // S_0 == s0
    MR_GLOBAL T* R0 = S.R(0);
    T J[48];
    double at[NX];
    for (int q = 0; q < 48; ++q) J[q] = R0[RCF::J + q];
    apply_At(J, 0, nu1, at);
    for (int q = 0; q < 6; ++q) put(1 + q, -at[q] * isc);  // X_{q,0} == state0
    put(rows - 2, S.I.has_thr0 ? (lam(7) - lam(6)) * isc : NAN);
    put(rows - 1, S.I.has_steer0 ? (lam(9) - lam(8)) * isc : NAN);
  }
}

template <typename Solver>
MR_HD void run_instance(Solver& S, const mr_inputs& in, const mr_outputs& out, int64_t B, int64_t i, int N,
                        double X0, double Y0, double s0, Wv w) {
  typedef decltype(S.mu) T;
  const MR_CONST ProbParams<T>& P = S.P;
  const Inst<T>& I = S.I;
  if (out.trace && out.trace_instance == i) { S.trace = out.trace; S.trace_cap = out.trace_cap; }
  S.init(in.u_init ? in.u_init + i : nullptr, B);
  SolveOut r = S.solve();
  const T viol = S.lane_violation();
  // outputs (the ret tuple of control/MPC.py:166-171), lane k writes stage k, global coordinates
  if (S.own()) {
    const int k = w.lane;
    T z[NZS];
    S.load_z(S.cur, z);
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
  if (out.lam_g) write_lam_g(S, out, B, i, N, w);
  (void)viol;
  if (w.lane == 0) {
    out.status[i] = r.status;
    out.iters[i] = r.iters;
    if (out.obj) out.obj[i] = r.obj - (double)P.lambda_s * s0;
    if (out.kkt) out.kkt[i] = r.kkt;
  }
}

}  // namespace mr
