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
#include <type_traits>

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
// trace rows reserved at the end of a trace buffer: the final status record's slack row and the cycle rows
// (MR_PHASE_CYCLES: rows trace_cap - 1 .. trace_cap - 4), never overwritten by per-iteration rows
#define MR_TRACE_RESERVED (MR_PHASE_CYCLES ? 4 : 2)

namespace mr {

struct SSF {
  enum {
    Z0 = 0, Z1 = Z0 + NZS, DZ = Z1 + NZS, S0 = DZ + NZS, S1 = S0 + NI, LAM = S1 + NI, DLAM = LAM + NI,
    DS = DLAM + NI, DNU = DS + NI, GL = DNU + NX,
    Y = GL + NZ, DY = Y + NI,  // IPOPT's row multipliers y_d and their step (mr_solver.h WF::Y)
    NF = DY + NI
  };
};
// The sparse pattern of the inertia correction's slack shift (mr_solver.h HD): sum over a stage's rows of
// a a^T -- box / rate / wrap rows on (7..13), the lane row on (0, 1, 6); packed upper (i, j) -> slot
MR_HD constexpr int hd_slot(int i, int j) {
  return (i == 7 && j == 7) ? 0 : (i == 7 && j == 11) ? 1 : (i == 8 && j == 8) ? 2 : (i == 8 && j == 12) ? 3
       : (i == 9 && j == 9) ? 4 : (i == 9 && j == 11) ? 5 : (i == 10 && j == 10) ? 6 : (i == 10 && j == 12) ? 7
       : (i == 11 && j == 11) ? 8 : (i == 12 && j == 12) ? 9 : (i == 13 && j == 13) ? 10 : (i == 0 && j == 0) ? 11
       : (i == 0 && j == 1) ? 12 : (i == 0 && j == 6) ? 13 : (i == 1 && j == 1) ? 14 : (i == 1 && j == 6) ? 15
       : (i == 6 && j == 6) ? 16 : -1;
}
constexpr int NHD = 17;
// Stage record (stage-major, RC_STRIDE words per stage): the evaluation sweep's stage QP data
// (Jacobian, defect, Hessian, gradients), then the Riccati sweep's outputs.
struct RCF {
  enum {
    J = 0, C = J + 48, H = C + NX, G0 = H + NHC, G1 = G0 + NZ,  // H: the 48 structural entries (hcidx)
    HD = G1 + NZ, GD = HD + NHD,  // the slack shift's pattern (hd_slot) and sum a (d - s) (delta_s)
    P = GD + NZ, PV0 = P + NP, K = PV0 + NX, K0 = K + NU * NX,
    LQ = K0 + NU,  // Q_uu's Cholesky factor: L10, L20, L21 and the reciprocal pivots (SOC re-solves)
    CONE = LQ + 6, CZERO, SELP, SEL0,  // constants 1, 0, [k > 0], [k == 0] (written once per solve)
    JUNK, NF                           // discard slot of the branch-free stores (any lane)
  };
};
constexpr int RC_STRIDE = (RCF::NF + 15) / 16 * 16;  // words; 16-word (64 B) multiple (304)
static_assert(RCF::NF <= RC_STRIDE, "record");
static_assert(RC_STRIDE == 304, "record stride (DESIGN.md §3)");
// Cold per-stage fields [f][64] after the records: touched only by the watchdog (its snapshot of the
// iterate and the search direction) and the restoration phase (the relaxations p, n of the rows and
// of the 6 vehicle dynamics rows, their bound duals and steps, the rows' equality multipliers y, the
// reference point z_R, the condensed disturbance weights of the Riccati sweep) -- same meaning as the
// WF fields of mr_solver.h's scalar solver.
struct CSF {
  enum {
    WZ = 0, WSL = WZ + NZS, WLAM = WSL + NI, WDZ = WLAM + NI, WDS = WDZ + NZS, WDLAM = WDS + NI,
    WDNU = WDLAM + NI, WY = WDNU + NX, WDY = WY + NI,
    // second-order corrections: right-hand sides c_soc / r_soc, the direction, the vector pass (g_soc,
    // costate p, feed-forward k); the restoration entry point; IPOPT's stored acceptable iterate
    SC = WDY + NI, SR = SC + NX, SG = SR + NI, SPV = SG + NZ, SK0 = SPV + NX, SDZ = SK0 + NU, SDS = SDZ + NZS,
    SDLAM = SDS + NI, SDY = SDLAM + NI, SDNU = SDY + NI, RS0 = SDNU + NX, RLAM = RS0 + NI, AZ = RLAM + NI,
    ASL = AZ + NZS, ALAM = ASL + NI, AY = ALAM + NI,  // the stored acceptable point's slacks and multipliers
    RP = AY + NI, RN = RP + NI, RVP = RN + NI, RVN = RVP + NI, RDP = RVN + NI, RDN = RDP + NI, RDVP = RDN + NI,
    RDVN = RDVP + NI, RY = RDVN + NI, RDY = RY + NI, RZ = RDY + NI,
    CP = RZ + NZS, CN = CP + 6, CVP = CN + 6, CVN = CVP + 6, CDP = CVN + 6, CDN = CDP + 6, CDVP = CDN + 6,
    CDVN = CDVP + 6, CSW = CDVN + 6, CGW0 = CSW + 6, CGW1 = CGW0 + 6,
    // a trial point's constraint values captured for the second-order correction that may follow it
    // (LS_CAP): the rows' (d - s) (NI) and the dynamics defects (NX), 0 where none is accumulated
    CTR = CGW1 + 6, CTC = CTR + NI,
    SJUNK = CTC + NX,  // discard slot of the SOC chains' lanes without a component
    // the filter's entries beyond the FMAX in LDS (mr_solver.h FCAP): [bank][theta | phi][FOVF] fields, entry
    // FMAX + 64 q + l in lane l of field q; bank 0 the original problem's, bank 1 the restoration phase's
    FOV = SJUNK + 1,
    NF = FOV + 4 * FOVF
  };
};
// The dynamics rows' multipliers nu (and their watchdog and acceptable-point snapshots) in fp64 whatever
// the solve precision, [3][NX][64] doubles after the cold fields: eval_sweep forms the stationarity residual and the
// Riccati right-hand side from them in fp64 (the correction form, see there).
constexpr int64_t WS_NU_OFF = (int64_t)SSF::NF * WL + (int64_t)RC_STRIDE * WL + (int64_t)CSF::NF * WL;  // words
template <typename T>
#ifndef MR_WS_PAD
#define MR_WS_PAD 0  // developer check (tools/build_flag_variants.py wspad): unused words after each instance's workspace
#endif
MR_HD constexpr int64_t ws_words() { return WS_NU_OFF + 3 * NX * WL * (int64_t)(sizeof(double) / sizeof(T)) + MR_WS_PAD; }

// Wave-uniform state of the watchdog and the restoration phase: one copy per wavefront next to the
// line-search filter (LDS on the device), every lane writing the same values -- not in the per-lane
// solver objects, whose LDS footprint sets the occupancy.
template <typename T>
struct WaveCold {
  int resto, in_wd, wd_short, wd_trial, onfilt, mrow, have_acc, tiny, resto_first, in_soft, soft_count;
  T rho, zeta, mu_o, th_entry, delta_last_o, theta_max_o, theta_min_o, tho, pho;
  T fo, fo_cur;  // restoration: the original (scaled) objective of the last trial point / of the current iterate
  T wd_th, wd_ph, wd_gphi, wd_ap, wd_ad, wd_amin, wd_thpow;
  // evaluation aggregates beyond the solver object's (mr_solver.h Solver): primal infeasibility of the
  // equality rows, bound violation of the rows, |y|_1, the damped slacks' sum, the original problem's
  // primal infeasibility in the restoration phase; the accepted factorisation's delta
  T pr_eq, viol, y1, lins, pr_o, delta_it;
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
MR_HD void row_bounds_raw(const ProbParams<T>& P, const Inst<T>& I, int k, int r, int& act, T& lo, T& hi);
// the bounds as IPOPT uses them (bound_relax_factor, mr_solver.h relax_amt)
template <typename T>
MR_HD void row_bounds(const ProbParams<T>& P, const Inst<T>& I, int k, int r, int& act, T& lo, T& hi) {
  row_bounds_raw(P, I, k, r, act, lo, hi);
  lo -= relax_amt(lo);
  hi += relax_amt(hi);
}
template <typename T>
MR_HD void row_bounds_raw(const ProbParams<T>& P, const Inst<T>& I, int k, int r, int& act, T& lo, T& hi) {
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
// a_l for lane l (l >= 5: a5) by lane-constant bit masks -- no branches, exact for any bit pattern
template <typename T>
MR_HD T pick6(int l, T a0, T a1, T a2, T a3, T a4, T a5) {
  typedef typename std::conditional<sizeof(T) == 4, unsigned, unsigned long long>::type U;
  const U z = U(0), o = ~U(0);
  const U r = (__builtin_bit_cast(U, a0) & (l == 0 ? o : z)) | (__builtin_bit_cast(U, a1) & (l == 1 ? o : z)) |
              (__builtin_bit_cast(U, a2) & (l == 2 ? o : z)) | (__builtin_bit_cast(U, a3) & (l == 3 ? o : z)) |
              (__builtin_bit_cast(U, a4) & (l == 4 ? o : z)) | (__builtin_bit_cast(U, a5) & (l >= 5 ? o : z));
  return __builtin_bit_cast(T, r);
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
  static constexpr int kModel = MODEL;
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
  MR_HD WaveCold<T>* cw() const { return const_cast<WaveCold<T>*>(&sh_store.cold); }
#endif
  int nfilt;
  T stat_max, pr_max, theta, slam_max, slam_min, nu1, lam1, fval, logs;
  int me, mi;
  // out-parameters of the non-inlined sweeps: members, so they land in the object's LDS slot
  // rather than in the caller's private stack (a scratch round trip after every call)
  T res_ap, res_ad, res_gphi, res_alpha, res_th, res_ph, res_atest;
  int res_flags, res_nls, res_ntr, res_nsoc;
  double* trace = nullptr;
  int trace_cap = 0;
#if MR_PHASE_CYCLES
  unsigned long long tsub[24] = {};  // diagnostics: sub-phase cycles of the trace instance
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
  MR_HD MR_GLOBAL double& ANUd(int i) const { return nub()[(2 * NX + i) * WL + ln]; }  // acceptable-point copy
  MR_HD auto& fth(int i) const { return filt[i]; }
  MR_HD auto& fph(int i) const { return filt[FMAX + i]; }
  MR_HD MR_GLOBAL T* R(int k) const { return rc + (int64_t)k * RC_STRIDE; }
  MR_HD bool own() const { return ln <= N; }

  MR_HD int zf(int b) const { return b ? SSF::Z1 : SSF::Z0; }
  MR_HD int sf(int b) const { return b ? SSF::S1 : SSF::S0; }
  MR_HD int nxt() const { return (ln + 1) & (WL - 1); }

  MR_HD void load_z(int b, T* z) const {
    for (int i = 0; i < NZS; ++i) {
      const T v = S(zf(b) + i);  // (unconditional: all loads in flight together)
      z[i] = own() ? v : T(0);
    }
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
      // IPOPT's slack push (mr_solver.h Solver::init): one-sided box rows at least 1e-2 max(1, |b|)
      // inside; a two-sided row's slack s projected into [lo + p_L, hi - p_U]
      T t[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) t[j] = T(1);
#pragma unroll
      for (int r = 0; r <= NROW; ++r) {
        const int j0 = r < NROW ? 2 * r : JL;
        if (!act[j0]) continue;
        int ra;
        T lo, hi, c;
        if (r < NROW) {
          row_bounds(P, I, k, r, ra, lo, hi);
          c = row_c(r, my);
        } else {
          hi = I.max_err + relax_amt(I.max_err);
          lo = -hi;
          c = e.eC;
        }
        if (r < 2) {
          t[j0] = mr_max(d[j0], T(1e-2) * mr_max(T(1), mr_abs(lo)));
          t[j0 + 1] = mr_max(d[j0 + 1], T(1e-2) * mr_max(T(1), mr_abs(hi)));
        } else {
          const T rng = hi - lo;
          const T pL = mr_min(T(1e-2) * mr_max(T(1), mr_abs(lo)), T(1e-2) * rng);
          const T pU = mr_min(T(1e-2) * mr_max(T(1), mr_abs(hi)), T(1e-2) * rng);
          const T sv = mr_min(mr_max(c, lo + pL), hi - pU);
          t[j0] = sv - lo;
          t[j0 + 1] = hi - sv;
        }
      }
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        S(SSF::S0 + j) = t[j];
        S(SSF::LAM + j) = act[j] ? T(1) : T(0);
        S(SSF::DLAM + j) = T(0);
        S(SSF::Y + j) = T(0);
        S(SSF::DY + j) = T(0);
        if (act[j] && yslot(j)) th += mr_abs(d[j] - t[j]);
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
    C->have_acc = 0;
    C->tiny = 0;
    C->resto_first = 0;
    C->in_soft = 0;
    C->soft_count = 0;
    C->delta_it = T(0);
  }

  // IPOPT's least-square multipliers at the initial point (mr_solver.h Solver::ls_init): the stage QP
  // min 1/2 sx' M sx + g' sx s.t. the linearised dynamics (c = 0), M = I on the reference's variables +
  // sum over rows a a^T, g = grad f - sum a rs (rs = v_L - v_U), by the Riccati and forward sweeps; the
  // costates are the dynamics rows' multipliers, y_d = a.sx - rs; both zero if one exceeds 1000.
  MR_SWEEP void ls_record() {
    MR_UNIFORM_P();
    MR_ASSUME_LDS_STATE();
    if (own()) {
      const int k = ln;
      T z[NZS];
      load_z(cur, z);
      MR_GLOBAL T* Rk = R(k);
      T H[NH], g[NZ];
      for (int i = 0; i < NH; ++i) H[i] = T(0);
      for (int i = 0; i < NZ; ++i) g[i] = T(0);
      if (k < N) {
        T Hd[36], fx[6], J[48], nz[NX];
        for (int i = 0; i < NX; ++i) nz[i] = T(0);
        Dyn<T, MODEL>::fjh(P, z, z + NX, nz, fx, J, Hd);
        for (int i = 0; i < 48; ++i) Rk[RCF::J + i] = J[i];
      }
      for (int i = 0; i < NZ; ++i)
        if (delta_var(i)) H[hidx(i, i)] = T(1);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      stage_cost(P, I, k, z, e, sc, g, (T*)nullptr);
      T d[NI];
      int act[NI];
      row_values(k, z, e, d, act);
#pragma unroll
      for (int r = 0; r < NROW; ++r) {
        if (!act[2 * r]) continue;
        const T nrow = r < 2 ? T(2) : T(1);
        const T rs = r < 2 ? S(SSF::LAM + 2 * r) - S(SSF::LAM + 2 * r + 1) : T(0);
#pragma unroll
        for (int a = 0; a < RN(r); ++a) {
          g[RI(r, a)] -= T(RS(a)) * rs;
#pragma unroll
          for (int bb = a; bb < RN(r); ++bb) H[hidx(RI(r, a), RI(r, bb))] += nrow * T(RS(a)) * T(RS(bb));
        }
      }
      if (lane_active(P, k)) {
        const int id3[3] = {0, 1, 6};
        for (int a = 0; a < 3; ++a)
          for (int bb = a; bb < 3; ++bb) H[hidx(id3[a], id3[bb])] += e.gC[a] * e.gC[bb];
      }
#pragma unroll
      for (int q = 0; q < NHC; ++q) Rk[RCF::H + q] = H[HCT.p[q]];
      for (int i = 0; i < NZ; ++i) { Rk[RCF::G0 + i] = g[i]; Rk[RCF::G1 + i] = T(0); Rk[RCF::GD + i] = T(0); }
      // the slack shift's pattern of the box / rate / wrap rows (eval_sweep hd): fixed by the stage's rows,
      // written once here; the evaluation sweep rewrites it only where the lane row adds its gC gC^T
      {
        T hdc[NHD];
#pragma unroll
        for (int q = 0; q < NHD; ++q) hdc[q] = T(0);
#pragma unroll
        for (int r = 0; r < NROW; ++r) {
          if (!act[2 * r]) continue;
          const T hdw = r < 2 ? T(2) : T(1);
#pragma unroll
          for (int a = 0; a < RN(r); ++a)
#pragma unroll
            for (int bb = 0; bb < RN(r); ++bb) {
              const int ia = RI(r, a), ib = RI(r, bb);
              if (ia <= ib) hdc[hd_slot(ia, ib)] += hdw * T(RS(a)) * T(RS(bb));
            }
        }
        for (int q = 0; q < NHD; ++q) Rk[RCF::HD + q] = hdc[q];
      }
      for (int i = 0; i < NX; ++i) Rk[RCF::C + i] = T(0);
    }
    wsync(w);
  }
  MR_SWEEP void ls_finish() {
    MR_UNIFORM_P();
    MR_ASSUME_LDS_STATE();
    const T big = T(IP_MULT_INIT_MAX);
    int ok_l = 1;
    T yv[NI];
    for (int j = 0; j < NI; ++j) yv[j] = T(0);
    if (own()) {
      const int k = ln;
      T z[NZS], dz[NZS];
      load_z(cur, z);
      for (int i = 0; i < NZS; ++i) dz[i] = S(SSF::DZ + i);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      row_values(k, z, e, d, act);
#pragma unroll
      for (int r = 0; r < NROW; ++r) {
        if (!act[2 * r]) continue;
        const T adz = row_c(r, dz);
        if (r < 2) {
          yv[2 * r] = adz - S(SSF::LAM + 2 * r);
          yv[2 * r + 1] = adz + S(SSF::LAM + 2 * r + 1);
        } else {
          yv[2 * r] = adz;
        }
      }
      if (lane_active(P, k)) yv[JL] = e.gC[0] * dz[0] + e.gC[1] * dz[1] + e.gC[2] * dz[6];
      for (int j = 0; j < NI; ++j) ok_l &= mr_abs(yv[j]) <= big ? 1 : 0;
      for (int i = 0; i < NX; ++i)
        if (i < 6 || (k == 0 && i == 6)) ok_l &= mr_abs(S(SSF::DNU + i)) <= big ? 1 : 0;
    }
    const bool ok = wall(w, ok_l != 0);
    if (own()) {
      for (int i = 0; i < NX; ++i) {
        NUd(i) = ok ? (double)S(SSF::DNU + i) : 0.0;
        S(SSF::DNU + i) = T(0);
      }
      for (int j = 0; j < NI; ++j) {
        S(SSF::Y + j) = ok ? yv[j] : T(0);
        S(SSF::DY + j) = T(0);
        S(SSF::DS + j) = T(0);
        S(SSF::DLAM + j) = T(0);
      }
    }
    wsync(w);
  }
  MR_HD void ls_init() {
    cw()->delta_it = T(0);
    ls_record();
    if (!riccati<false>(T(0), T(0))) return;
    T ap, ad, gphi;
    forward(ap, ad, gphi);
    ls_finish();
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
      f_l = T(0), lg_l = T(0), preq_l = T(0), viol_l = T(0), y1_l = T(0), lin_l = T(0), pro_l = T(0);
    int mi_l = 0, mrow_l = 0;
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
        for (int i = 0; i < NX; ++i) pro_l = mr_max(pro_l, mr_abs(c[i]));
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
          preq_l = mr_max(preq_l, mr_abs(c[i]));
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
        viol_l = mr_max(viol_l, -d[j]);
        if (oneslot(j)) lin_l += s;
        if (yslot(j)) pro_l = mr_max(pro_l, mr_abs(rd));
        if constexpr (!RESTO) {  // an IPOPT row (y-slot): its multiplier y_d, lazily stepped with alpha_p
          if (yslot(j)) {
            const T y = S(SSF::Y + j) + alpha_p * S(SSF::DY + j);
            S(SSF::Y + j) = y;
            y_j[j] = y;
            y1_l += mr_abs(y);
            mrow_l += 1;
            pr_l = mr_max(pr_l, mr_abs(rd));
            th_l += mr_abs(rd);
          }
        }
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
          pr_l = mr_max(pr_l, mr_abs(rd));
          th_l += mr_abs(rd);
        }
      }
      T hd[NHD], gd[NZ];  // the slack shift's pattern and its right-hand side (delta_s), regular phase only
#pragma unroll
      for (int q = 0; q < NHD; ++q) hd[q] = T(0);
#pragma unroll
      for (int q = 0; q < NZ; ++q) gd[q] = T(0);
      if constexpr (RESTO) {
#pragma unroll
        for (int r = 0; r < NROW; ++r) {
          if (!act[2 * r]) continue;
          T sig_sum = T(0), gsc0 = T(0), gsc1 = T(0), lamdiff = T(0);
#pragma unroll
          for (int sd = 0; sd < 2; ++sd) {
            int j = 2 * r + sd;
            T sgn = sd == 0 ? T(1) : T(-1);
            sig_sum += sg_j[j];
            gsc0 += sgn * c0_j[j];
            gsc1 += sgn * c1_j[j];
            lamdiff += sgn * y_j[j];
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
          const int id3[3] = {0, 1, 6};
          const T sig0 = sg_j[JL], sig1 = sg_j[JL + 1];
          const T lamdiff = y_j[JL] - y_j[JL + 1];
          const T gz0 = c0_j[JL] - c0_j[JL + 1], gz1 = c1_j[JL] - c1_j[JL + 1];
          int q = 0;
          for (int a = 0; a < 3; ++a) {
            g0[id3[a]] += e.gC[a] * gz0;
            g1[id3[a]] += e.gC[a] * gz1;
            st[id3[a]] -= lamdiff * e.gC[a];
            for (int bb = a; bb < 3; ++bb, ++q)
              H[hidx(id3[a], id3[bb])] += (sig0 + sig1) * e.gC[a] * e.gC[bb] - lamdiff * e.hC[q];
          }
        }
      } else {
        // IPOPT's rows condensed into the stage QP (mr_solver.h Solver::eval_sweep): H += Sigma_s a a^T,
        // g0 += a Sigma_s (d - s), g1 += a (grad_s phi)/mu (+-kappa_d on a one-sided row), the Lagrangian
        // gradient y a, the slack stationarity -y - v_L + v_U; hd / gd: delta_s's a a^T and a (d - s)
#pragma unroll
        for (int r = 0; r < NROW; ++r) {
          const int j0 = 2 * r, j1 = j0 + 1;
          if (!act[j0]) continue;
          T hs, gr0, gr1, ys, hdw, gdw;
          if (r < 2) {  // two one-sided rows
            const T sg0 = lam_j[j0] / s_j[j0], sg1 = lam_j[j1] / s_j[j1];
            hs = sg0 + sg1;
            gr0 = sg0 * (d[j0] - s_j[j0]) - sg1 * (d[j1] - s_j[j1]);
            gr1 = (-T(1) / s_j[j0] + T(IP_KAPPA_D)) + (T(1) / s_j[j1] - T(IP_KAPPA_D));
            ys = y_j[j0] + y_j[j1];
            hdw = T(2);
            gdw = (d[j0] - s_j[j0]) - (d[j1] - s_j[j1]);
            st_l = mr_max(st_l, mr_max(mr_abs(-y_j[j0] - lam_j[j0]), mr_abs(-y_j[j1] + lam_j[j1])));
          } else {  // one two-sided row
            hs = lam_j[j0] / s_j[j0] + lam_j[j1] / s_j[j1];
            gr0 = hs * (d[j0] - s_j[j0]);
            gr1 = -T(1) / s_j[j0] + T(1) / s_j[j1];
            ys = y_j[j0];
            hdw = T(1);
            gdw = d[j0] - s_j[j0];
            st_l = mr_max(st_l, mr_abs(-y_j[j0] - lam_j[j0] + lam_j[j1]));
          }
#pragma unroll
          for (int a = 0; a < RN(r); ++a) {
            const T sa = T(RS(a));
            g0[RI(r, a)] += sa * gr0;
            g1[RI(r, a)] += sa * gr1;
            st[RI(r, a)] += ys * sa;
            gd[RI(r, a)] += sa * gdw;
#pragma unroll
            for (int bb = 0; bb < RN(r); ++bb) {
              const int ia = RI(r, a), ib = RI(r, bb);
              if (ia <= ib) {
                H[hidx(ia, ib)] += hs * sa * T(RS(bb));
                hd[hd_slot(ia, ib)] += hdw * sa * T(RS(bb));
              }
            }
          }
        }
        if (lane_active(P, k)) {  // the lane row: two-sided, nonlinear in (X, Y, S)
          const int id3[3] = {0, 1, 6};
          const T hs = lam_j[JL] / s_j[JL] + lam_j[JL + 1] / s_j[JL + 1];
          const T gr0 = hs * (d[JL] - s_j[JL]), gr1 = -T(1) / s_j[JL] + T(1) / s_j[JL + 1];
          const T ys = y_j[JL];
          st_l = mr_max(st_l, mr_abs(-ys - lam_j[JL] + lam_j[JL + 1]));
          int q = 0;
          for (int a = 0; a < 3; ++a) {
            g0[id3[a]] += e.gC[a] * gr0;
            g1[id3[a]] += e.gC[a] * gr1;
            st[id3[a]] += ys * e.gC[a];
            gd[id3[a]] += e.gC[a] * (d[JL] - s_j[JL]);
            for (int bb = a; bb < 3; ++bb, ++q) {
              H[hidx(id3[a], id3[bb])] += hs * e.gC[a] * e.gC[bb] + ys * e.hC[q];
              hd[hd_slot(id3[a], id3[bb])] += e.gC[a] * e.gC[bb];
            }
          }
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
#if !MR_DEVICE_BUILD
      for (int a = 0; a < NZ; ++a)  // host build: the structural pattern holds (tests run every model / phase)
        for (int bb = a; bb < NZ; ++bb)
          if (!h_struct(a, bb) && H[hidx(a, bb)] != T(0)) {
            fprintf(stderr, "mr_wave.h: stage Hessian entry (%d, %d) outside h_struct\n", a, bb);
            abort();
          }
#endif
      // the structural entries only, contiguous (48 words instead of 105: the record is written back by
      // whole lines, so skipped zeros inside the packed triangle saved nothing -- a compact layout does)
#pragma unroll
      for (int q = 0; q < NHC; ++q) rbe.st(H[HCT.p[q]], 0u, Rk + RCF::H + q);
      for (int i = 0; i < NZ; ++i) {
        rbe.st(T((double)g0[i] + dd[i]), 0u, Rk + RCF::G0 + i);
        rbe.st(g1[i], 0u, Rk + RCF::G1 + i);
      }
      if constexpr (!RESTO) {  // the slack shift (delta_s) enters the regular phase's factorisations only
        for (int i = 0; i < NZ; ++i) rbe.st(gd[i], 0u, Rk + RCF::GD + i);
        // its pattern is the rows' constant one (ls_record) unless the lane row adds gC gC^T
        if (lane_active(P, k))
          for (int q = 0; q < NHD; ++q) rbe.st(hd[q], 0u, Rk + RCF::HD + q);
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
    {
      auto* C = cw();
      const T preq = wmax(w, preq_l);
      pr_max = mr_max(preq, wmax(w, pr_l));
      const T vio = wmax(w, viol_l), y1v = wsum(w, y1_l), lin = wsum(w, lin_l), pro = wmax(w, pro_l);
      const int mrw = wsum(w, mrow_l);
      C->pr_eq = preq;
      C->viol = vio;
      C->y1 = y1v;
      C->lins = lin;
      C->pr_o = pro;
      C->mrow = mrw;
    }
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
    (void)te0; (void)te1;  // (tsub[2..3] carry forward_soc's chain / stage-parallel split)
#endif
  }

  // IPOPT's error measures (mr_solver.h Solver: s_d, s_c, nlp_error, barrier_error, converged, acceptable)
  MR_HD T s_d() { return mr_max(T(100), (nu1 + cw()->y1 + lam1) / T(me + cw()->mrow + (mi > 0 ? mi : 1))) / T(100); }
  MR_HD T s_c() const { return mr_max(T(100), lam1 / T(mi > 0 ? mi : 1)) / T(100); }
  MR_HD T compl_err(T m) const {
    if (mi == 0) return T(0);
    return mr_max(mr_abs(slam_max - m), mr_abs(m - slam_min));
  }
  MR_HD T nlp_error(bool rs) {
    const T pr = rs ? pr_max : mr_max(cw()->pr_eq, cw()->viol);
    return mr_max(mr_max(stat_max / s_d(), pr), compl_err(T(0)) / s_c());
  }
  MR_HD T barrier_error(T m) { return mr_max(mr_max(stat_max / s_d(), pr_max), compl_err(m) / s_c()); }
  MR_HD T kkt_error(T m) { return barrier_error(m); }
  MR_HD bool converged(T err) {
    MR_UNIFORM_P();
    if (!(err <= P.tol)) return false;
    return stat_max / sc <= T(IP_DUAL_INF_TOL) && mr_max(cw()->pr_eq, cw()->viol) <= T(IP_CONSTR_VIOL_TOL) &&
           compl_err(T(0)) / sc <= T(IP_COMPL_INF_TOL);
  }
  MR_HD bool acceptable(T err) {
    MR_UNIFORM_P();
    if (!(err <= P.acc_tol)) return false;
    return stat_max / sc <= T(IP_ACC_DUAL_INF) && mr_max(cw()->pr_eq, cw()->viol) <= T(IP_ACC_CONSTR_VIOL) &&
           compl_err(T(0)) / sc <= T(IP_ACC_COMPL);
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
  static constexpr int NGATHER = 12;
  struct FragPlan {
    int off[NGATHER];  // record offsets: data entries, or the record's constant slots (CONE, CZERO, SELP, SEL0);
                       // 8..11: the slack shift's entry of each D register (delta_s: HD, or GD in column 14)
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
    constexpr HCInv hci = make_hcinv();
    fp.dlt = 0u;
#pragma unroll
    for (int s = 0; s < 4; ++s) fp.off[s] = ehat_slot(4 * s + g, c, true);
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const int a = drow(g, v);
      const int a_ = a < NZ ? a : 0;
      const int hc = (a < NZ && c < NZ) ? hci.c[hidx(a_, c)] : -1;
      fp.off[4 + v] = a < NZ ? (c < NZ ? (hc >= 0 ? RCF::H + hc : RCF::CZERO)
                                        : (c == 14 ? RCF::G0 + a_ : RCF::G1 + a_))
                             : RCF::CZERO;
      if (a < NZ && a == c && delta_var(a)) fp.dlt |= 1u << v;
      {
        const int lo_ = a < c ? a : c, hi_ = a < c ? c : a;
        const int hs = (a < NZ && c < NZ) ? hd_slot(lo_, hi_) : -1;
        fp.off[8 + v] = hs >= 0 ? RCF::HD + hs : ((a < NZ && c == 14) ? RCF::GD + a_ : RCF::CZERO);
      }
      // outputs of D register v: packed-upper P | p (column 14) to the record; the whole tile of P^
      // (both triangles as the product computes them, one LDS write per register) to LDS
      const int junk_r = RCF::JUNK, junk_l = LJUNK_OFF - LP_OFF + lane;  // lp index from LP
      const bool ax = a < NX, sq = ax & (c < NX), up = sq & (a <= c);
      const bool c14 = ax & (c == 14);
      fp.st_p[v] = up ? RCF::P + pidx(a, c) : (c14 ? RCF::PV0 + a : junk_r);
      fp.lp[v] = sq ? a * LDS_LD + c : (c14 ? a * LDS_LD + 11 : junk_l);
    }
  }
  // DS: the slack shift's gathers (8..11) only when delta > 0 (a delta = 0 factorisation skips them)
  template <bool DS>
  static MR_HD void frag_load(const WBuf<T>& rb, unsigned ro, const FragPlan& fp, T* raw) {
#pragma unroll
    for (int q = 0; q < (DS ? NGATHER : 8); ++q) raw[q] = rb.ld(ro, (unsigned)fp.off[q]);
  }
  // operands straight from the gathered words (constants come from the record's constant slots); the
  // inertia correction: delta on the reference's variables (dd) and delta_s = delta on the slacks (delta x
  // the gathered slack-shift entry)
  template <bool DS>
  static MR_HD void frag_finish(const T* dd, T delta, const T* raw, T* eb, T* hc) {
#pragma unroll
    for (int s = 0; s < 4; ++s) eb[s] = raw[s];
#pragma unroll
    for (int v = 0; v < 4; ++v) hc[v] = raw[4 + v] + dd[v] + (DS ? delta * raw[8 + v] : T(0));
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
  // registers), Y = L^-1 [P_v. | p_v + gw0 + mu gw1] (lane c < 12: column c, to the LX scratch
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
    // 12 columns: the 11 states and the right-hand side (mu folded in, column 11); the tile's column 12
    // is not part of the wave Riccati's record
    const int c = l < 12 ? l : 0;
    D col[6];
    for (int i = 0; i < 6; ++i) col[i] = (D)LP[i * LDS_LD + c] + (c == 11 ? gw0[i] + (D)mu * gw1[i] : 0.0);
    lsolve6(L, col);
    if (l < 12)
      for (int a = 0; a < 6; ++a) LX[a * 16 + l] = col[a];
    wsync_lds(w);
    for (int e = l; e < NX * 12; e += WL) {
      const int i = e / 12, j = e - 12 * (e / 12);
      D v = (D)LP[i * LDS_LD + j];
      for (int a = 0; a < 6; ++a) v -= LX[a * 16 + i] * LX[a * 16 + j];
      LP[i * LDS_LD + j] = (T)v;
    }
    wsync_lds(w);
    return true;
  }

  // DS: delta > 0 in the regular phase (the slack shift delta_s = delta enters); false for delta = 0 and in
  // the restoration phase, whose records carry no slack-shift data
  template <bool RESTO, bool DS = false>
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
    constexpr HCInv hci = make_hcinv();
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
    frag_load<DS>(rb, R(N - 1), fp, raw_a);
    frag_load<DS>(rb, R(N >= 2 ? N - 2 : 0), fp, raw_b);
    {  // terminal cost-to-go: P_N = H_N,xx + delta I, p_N = g_N.  Branch-free (lanes >= NX write
       // discard slots), so at least as many memory ops follow the first prefetch on this path as
       // on the loop back-edge and the wait at the loop head stays exact.
      const unsigned Rn = R(N);
      const bool row = l < NX;
      const int lr = row ? l : 0, jl = RCF::JUNK, jd = LJUNK_OFF - LP_OFF + l;
      T hv[NX], hdv[NX];  // all loads ahead of the stores (the compiler cannot disambiguate H from P)
#pragma unroll
      for (int j = 0; j < NX; ++j) {
        hv[j] = rb.ld(Rn, hci.c[hidx(lr, j)] >= 0 ? RCF::H + hci.c[hidx(lr, j)] : RCF::CZERO);
        const int hs = hd_slot(lr < j ? lr : j, lr < j ? j : lr);
        hdv[j] = DS ? rb.ld(Rn, hs >= 0 ? RCF::HD + hs : RCF::CZERO) : T(0);
      }
      const T p0 = rb.ld(Rn, RCF::G0 + lr) + (DS ? delta * rb.ld(Rn, RCF::GD + lr) : T(0)), p1 = rb.ld(Rn, RCF::G1 + lr);
#pragma unroll
      for (int j = 0; j < NX; ++j) {
        const T v = hv[j] + delta * hdv[j] + (l == j && delta_var(j) ? delta : T(0));
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
      frag_finish<DS>(dd, delta, raw_use, eb, dq);
#pragma unroll
      for (int v = 0; v < 4; ++v) dq[v] = (dq[v] + s14 * wrow_next(w, dq[v])) * k15;  // g0 + mu g1 | 0
      frag_load<DS>(rb, (unsigned)wu(w, (int)R(k >= 2 ? k - 2 : 0)), fp, raw_fill);  // unconditional: k < 2 re-read stage 0's record
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
      {  // Q_uu's factor for second-order corrections: lanes 0..5 store L10, L20, L21, 1/L00, 1/L11, 1/L22
        // selected by lane-constant bit masks: the nested conditional compiled to a divergent branch tree
        // (~40 scalar and exec-mask instructions per stage)
        const T lq = pick6(l, L[1], L[3], L[4], iv[0], iv[1], iv[2]);
        rb.st(lq, Rk, l < 6 ? (unsigned)(RCF::LQ + l) : (unsigned)RCF::JUNK);
      }
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
    for (int k = N - 1;; k -= 3) {
      ok = step(k, raw_a, raw_c) & ok;
      if (k == 0) break;
      ok = step(k - 1, raw_b, raw_a) & ok;
      if (k == 1) break;
      ok = step(k - 2, raw_c, raw_b) & ok;
      if (k == 2) break;
      if (!wuni(w, ok)) return false;
    }
    if (!wuni(w, ok)) return false;
    wsync(w);  // records (P, p, K, k) visible to every lane
    return true;
  }


  // The forward recursion of sweep 3 (dz of the lane's stage, from LDS): the Newton direction, or with SOCM
  // the second-order correction's (feed-forward k_soc, constant c_soc, costate p_soc from the SOC's cold
  // fields, its costate step to SDNU) -- the same lane-group recursion for both.
  template <bool SOCM>
  MR_HD void fwd_recursion(T* dz) {
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
      // SOCM: the constants come from the SOC's cold fields (c_soc, its costate vector, its feed-forward)
      // of stage kk, one extra gather per stage; lanes without a row keep the record's zero slot
      const bool cold_c = SOCM && (g0r | g1r | g2r);
      const unsigned cold0 = (unsigned)(SSF::NF * WL) + (unsigned)RC_STRIDE * WL;  // cold fields' base word
      const unsigned ccoff = g0r ? (unsigned)(CSF::SC + r) * WL : (g1r ? (unsigned)(CSF::SPV + r) * WL
                                                                       : (unsigned)(CSF::SK0 + (g2r ? r : 0)) * WL);
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
        if constexpr (SOCM) {
          const T cc = wb.ld(cold0 + (unsigned)kk, ccoff);
          f.c0 = cold_c ? cc : f.c0;
        }
      };
      auto fstep = [&](int k, const FwdRow& f) {
        T dxv[NX];
        wgather<T, NX>(w, dxi, dxv);
        T acc = f.c0;
        for (int j = 0; j < NX; ++j) acc += f.rw[j] * dxv[j];
        // dx_{k+1} = (A dx_k + c) + B du_k on group 0, du_k from group 2 (lanes 32..34)
        T accx = acc;
#pragma unroll
        for (int a = 0; a < NU; ++a) accx += f.bw[a] * wbcast(w, acc, 32 + a);
        dxi = g0r ? accx : T(0);
        lds[lbase + lstep * k] = g0r ? accx : acc;
        const bool dn = g1r & (k >= 1 || !MR_KKT_RESTATED);  // k = 0: the initial-state rows' multiplier step
        if constexpr (SOCM) {  // the SOC's costate step to its cold field (branch-free: others the discard slot)
          wb.st(acc, (unsigned)k, dn ? cold0 + (unsigned)(CSF::SDNU + r) * WL : R(k) + RCF::JUNK - (unsigned)k);
        } else if constexpr (SSL) {
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
    fwd_recursion<false>(dz);
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
      row_steps<false>(d, act, adz, tau, ap_l, ad_l, g_l);
    }
    ap = wmin(w, ap_l);
    ad = wmin(w, ad_l);
    gphi = wsum(w, g_l);
#if MR_PHASE_CYCLES
    if (trace) { tsub[0] += tf1 - tf0; tsub[1] += MR_CLOCK() - tf1; }
#endif
  }

  // IPOPT's row steps of this lane's stage (mr_solver.h Solver::forward): the slack step of each row
  // ds = a.dz + (d - s) (SOC: + the correction's r_soc instead of d - s), the distance steps (a two-sided
  // row's upper distance: -ds), bound-dual steps dv = mu/t - v - (v/t) dt, the multiplier step
  // dy = (Sigma_s + delta) ds + grad_s phi - y; into the regular fields or the SOC's (SOC)
  template <bool SOC>
  MR_HD void row_steps(const T* d, const int* act, const T* adz, T tau, T& ap_l, T& ad_l, T& g_l) {
    const T mu = this->mu, dl = cw()->delta_it, kd = T(IP_KAPPA_D);
#pragma unroll
    for (int r = 0; r <= NROW; ++r) {
      const int j0 = r < NROW ? 2 * r : JL, j1 = j0 + 1;
      if (!act[j0]) continue;
      const bool a = true;
      const T t0 = S(sf(cur) + j0), t1 = S(sf(cur) + j1);
      const T l0 = S(SSF::LAM + j0), l1 = S(SSF::LAM + j1);
      const T s0 = l0 / t0, s1 = l1 / t1;
      T dt0, dt1, dy0, dy1;
      if (r < 2) {
        const T R0 = SOC ? Cf(CSF::SR + j0) : d[j0] - t0;
        const T R1 = SOC ? Cf(CSF::SR + j1) : -(d[j1] - t1);
        const T Ds0 = adz[j0] + R0, Ds1 = -adz[j1] + R1;
        dt0 = Ds0;
        dt1 = -Ds1;
        dy0 = (s0 + dl) * Ds0 - mu / t0 + kd * mu - S(SSF::Y + j0);
        dy1 = (s1 + dl) * Ds1 + mu / t1 - kd * mu - S(SSF::Y + j1);
        if (!SOC) g_l += a ? kd * mu * (dt0 + dt1) : T(0);
      } else {
        const T R0 = SOC ? Cf(CSF::SR + j0) : d[j0] - t0;
        const T Ds = adz[j0] + R0;
        dt0 = Ds;
        dt1 = -Ds;
        dy0 = (s0 + s1 + dl) * Ds - mu / t0 + mu / t1 - S(SSF::Y + j0);
        dy1 = T(0);
      }
      T dv0 = mu / t0 - l0 - s0 * dt0, dv1 = mu / t1 - l1 - s1 * dt1;
      if (!a) { dt0 = dt1 = dv0 = dv1 = dy0 = dy1 = T(0); }
      if constexpr (SOC) {
        Cf(CSF::SDS + j0) = dt0; Cf(CSF::SDS + j1) = dt1;
        Cf(CSF::SDLAM + j0) = dv0; Cf(CSF::SDLAM + j1) = dv1;
        Cf(CSF::SDY + j0) = dy0; Cf(CSF::SDY + j1) = dy1;
      } else {
        S(SSF::DS + j0) = dt0; S(SSF::DS + j1) = dt1;
        S(SSF::DLAM + j0) = dv0; S(SSF::DLAM + j1) = dv1;
        S(SSF::DY + j0) = dy0; S(SSF::DY + j1) = dy1;
        g_l -= mu * dt0 / t0 + mu * dt1 / t1;
      }
      ap_l = dt0 < T(0) ? mr_min(ap_l, -tau * t0 / dt0) : ap_l;
      ap_l = dt1 < T(0) ? mr_min(ap_l, -tau * t1 / dt1) : ap_l;
      ad_l = dv0 < T(0) ? mr_min(ad_l, -tau * l0 / dv0) : ad_l;
      ad_l = dv1 < T(0) ? mr_min(ad_l, -tau * l1 / dv1) : ad_l;
    }
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

  // ---------------- sweep 4: the filter line search (IPOPT's backtracking) ----------------
  // The lane's stage iterate, step, slacks and slack steps are loaded once; every trial point is formed
  // and measured in registers (one pass per trial: the trial's stage values, its dynamics defect against
  // the neighbour's trial state, three wave sums), and only the accepted (or forced) point is written to
  // iterate buffer 1-cur.  Rules (IPOPT's BacktrackingLineSearch / FilterLSAcceptor, mr_solver.h
  // Solver::backtrack): alpha = a0, a0/2, ... while alpha > a_min (the first trial always); acceptance =
  // theta_max, then (f-type at the test step size with theta_ref <= theta_min) Armijo or sufficient
  // decrease (Compare_le, obj_max_inc), then the filter.  Modes (flags):
  //   LS_WD     one trial, judged at the given test step size (the watchdog's, or the SOC's original), and
  //             stored whatever its acceptance (the watchdog's tentative full step needs no re-evaluation);
  //   LS_FORCE  one trial, stored whatever its acceptance;
  //   LS_CAP    the first trial's constraint values are also written to the cold fields CTR / CTC, so a
  //             second-order correction of that trial point accumulates them (soc_backward) instead of
  //             evaluating the point again;
  //   otherwise backtracking; a rejected first trial (a0 = the fraction-to-boundary step, theta not
  //   decreased) returns with LS_NEED_SOC so the caller runs the second-order corrections.
  // SOCDIR: the trial points lie along the SOC direction (SDZ, SDS) instead of the Newton direction.
  // RESTO: the restoration phase's NLP (mr_solver.h trial() with resto set).
  enum { LS_WD = 1, LS_FORCE = 2, LS_NOSOC = 8, LS_CAP = 16 };
  enum { LSR_ACC = 1, LSR_AUG = 2, LSR_REJF = 4, LSR_NEED_SOC = 8, LSR_FIN = 16 };
  template <bool RESTO, bool SOCDIR>
  MR_SWEEP void line_search(T th, T ph, T gphi, T th_pow, T a0, T a_max, T a_min, int nls0, int mode, T a_fix) {
    MR_UNIFORM_P();
    MR_ASSUME_LDS_STATE();
#if MR_PHASE_CYCLES
    const unsigned long long tls0 = trace ? MR_CLOCK() : 0ull;
#endif
    const int nb = 1 - cur;
    const int k = ln;
    const int N = wu(w, this->N);
    T z[NZS], dz[NZS], s_c[NI], ds[NI];
    // every operand loaded unconditionally (every lane's fields exist), then selected: one memory round
    // trip for the whole set instead of masked loads, each waited for in its branch
    load_z(cur, z);
    for (int i = 0; i < NZS; ++i) {
      const T v = SOCDIR ? Cf(CSF::SDZ + i) : S(SSF::DZ + i);
      dz[i] = own() ? v : T(0);
    }
    T sv[NI], dv[NI];
    for (int j = 0; j < NI; ++j) {
      sv[j] = S(sf(cur) + j);
      dv[j] = SOCDIR ? Cf(CSF::SDS + j) : S(SSF::DS + j);
    }
    unsigned actm = 0u;  // active rows of this stage (depend on the stage only, not on the point)
    T rlo[NROW], rhi[NROW];  // their bounds, once per line search (row_values recomputed them per trial)
#pragma unroll
    for (int r = 0; r < NROW; ++r) {
      int a;
      row_bounds(P, I, k, r, a, rlo[r], rhi[r]);
      actm |= (own() && a) ? (3u << (2 * r)) : 0u;
    }
    const T lmax = I.max_err + relax_amt(I.max_err);  // the lane rows' relaxed bound (lane_d)
    actm |= (own() && lane_active(P, k)) ? (3u << JL) : 0u;
    for (int j = 0; j < NI; ++j) {
      const bool a = (actm >> j) & 1u;
      s_c[j] = a ? sv[j] : T(1);
      ds[j] = a ? dv[j] : T(0);
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
        const T v0 = Cf(CSF::RP + j), v1 = Cf(CSF::RN + j), v2 = Cf(CSF::RDP + j), v3 = Cf(CSF::RDN + j);
        rp[j] = a ? v0 : T(1);
        rn[j] = a ? v1 : T(1);
        rdp[j] = a ? v2 : T(0);
        rdn[j] = a ? v3 : T(0);
      }
      const bool dk = own() && k < N;
      for (int i = 0; i < 6; ++i) {
        const T v0 = Cf(CSF::CP + i), v1 = Cf(CSF::CN + i), v2 = Cf(CSF::CDP + i), v3 = Cf(CSF::CDN + i);
        cp[i] = dk ? v0 : T(1);
        cn[i] = dk ? v1 : T(1);
        cdp[i] = dk ? v2 : T(0);
        cdn[i] = dk ? v3 : T(0);
      }
      for (int i = 0; i < NZS; ++i) {
        const T v = Cf(CSF::RZ + i);
        zr[i] = own() ? v : T(0);
      }
    }
    T zt[NZS], st[NI];
    const T kdm = T(IP_KAPPA_D) * mu;
    // one trial point: zt, st (registers), theta, phi; false if a slack is not positive or a value is
    // not finite.  cap: also write its constraint values to the cold fields CTR / CTC for a second-order
    // correction (LS_CAP).  One body with a run-time flag: the form with two compile-time instantiations
    // selected by (capm && n == 0) -- a branch the compiler must treat as divergent, mode being a VGPR
    // argument -- made the fp64 C5 solves differ from run to run in the second-order-correction steps
    // (tools/determinism_probe.py; bisected to that change); this form is bit-identical run to run
    auto eval = [&](T alpha, T& th_t, T& ph_t, bool cap) -> bool {
#if MR_PHASE_CYCLES
      const unsigned long long te0 = trace ? MR_CLOCK() : 0ull;
#endif
      for (int i = 0; i < NZS; ++i) zt[i] = z[i] + alpha * dz[i];
      if (k == 0)
        for (int i = 0; i < NX; ++i) zt[i] = z[i];  // x_0 fixed
      if (k >= N) { zt[11] = zt[12] = zt[13] = T(0); }
      T ztn[NX];
      for (int i = 0; i < NX; ++i) ztn[i] = wnext(w, zt[i]);
      T th_l = T(0), f_l = T(0), lg_l = T(0), lgr_l = T(0), tho_l = T(0), fo_l = T(0), lin_l = T(0);
      int ok_l = 1;
      if (own()) {
        Err<T> e;
        errors(I, zt[0], zt[1], zt[6], e, false);
        T d[NI];  // row_values with the line search's bounds (the same values; activity from actm)
#pragma unroll
        for (int r = 0; r < NROW; ++r) {
          const T c = row_c(r, zt);
          d[2 * r] = c - rlo[r];
          d[2 * r + 1] = rhi[r] - c;
        }
        d[JL] = e.eC + lmax + T(0);
        d[JL + 1] = lmax - e.eC + T(0);
        d[JL + 2] = T(0);
        if constexpr (!RESTO) {
          // branch-free over the slots (the per-slot activity test compiled to a divergent branch each):
          // an inactive slot has s = 1, ds = 0 (setup above), so s + alpha ds = 1 > 0 and log 1 = 0 add
          // nothing, and its other terms are selected out -- the same sums as the branching form
#pragma unroll
          for (int j = 0; j < NI; ++j) {
            const bool a = (actm >> j) & 1u;
            const T sj = s_c[j] + alpha * ds[j];
            ok_l &= sj > T(0) ? 1 : 0;
            st[j] = sj;
            lg_l += mr_log(sj > T(0) ? sj : T(1));
            if (oneslot(j)) lin_l += a ? sj : T(0);
            if (yslot(j)) {
              const T r = d[j] - sj;
              th_l += a ? mr_abs(r) : T(0);
              if (cap) Cf(CSF::CTR + j) = a ? T(slot_sign(j)) * r : T(0);
            } else if (cap) {
              Cf(CSF::CTR + j) = T(0);
            }
          }
        }
        for (int j = 0; j < NI; ++j) {
          if (!RESTO) break;  // (the regular trial's slots: the branch-free loop above)
          st[j] = s_c[j];
          if (!((actm >> j) & 1u)) continue;
          const T sj = s_c[j] + alpha * ds[j];
          if (!(sj > T(0))) ok_l = 0;
          st[j] = sj;
          lg_l += mr_log(sj > T(0) ? sj : T(1));
          if (oneslot(j)) lin_l += sj;
          if constexpr (RESTO) {
            const T pt = rp[j] + alpha * rdp[j], nt = rn[j] + alpha * rdn[j];
            if (!(pt > T(0)) || !(nt > T(0))) ok_l = 0;
            th_l += mr_abs(d[j] - sj - pt + nt);
            if (yslot(j)) tho_l += mr_abs(d[j] - sj);
            lgr_l += mr_log(pt > T(0) ? pt : T(1)) + mr_log(nt > T(0) ? nt : T(1));
            f_l += rho * (pt + nt);
          }
        }
        if constexpr (RESTO) {
          f_l += prox_term(I, k, N, zt, zr, zeta, (T*)nullptr, (T*)nullptr);
          fo_l += stage_cost(P, I, k, zt, e, sc, (T*)nullptr, (T*)nullptr);
        } else {
          f_l += stage_cost(P, I, k, zt, e, sc, (T*)nullptr, (T*)nullptr);
        }
        if (k < N) {
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
            for (int i = 0; i < NX; ++i) {
              th_l += mr_abs(xn[i] - ztn[i]);
              if (cap) Cf(CSF::CTC + i) = xn[i] - ztn[i];
            }
          }
        } else if (!RESTO && cap) {
          for (int i = 0; i < NX; ++i) Cf(CSF::CTC + i) = T(0);
        }
      }
#if MR_PHASE_CYCLES
      const unsigned long long te1 = trace ? MR_CLOCK() : 0ull;
#endif
      th_t = wsum(w, th_l);
      const T fv = wsum(w, f_l), lg = wsum(w, lg_l), lin = wsum(w, lin_l);
      int ok = wall(w, ok_l != 0) ? 1 : 0;
#if MR_PHASE_CYCLES
      if (trace) { tsub[8] += te1 - te0; tsub[9] += MR_CLOCK() - te1; }
#endif
      ph_t = fv - mu * lg + kdm * lin;
      if constexpr (RESTO) {
        ph_t = fv - mu * (lg + wsum(w, lgr_l)) + kdm * lin;
        cw()->tho = wsum(w, tho_l);  // the point as the original problem sees it (restoration exit test)
        cw()->fo = wsum(w, fo_l);
        cw()->pho = cw()->fo - mu_o * lg + T(IP_KAPPA_D) * mu_o * lin;
      }
      if (!(th_t == th_t) || !(ph_t == ph_t)) ok = 0;
      return wuni(w, ok != 0);
    };
#if MR_PHASE_CYCLES
    if (trace) tsub[11] += MR_CLOCK() - tls0;
#endif
    const LSRef<T> ref{th, ph, gphi, th_pow};
    // the reference point's transcendental terms, once per line search (is_ftype's (-gphi)^2.3 and
    // acc_to_iterate's log10 |phi|; the same expressions, so the same values, as the per-trial forms)
    const T gpow = gphi < T(0) ? mr_exp(T(2.3) * mr_log(-gphi)) : T(0);
    const T phbas = mr_abs(ph) > T(10) ? mr_log(mr_abs(ph)) / mr_log(T(10)) : T(1);
    auto ftype = [&](T at) { return gphi < T(0) && at * gpow > th_pow; };
    auto acc_it = [&](T tht, T pht) {
      if (pht > ph && mr_log(pht - ph) / mr_log(T(10)) > T(IP_OBJ_MAX_INC) + phbas) return false;
      const T g = T(1e-5);
      return cmp_le(tht, (T(1) - g) * th, th) || cmp_le(pht - ph, -g * th, ph);
    };
    T alpha = a0, ph_acc = ph, a_test = a0, th_t = T(0), ph_t = T(0);
    int nls = nls0, ntr = 0;
    int flags = 0;
    bool store = false;
    if (mode & LS_FORCE) {
      alpha = a_fix;
      const bool fin = eval(alpha, th_t, ph_t, false);
      ntr++;
      flags |= fin ? LSR_FIN : 0;
      store = true;
      ph_acc = ph_t;  // (the forced trial's own barrier objective: the soft restoration's test)
    } else {
      const bool capm = !RESTO && (mode & LS_CAP);
      for (int n = 0; n < IP_LS_MAX; ++n) {
        if (!(alpha > a_min || n == 0)) break;
        a_test = (mode & LS_WD) ? a_fix : alpha;
        const bool fin = eval(alpha, th_t, ph_t, capm && n == 0);
        ntr++;
#if MR_PHASE_CYCLES
        const unsigned long long ta0 = trace ? MR_CLOCK() : 0ull;
#endif
        bool ok = false;
        if (fin) {
          ok = th_t <= theta_max;
          if (ok) {
            if (a_test > T(0) && ftype(a_test) && th <= theta_min) ok = armijo(ph_t, a_test, ref);
            else ok = acc_it(th_t, ph_t);
          }
          if (ok && !filter_ok(th_t, ph_t)) { ok = false; flags |= LSR_REJF; }
        }
#if MR_PHASE_CYCLES
        if (trace) tsub[10] += MR_CLOCK() - ta0;
#endif
        if (wuni(w, ok)) {
          flags |= LSR_ACC | LSR_FIN;
          if (!(ftype(a_test) && armijo(ph_t, a_test, ref))) flags |= LSR_AUG;
          ph_acc = ph_t;
          store = true;
          break;
        }
        if (mode & LS_WD) {  // the single trial is stored either way: the watchdog takes it anyway if its
          store = true;      // trial budget lasts (no re-evaluation); otherwise the point is overwritten
          flags |= fin ? LSR_FIN : 0;
          break;
        }
        if (!RESTO && !(mode & LS_NOSOC) && fin && n == 0 && alpha == a_max && theta <= th_t) {
          flags |= LSR_NEED_SOC;  // the caller runs the second-order corrections, then resumes at alpha/2
          break;
        }
        alpha *= T(0.5);
        nls++;
      }
    }
    if (store && own()) {  // the chosen point
      for (int j = 0; j < NI; ++j)
        if ((actm >> j) & 1u) S(sf(nb) + j) = st[j];
      for (int i = 0; i < NZS; ++i) S(zf(nb) + i) = zt[i];
      if constexpr (RESTO) {  // the relaxations move in place (their step is applied once, here)
        if (flags & LSR_ACC) {
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
    res_flags = flags;
    res_nls = nls;
    res_ntr = ntr;
    res_th = th_t;
    res_ph = ph_acc;
    res_atest = a_test;
  }

  // FilterLSAcceptor's tests (mr_solver.h Solver: Compare_le with 10 eps |ref|, obj_max_inc 5)
  static MR_HD bool cmp_le(T lhs, T rhs, T bas) { return lhs - rhs <= T(10) * mr_eps<T>() * mr_abs(bas); }
  static MR_HD bool is_ftype(T a_test, const LSRef<T>& r) {
    return r.gphi < T(0) && a_test * mr_exp(T(2.3) * mr_log(-r.gphi)) > r.thpow;
  }
  static MR_HD bool armijo(T ph_t, T a_test, const LSRef<T>& r) {
    return cmp_le(ph_t - r.ph, T(1e-4) * a_test * r.gphi, r.ph);
  }
  static MR_HD bool acc_to_iterate(T th_t, T ph_t, const LSRef<T>& r) {
    if (ph_t > r.ph) {
      const T bas = mr_abs(r.ph) > T(10) ? mr_log(mr_abs(r.ph)) / mr_log(T(10)) : T(1);
      if (mr_log(ph_t - r.ph) / mr_log(T(10)) > T(IP_OBJ_MAX_INC) + bas) return false;
    }
    const T g = T(1e-5);
    return cmp_le(th_t, (T(1) - g) * r.th, r.th) || cmp_le(ph_t - r.ph, -g * r.th, r.ph);
  }

  // ---------------- second-order corrections (IPOPT's TrySecondOrderCorrection, linear) ----------------
  // mr_solver.h Solver::try_soc / soc_backward: the Newton system re-solved on the stored factorisation
  // with the constraint right-hand sides c_soc (dynamics rows, CSF::SC) and r_soc (the rows' d - s,
  // CSF::SR), c_soc = alpha c_soc + c(trial) per correction (accumulated in soc_backward's stage-parallel pass).
  // Up to max_soc = 4 per iteration; the batch's long solves run 2-3 per iteration, so the two recursions
  // (socb_chain backward, fwd_recursion<true> forward) are lane recursions on the stage records.
  // The SOC costate recursion given v_k, u_k (cold fields SPV, SK0: everything that does not depend on
  // pv_{k+1}): pv_k = v_k + A_k^T pv_{k+1} + K_k^T b_k with b_k = B_k^T pv_{k+1}, and r_k = b_k + u_k (the
  // feed-forward's right-hand side).  Two lane groups share one 11-term dot product with pv_{k+1} (broadcast
  // from lanes 0..10 by v_readlane), each lane gathering its coefficient column of the stage map E^ from the
  // record (ehat_slot: its data word or the record's constant slots): group 0 (lanes 0..10) column i of A_k
  // -> (A_k^T pv)[i], group 1 (lanes 16..18) column a of B_k -> b_k[a]; then group 0 adds K_k^T b_k with b_k
  // read from group 1 (the forward recursion's structure, transposed).  B_k^T pv is thus three lanes' dot
  // products instead of twelve FMAs in every lane.  Per stage: 14 v_readlane, ~16 FMAs, 15 single-line
  // gathers issued two stages ahead; results to LDS only (pv_k to LDX row k, r_k to [LX_OFF + 3 k]), so the
  // in-order vmcnt waits for the prefetched operands stay exact.
  MR_HD void socb_chain() {
    const int N = wu(this->w, this->N), ln = this->ln;
    const Wv w = this->w;
    const WBuf<T> wb(rc - (int64_t)SSF::NF * WL, (unsigned)WS_NU_OFF);
    auto R = [](int k) { return (unsigned)(SSF::NF * WL) + (unsigned)k * (unsigned)RC_STRIDE; };
    const unsigned cold0 = (unsigned)(SSF::NF * WL) + (unsigned)RC_STRIDE * WL;
    const int grp = ln >> 4, r = ln & 15;
    const bool g0r = (grp == 0) & (r < NX), g1r = (grp == 1) & (r < NU);
    const int li = g0r ? r : 0;
    // per-lane gather plan: the coefficient column (E^ column r of A, or column 11 + r of B), K_k[0..2][r]
    // (group 0), and the constant v_k[r] (group 0) / u_k[r] (group 1) from the cold fields
    int coff[NX], koff[NU];
#pragma unroll
    for (int j = 0; j < NX; ++j) coff[j] = g0r ? ehat_slot(j, r, true) : (g1r ? ehat_slot(j, NX + r, true) : RCF::CZERO);
#pragma unroll
    for (int a = 0; a < NU; ++a) koff[a] = g0r ? RCF::K + a * NX + r : RCF::CZERO;
    const unsigned voff = g0r ? (unsigned)(CSF::SPV + r) * WL : (g1r ? (unsigned)(CSF::SK0 + r) * WL : (unsigned)CSF::SJUNK * WL);
    struct Ops {
      T c[NX], kc[NU], v;
    };
    auto ld = [&](int k, Ops& o) {
      const unsigned rk = (unsigned)wu(w, (int)R(k)), ck = (unsigned)wu(w, (int)(cold0 + (unsigned)k));
#pragma unroll
      for (int j = 0; j < NX; ++j) o.c[j] = wb.ld(rk, (unsigned)coff[j]);
#pragma unroll
      for (int a = 0; a < NU; ++a) o.kc[a] = wb.ld(rk, (unsigned)koff[a]);
      o.v = wb.ld(ck, voff);
    };
    T pv = wb.ld((unsigned)wu(w, (int)(cold0 + (unsigned)N)), (unsigned)(CSF::SG + li) * WL);  // pv_N = g_x,N
    // the LDS base in a register (a member read after an LDS store is reloaded from the solver object,
    // itself in LDS: one LDS round trip per step); group 0: LDX row k, group 1: r_k's slot, others: the
    // lane's discard slot
    MR_LDS T* const LB = lds;
    const int pbase = g0r ? LDX_OFF + r : (g1r ? LX_OFF + r : LJUNK_OFF + ln), pstride = g0r ? 12 : (g1r ? 3 : 0);
    if (g0r) lds[LDX_OFF + N * 12 + r] = pv;
    auto step = [&](int k, const Ops& o) {
      T p[NX];
      wgather<T, NX>(w, pv, p);
      T s0 = o.c[0] * p[0], s1 = o.c[1] * p[1];
#pragma unroll
      for (int j = 2; j < NX; j += 2) {
        s0 += o.c[j] * p[j];
        if (j + 1 < NX) s1 += o.c[j + 1] * p[j + 1];
      }
      const T sd = s0 + s1;  // group 0: (A^T pv)[r]; group 1: b[r] = (B^T pv)[r]
      T pn = o.v + sd;       // group 1: r_k = b + u
#pragma unroll
      for (int a = 0; a < NU; ++a) pn += o.kc[a] * wbcast(w, sd, 16 + a);  // group 0: + K^T b (kc = 0 elsewhere)
      pv = pn;
      LB[pbase + pstride * k] = pn;
    };
    // operands two stages ahead, three rotating sets (unrolled by three: no register copies of in-flight
    // loads); a prefetch past stage 0 re-reads stage 0 (unconditional loads, exact waits).  Two ahead, not
    // three: a wave has at most 63 vector-memory instructions outstanding (vmcnt).  Scheduling barriers keep
    // each prefetch ahead of the step it overlaps (left free, the scheduler sank the loads to the loop's end)
    if (N > 0) {
      auto kc = [](int k) { return k > 0 ? k : 0; };
      Ops b0, b1, b2;
      ld(N - 1, b0);
      ld(kc(N - 2), b1);
      for (int k = N - 1;; k -= 3) {
        ld(kc(k - 2), b2);
        MR_SCHED_BARRIER();
        step(k, b0);
        if (k == 0) break;
        ld(kc(k - 3), b0);
        MR_SCHED_BARRIER();
        step(k - 1, b1);
        if (k == 1) break;
        ld(kc(k - 4), b1);
        MR_SCHED_BARRIER();
        step(k - 2, b2);
        if (k == 2) break;
      }
    }
    wsync_lds(w);
  }

  // The SOC's costate vector and feed-forward on the stored factorisation:
  //   pc = pv_{k+1} + P_{k+1} c_k,  r = B^T pc + g_u,  k_k = -Q_uu^-1 r,  pv_k = g_x + A^T pc + K^T r.
  // The stage gradients (with the rows' r_soc) are stage-parallel (lane = stage); the recursion runs on
  // lanes 0..10 (lane i: component i of pc / pv, the others' by v_readlane), every lane gathering its
  // row of P_{k+1}, its column of A_k and K_k from the stage's record (a few cache lines per stage) and
  // the shared terms (B's J columns, Q_uu's factor, c_k, g_u) as uniform loads, one stage ahead.
  // first: the episode's first correction (its right-hand sides start from the current point); acc: the
  // previous trial's step size (IPOPT: c_soc = alpha c_soc + c(trial), r_soc likewise)
  MR_SWEEP void soc_backward(bool first, T acc) {
    MR_UNIFORM_P();
    MR_ASSUME_LDS_STATE();
#if MR_PHASE_CYCLES
    unsigned long long tb = trace ? MR_CLOCK() : 0ull;
#define MR_TSUB(q) do { if (trace) { const unsigned long long tn = MR_CLOCK(); tsub[q] += tn - tb; tb = tn; } } while (0)
#else
#define MR_TSUB(q) ((void)0)
#endif
    const T mu = this->mu, dl = cw()->delta_it;
    const int N = wu(w, this->N);
    if (own()) {
      const int k = ln;
      const MR_GLOBAL T* Rk = R(k);
      T g[NZ];
      for (int i = 0; i < NZ; ++i) g[i] = Rk[RCF::G0 + i] + mu * Rk[RCF::G1 + i] + dl * Rk[RCF::GD + i];
      T z[NZS];
      load_z(cur, z);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      row_values(k, z, e, d, act);
      // the right-hand sides c_soc (dynamics rows, SC) and r_soc (the rows' d - s, SR): on the episode's first
      // correction the current point's values, then accumulated with the trial point's values its evaluation
      // captured (LS_CAP; 0 where nothing is accumulated) -- in this stage-parallel pass, which evaluates the
      // current point's rows anyway (a separate prepare / accumulate sweep cost two round trips per correction).
      // Every operand loaded unconditionally first, then selected: no load waited for inside a per-slot branch
      T srv[NI], ctr[NI], slk[NI], scv[NX], ctc[NX], cdef[NX];
      for (int j = 0; j < NI; ++j) {
        srv[j] = Cf(CSF::SR + j);
        ctr[j] = Cf(CSF::CTR + j);
        slk[j] = S(sf(cur) + j);
      }
      for (int i = 0; i < NX; ++i) {
        scv[i] = Cf(CSF::SC + i);
        ctc[i] = Cf(CSF::CTC + i);
        cdef[i] = Rk[RCF::C + i];
      }
      T sr[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        const T p0 = (act[j] && yslot(j)) ? T(slot_sign(j)) * (d[j] - slk[j]) : T(0);
        sr[j] = acc * (first ? p0 : srv[j]) + ctr[j];
      }
      T scn[NX];
#pragma unroll
      for (int i = 0; i < NX; ++i) scn[i] = acc * (first ? (k < N ? cdef[i] : T(0)) : scv[i]) + ctc[i];
      for (int j = 0; j < NI; ++j) Cf(CSF::SR + j) = sr[j];
      for (int i = 0; i < NX; ++i) Cf(CSF::SC + i) = scn[i];
#pragma unroll
      for (int r = 0; r <= NROW; ++r) {
        const int j0 = r < NROW ? 2 * r : JL, j1 = j0 + 1;
        if (!act[j0]) continue;
        const T t0 = slk[j0], t1 = slk[j1];
        const T s0 = S(SSF::LAM + j0) / t0, s1 = S(SSF::LAM + j1) / t1;
        T dg;
        if (r < 2) dg = (s0 + dl) * (sr[j0] - (d[j0] - t0)) + (s1 + dl) * (sr[j1] + (d[j1] - t1));
        else dg = (s0 + s1 + dl) * (sr[j0] - (d[j0] - t0));
        if (r < NROW) {
#pragma unroll
          for (int a = 0; a < RN(r); ++a) g[RI(r, a)] += T(RS(a)) * dg;
        } else {
          g[0] += e.gC[0] * dg;
          g[1] += e.gC[1] * dg;
          g[6] += e.gC[2] * dg;
        }
      }
      for (int i = 0; i < NZ; ++i) Cf(CSF::SG + i) = g[i];
    }
    wsync(w);
    MR_TSUB(12);
    // pv_k = Acl_k^T pv_{k+1} + v_k with v_k = A_k^T q + K_k^T u_k + g_x, q = P_{k+1} c_k, u_k = B_k^T q + g_u
    // (then r_k = B_k^T pv_{k+1} + u_k): v_k, u_k stage-parallel into the cold fields SPV / SK0 (everything
    // that does not depend on pv_{k+1}), then the lean lane recursion (socb_chain: pv_{k+1} broadcast,
    // A_k^T pv + K_k^T (B_k^T pv) + v_k, r_k on the way), then the feed-forward stage-parallel
    if (own() && ln < N) {
      const int k = ln;
      const MR_GLOBAL T* Rk = R(k);
      const MR_GLOBAL T* Rn = R(k + 1);
      T c[NX], q[NX], J[48];
      for (int j = 0; j < NX; ++j) c[j] = Cf(CSF::SC + j);
      for (int r = 0; r < NX; ++r) {
        T v = T(0);
        for (int j = 0; j < NX; ++j) v += Rn[RCF::P + pidx(r, j)] * c[j];
        q[r] = v;
      }
      for (int j = 0; j < 48; ++j) J[j] = Rk[RCF::J + j];
      T u[NU], at[NX], Kr[NU][NX];
      for (int a = 0; a < NU; ++a)
        for (int r = 0; r < NX; ++r) Kr[a][r] = Rk[RCF::K + a * NX + r];
      apply_Bt(J, k, q, u);
      for (int a = 0; a < NU; ++a) u[a] += Cf(CSF::SG + NX + a);
      apply_At(J, k, q, at);
      for (int r = 0; r < NX; ++r) {
        T v = at[r] + Cf(CSF::SG + r);
        for (int a = 0; a < NU; ++a) v += Kr[a][r] * u[a];
        Cf(CSF::SPV + r) = v;
      }
      for (int a = 0; a < NU; ++a) Cf(CSF::SK0 + a) = u[a];
    }
    MR_LDS T* const LDX = lds + LDX_OFF;
    wsync(w);  // v_k, u_k (cold fields) visible
    MR_TSUB(13);
    socb_chain();
    MR_TSUB(14);
    if (own()) {
      const int k = ln;
      T pv[NX];
      for (int r = 0; r < NX; ++r) pv[r] = LDX[k * 12 + r];
      if (k < N) {
        const MR_GLOBAL T* Rk = R(k);
        const T Lf[6] = {T(0), Rk[RCF::LQ + 0], T(0), Rk[RCF::LQ + 1], Rk[RCF::LQ + 2], T(0)};
        const T iv[3] = {Rk[RCF::LQ + 3], Rk[RCF::LQ + 4], Rk[RCF::LQ + 5]};
        T kf[NU];
        for (int a = 0; a < NU; ++a) kf[a] = -lds[LX_OFF + 3 * k + a];  // r_k from the chain
        lsolve3r(Lf, iv, kf);
        ltsolve3r(Lf, iv, kf);
        for (int a = 0; a < NU; ++a) Cf(CSF::SK0 + a) = kf[a];
      }
      for (int r = 0; r < NX; ++r) Cf(CSF::SPV + r) = pv[r];
    }
    wsync(w);
    MR_TSUB(15);
#undef MR_TSUB
  }
  // the SOC direction (mr_solver.h Solver::forward with soc set): SDZ, SDS, SDLAM, SDY, SDNU.  The recursion
  // is the Newton direction's (fwd_recursion, its lane groups and prefetch) with the SOC's feed-forward,
  // constant and costate vector; then stage-parallel the rows' steps and the step limits.
  MR_SWEEP void forward_soc(T& ap, T& ad) {
    MR_UNIFORM_P();
    MR_ASSUME_LDS_STATE();
    const T tau = mr_max(T(0.99), T(1) - mu);
    const int N = wu(w, this->N);
    T dzr[NZS];
    for (int i = 0; i < NZS; ++i) dzr[i] = T(0);
#if MR_PHASE_CYCLES
    const unsigned long long tc0 = trace ? MR_CLOCK() : 0ull;
#endif
    fwd_recursion<true>(dzr);
    wsync(w);  // SDNU (the recursion's costate steps) visible
#if MR_PHASE_CYCLES
    if (trace) tsub[2] += MR_CLOCK() - tc0;
    const unsigned long long tp0 = trace ? MR_CLOCK() : 0ull;
#endif
    T ap_l = T(1), ad_l = T(1), g_l = T(0);
    if (own()) {
      const int k = ln;
      const MR_GLOBAL T* Rk = R(k);
      T dz[NZS];
      for (int i = 0; i < NZS; ++i) dz[i] = dzr[i];
      (void)Rk;
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
      for (int i = 0; i < NZS; ++i) Cf(CSF::SDZ + i) = dz[i];
      row_steps<true>(d, act, adz, tau, ap_l, ad_l, g_l);
    }
    ap = wmin(w, ap_l);
    ad = wmin(w, ad_l);
    wsync(w);
#if MR_PHASE_CYCLES
    if (trace) tsub[3] += MR_CLOCK() - tp0;
#endif
  }
  // the accepted correction becomes the iteration's direction; returns its dual step size
  MR_SWEEP T soc_commit() {
    MR_ASSUME_LDS_STATE();
    const T tau = mr_max(T(0.99), T(1) - mu);
    T ad_l = T(1);
    if (own()) {
      for (int i = 0; i < NZS; ++i) S(SSF::DZ + i) = Cf(CSF::SDZ + i);
      for (int j = 0; j < NI; ++j) {
        const T dl = Cf(CSF::SDLAM + j), lam = S(SSF::LAM + j);
        S(SSF::DS + j) = Cf(CSF::SDS + j);
        S(SSF::DLAM + j) = dl;
        S(SSF::DY + j) = Cf(CSF::SDY + j);
        if (lam != T(0) && dl < T(0)) ad_l = mr_min(ad_l, -tau * lam / dl);
      }
      for (int i = 0; i < NX; ++i) S(SSF::DNU + i) = Cf(CSF::SDNU + i);
    }
    const T ad = wmin(w, ad_l);
    wsync(w);
    return ad;
  }

  // The filter: entries 0..FMAX-1 in LDS (every lane the same values), the rest in the cold fields FOV of
  // the phase's bank, lane l holding entries FMAX + 64 q + l (one coalesced load per 64 entries, tested
  // stage-parallel and OR-reduced) -- IPOPT's unbounded filter up to FCAP entries (mr_solver.h)
  MR_HD int fbank() const { return cw()->resto ? 1 : 0; }
  MR_HD bool filter_hit_ov(T th, T ph, int n, int bank) const {
    int hit = 0;
    for (int q = 0; q < FOVF; ++q) {
      const int base = FMAX + q * WL;
      if (base >= n) break;  // (n wave-uniform)
      const T a = Cf(CSF::FOV + (2 * bank) * FOVF + q), b = Cf(CSF::FOV + (2 * bank + 1) * FOVF + q);
      hit |= (base + ln < n && th >= a && ph >= b) ? 1 : 0;
    }
    return wany(w, hit != 0);
  }
  // entry i of the LDS bank tested by lane i (th, ph wave-uniform)
  MR_HD bool filter_hit_lds(T th, T ph, int n, const MR_LDS T* fth0, const MR_LDS T* fph0) const {
    const int i = ln < FMAX ? ln : FMAX - 1;
    return wany(w, ln < n && ln < FMAX && th >= fth0[i] && ph >= fph0[i]);
  }
  MR_HD bool filter_ok(T th, T ph) const {
    if (filter_hit_lds(th, ph, nfilt, &fth(0), &fph(0))) return false;
    if (nfilt > FMAX && filter_hit_ov(th, ph, nfilt, fbank())) return false;
    return true;
  }
  MR_HD void filter_add(T th, T ph) {
    if (nfilt < FMAX) {
      for (int i = 0; i < FMAX; ++i)
        if (i == nfilt) { fth(i) = th; fph(i) = ph; }
      nfilt++;
    } else if (nfilt < FCAP) {  // (full -- beyond max_iter 500 -- the entry is dropped, as in mr_solver.h)
      const int o = nfilt - FMAX, b = fbank();
      if (ln == (o & (WL - 1))) {
        Cf(CSF::FOV + (2 * b) * FOVF + (o >> 6)) = th;
        Cf(CSF::FOV + (2 * b + 1) * FOVF + (o >> 6)) = ph;
      }
      nfilt++;
      wsync(w);  // the entry visible to every lane's later filter tests
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
        Cf(CSF::WY + j) = S(SSF::Y + j); Cf(CSF::WDY + j) = S(SSF::DY + j);
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
        S(SSF::Y + j) = Cf(CSF::WY + j); S(SSF::DY + j) = Cf(CSF::WDY + j);
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
    filter_add((T(1) - g_th) * th, ph - g_ph * th);  // PrepareRestoPhaseStart: the entry point augments the filter
    C->onfilt = nfilt;
    for (int i = 0; i < 2 * FMAX; ++i) C->ofilt[i] = filt[i];
    C->mu_o = mu;
    C->th_entry = th;
    C->delta_last_o = delta_last;
    C->theta_max_o = theta_max;
    C->theta_min_o = theta_min;
    C->rho = rho;
    // the current point's constraint values, measured here: after a watchdog restore the evaluation
    // sweep's (defects in the stage record, pr_max, theta) belong to the abandoned iterate
    const int k = ln;
    T z[NZS];
    load_z(cur, z);
    T znext[NX], c[NX], d[NI];
    int act[NI];
    for (int i = 0; i < NX; ++i) { znext[i] = wnext(w, z[i]); c[i] = T(0); }
    T pr_l = T(0), th_def_l = T(0), fo_l = T(0);
    if (own()) {
      if (k < N) {
        T xn[NX];
        faug<T, MODEL>(P, k, z, xn);
        for (int i = 0; i < NX; ++i) {
          c[i] = xn[i] - znext[i];
          pr_l = mr_max(pr_l, mr_abs(c[i]));
          if (i >= 6) th_def_l += mr_abs(c[i]);  // definitional rows (S, previous controls): not relaxed
        }
      }
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      row_values(k, z, e, d, act);
      for (int j = 0; j < NI; ++j)
        if (act[j] && yslot(j)) pr_l = mr_max(pr_l, mr_abs(d[j] - S(sf(cur) + j)));
      fo_l = stage_cost(P, I, k, z, e, sc, (T*)nullptr, (T*)nullptr);
    }
    // the original objective at the entry point (reported if the restoration phase ends the solve)
    C->fo_cur = wsum(w, fo_l);
    // IPOPT's RestoIterateInitializer: mu_r = max(mu, ||c||_inf, ||d - s||_inf)
    const T mu_r = mr_max(mu, wmax(w, pr_l));
    const T th_r = wsum(w, th_def_l);  // relaxed rows start satisfied: the definitional rows only
    if (own()) {
      for (int i = 0; i < NZS; ++i) Cf(CSF::RZ + i) = z[i];
      for (int j = 0; j < NI; ++j) {
        T p = T(1), n = T(1);
        Cf(CSF::RS0 + j) = S(sf(cur) + j);
        Cf(CSF::RLAM + j) = S(SSF::LAM + j);
        if (act[j]) {
          resto_pn(d[j] - S(sf(cur) + j), mu_r, rho, p, n);
          // the slacks' bound duals: the original problem's, but not above rho (RestoIterateInitializer)
          S(SSF::LAM + j) = mr_min(S(SSF::LAM + j), rho);
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
          resto_pn(c[i], mu_r, rho, p, n);
          Cf(CSF::CP + i) = p;
          Cf(CSF::CN + i) = n;
          Cf(CSF::CVP + i) = mu_r / p;
          Cf(CSF::CVN + i) = mu_r / n;
          Cf(CSF::CDP + i) = T(0); Cf(CSF::CDN + i) = T(0); Cf(CSF::CDVP + i) = T(0); Cf(CSF::CDVN + i) = T(0);
        }
    }
    alpha_p = alpha_d = T(0);
    mu = mu_r;
    C->resto = 1;
    C->resto_first = 1;  // no barrier update in the restoration phase's first iteration
    C->in_soft = 0;
    C->soft_count = 0;
    nfilt = 0;
    delta_last = T(0);
    theta_max = T(1e4) * mr_max(T(1), th_r);
    theta_min = T(1e-4) * mr_max(T(1), th_r);
    wsync(w);
    if (MR_RESTO_LS_MULT) ls_resto();
  }

  // IPOPT's least-square multipliers of the restoration NLP at its start (mr_solver.h Solver::ls_resto, the
  // derivation there): the stage QP H = I on the reference's variables + a a^T / 3 per relaxed row slot,
  // g = -a cg / 3 (cg = v + v_p - v_n), the vehicle rows' disturbance with sw = 1/2, gw = (v_p - v_n) / 2,
  // solved by the restoration Riccati and forward sweeps; y = (cg - a.sx) / 3, the costates the dynamics rows'
  // multipliers; all zero if one exceeds 1000.  Run once per restoration phase, by few instances.
  MR_SWEEP void ls_record_resto() {
    MR_UNIFORM_P();
    MR_ASSUME_LDS_STATE();
    if (own()) {
      const int k = ln;
      T z[NZS];
      load_z(cur, z);
      MR_GLOBAL T* Rk = R(k);
      T H[NH], g[NZ];
      for (int i = 0; i < NH; ++i) H[i] = T(0);
      for (int i = 0; i < NZ; ++i) g[i] = T(0);
      if (k < N) {
        T Hd[36], fx[6], J[48], nz[NX];
        for (int i = 0; i < NX; ++i) nz[i] = T(0);
        Dyn<T, MODEL>::fjh(P, z, z + NX, nz, fx, J, Hd);
        for (int i = 0; i < 48; ++i) Rk[RCF::J + i] = J[i];
        for (int i = 0; i < 6; ++i) {
          Cf(CSF::CSW + i) = T(0.5);
          Cf(CSF::CGW0 + i) = T(0.5) * (Cf(CSF::CVP + i) - Cf(CSF::CVN + i));
          Cf(CSF::CGW1 + i) = T(0);
        }
      }
      for (int i = 0; i < NZ; ++i)
        if (delta_var(i)) H[hidx(i, i)] = T(1);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      row_values(k, z, e, d, act);
      auto cg = [&](int j) { return S(SSF::LAM + j) + Cf(CSF::RVP + j) - Cf(CSF::RVN + j); };
#pragma unroll
      for (int r = 0; r < NROW; ++r) {
        if (!act[2 * r]) continue;
        const T gs = (cg(2 * r) - cg(2 * r + 1)) / T(3);  // slot 2r on +a, slot 2r + 1 on -a
#pragma unroll
        for (int a = 0; a < RN(r); ++a) {
          g[RI(r, a)] -= T(RS(a)) * gs;
#pragma unroll
          for (int bb = a; bb < RN(r); ++bb) H[hidx(RI(r, a), RI(r, bb))] += T(2) / T(3) * T(RS(a)) * T(RS(bb));
        }
      }
      if (lane_active(P, k)) {
        const int id3[3] = {0, 1, 6};
        const T gs = (cg(JL) - cg(JL + 1)) / T(3);
        for (int a = 0; a < 3; ++a) {
          g[id3[a]] -= e.gC[a] * gs;
          for (int bb = a; bb < 3; ++bb) H[hidx(id3[a], id3[bb])] += T(2) / T(3) * e.gC[a] * e.gC[bb];
        }
      }
#pragma unroll
      for (int q = 0; q < NHC; ++q) Rk[RCF::H + q] = H[HCT.p[q]];
      for (int i = 0; i < NZ; ++i) { Rk[RCF::G0 + i] = g[i]; Rk[RCF::G1 + i] = T(0); Rk[RCF::GD + i] = T(0); }
      for (int i = 0; i < NX; ++i) Rk[RCF::C + i] = T(0);
    }
    wsync(w);
  }
  MR_SWEEP void ls_finish_resto() {
    MR_UNIFORM_P();
    MR_ASSUME_LDS_STATE();
    const T big = T(IP_MULT_INIT_MAX);
    int ok_l = 1;
    T yv[NI];
    for (int j = 0; j < NI; ++j) yv[j] = T(0);
    if (own()) {
      const int k = ln;
      T z[NZS], dz[NZS];
      load_z(cur, z);
      for (int i = 0; i < NZS; ++i) dz[i] = S(SSF::DZ + i);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      row_values(k, z, e, d, act);
      auto cg = [&](int j) { return S(SSF::LAM + j) + Cf(CSF::RVP + j) - Cf(CSF::RVN + j); };
#pragma unroll
      for (int r = 0; r < NROW; ++r) {
        if (!act[2 * r]) continue;
        const T adz = row_c(r, dz);
        yv[2 * r] = (cg(2 * r) - adz) / T(3);
        yv[2 * r + 1] = (cg(2 * r + 1) + adz) / T(3);
      }
      if (lane_active(P, k)) {
        const T adz = e.gC[0] * dz[0] + e.gC[1] * dz[1] + e.gC[2] * dz[6];
        yv[JL] = (cg(JL) - adz) / T(3);
        yv[JL + 1] = (cg(JL + 1) + adz) / T(3);
      }
      for (int j = 0; j < NI; ++j) ok_l &= mr_abs(yv[j]) <= big ? 1 : 0;
      if (k >= 1)
        for (int i = 0; i < 6; ++i) ok_l &= mr_abs(S(SSF::DNU + i)) <= big ? 1 : 0;
      else  // the initial-state rows' multipliers (dx_0 = 0: stage 0's costate), checked, not kept
        for (int i = 0; i <= 6; ++i) ok_l &= mr_abs(R(0)[RCF::PV0 + i]) <= big ? 1 : 0;
    }
    const bool ok = wall(w, ok_l != 0);
    if (own()) {
      const int k = ln;
      for (int i = 0; i < NX; ++i) {
        if (ok && k >= 1) NUd(i) = (double)S(SSF::DNU + i);
        S(SSF::DNU + i) = T(0);
      }
      for (int i = 0; i < NZS; ++i) S(SSF::DZ + i) = T(0);
      for (int j = 0; j < NI; ++j) {
        if (ok) Cf(CSF::RY + j) = yv[j];
        Cf(CSF::RDY + j) = T(0);
        Cf(CSF::RDP + j) = T(0); Cf(CSF::RDN + j) = T(0); Cf(CSF::RDVP + j) = T(0); Cf(CSF::RDVN + j) = T(0);
        S(SSF::DS + j) = T(0);
        S(SSF::DLAM + j) = T(0);
      }
      for (int i = 0; i < 6; ++i) {
        Cf(CSF::CDP + i) = T(0); Cf(CSF::CDN + i) = T(0); Cf(CSF::CDVP + i) = T(0); Cf(CSF::CDVN + i) = T(0);
      }
    }
    wsync(w);
  }
  MR_HD void ls_resto() {
    ls_record_resto();
    if (!riccati<true>(T(0), mu)) return;  // (not positive definite on the null space: the multipliers stay 0)
    T ap, ad, gphi;
    forward_resto(ap, ad, gphi);
    ls_finish_resto();
  }
  MR_HD bool resto_done() {  // the accepted restoration step's point, seen by the original problem
    auto* C = cw();
    const T tho = C->tho, pho = C->pho;
    bool ok = tho <= T(RESTO_KAPPA) * C->th_entry;
    if (filter_hit_lds(tho, pho, C->onfilt, &C->ofilt[0], &C->ofilt[FMAX])) ok = false;
    if (C->onfilt > FMAX && filter_hit_ov(tho, pho, C->onfilt, 0)) ok = false;  // the original filter's bank
    return wuni(w, ok);
  }
  MR_SWEEP void resto_exit() {
    // mr_solver.h Solver::resto_exit: a two-sided row's distances rescaled to one slack; bound duals by a
    // complementarity Newton step over the whole restoration (dual fraction to the boundary), all reset to 1
    // if one exceeds 1000; y = 0; the original problem's barrier parameter, filter, perturbation state
    MR_UNIFORM_P();
    MR_ASSUME_LDS_STATE();
    auto* C = cw();
    const T mu_o = C->mu_o;
    const T tau = mr_max(T(0.99), T(1) - mu_o);
    T ad_l = T(1), vmax_l = T(0);
    if (own()) {
      const int k = ln;
      T z[NZS];
      load_z(cur, z);
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      row_values(k, z, e, d, act);
      for (int r = 2; r <= NROW; ++r) {
        const int j0 = r < NROW ? 2 * r : JL;
        if (!act[j0]) continue;
        const T t0 = S(sf(cur) + j0), t1 = S(sf(cur) + j0 + 1), rng = d[j0] + d[j0 + 1];
        S(sf(cur) + j0) = t0 * rng / (t0 + t1);
        S(sf(cur) + j0 + 1) = t1 * rng / (t0 + t1);
      }
      for (int j = 0; j < NI; ++j) {
        S(SSF::DLAM + j) = T(0);
        if (!act[j]) continue;
        const T t0 = Cf(CSF::RS0 + j), v0 = Cf(CSF::RLAM + j), t = S(sf(cur) + j);
        const T dv = mu_o / t0 - v0 - v0 / t0 * (t - t0);
        S(SSF::DLAM + j) = dv;
        if (dv < T(0)) ad_l = mr_min(ad_l, -tau * v0 / dv);
      }
    }
    const T ad = wmin(w, ad_l);
    if (own())
      for (int j = 0; j < NI; ++j) {
        const T v0 = Cf(CSF::RLAM + j);
        const T v = v0 == T(0) ? T(0) : v0 + ad * S(SSF::DLAM + j);
        S(SSF::LAM + j) = v;
        vmax_l = mr_max(vmax_l, mr_abs(v));
      }
    const T vmax = wmax(w, vmax_l);
    if (own()) {
      for (int j = 0; j < NI; ++j) {
        if (vmax > T(RESTO_MULT_RESET) && Cf(CSF::RLAM + j) != T(0)) S(SSF::LAM + j) = T(1);
        S(SSF::DLAM + j) = T(0);
        S(SSF::Y + j) = T(0);
        S(SSF::DY + j) = T(0);
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
  // IPOPT's backup acceptable iterate (RestoreAcceptablePoint): stored when the current point is acceptable
  // -- the whole iterate, primal part, slacks and every multiplier (bound duals, row multipliers y_d, the
  // fp64 dynamics multipliers) -- and returned whole if the line search later fails at an almost feasible
  // point or the fp32 stall exit fires, so the exported lam_g belongs to the returned X / U
  MR_SWEEP void acc_save() {
    MR_ASSUME_LDS_STATE();
    if (own()) {
      for (int i = 0; i < NZS; ++i) Cf(CSF::AZ + i) = S(zf(cur) + i);
      for (int j = 0; j < NI; ++j) {
        Cf(CSF::ASL + j) = S(sf(cur) + j);
        Cf(CSF::ALAM + j) = S(SSF::LAM + j);
        Cf(CSF::AY + j) = S(SSF::Y + j);
      }
      for (int i = 0; i < NX; ++i) ANUd(i) = NUd(i);
    }
    cw()->have_acc = 1;
    wsync(w);
  }
  MR_SWEEP void acc_restore() {
    MR_ASSUME_LDS_STATE();
    if (own()) {
      for (int i = 0; i < NZS; ++i) S(zf(cur) + i) = Cf(CSF::AZ + i);
      for (int j = 0; j < NI; ++j) {
        S(sf(cur) + j) = Cf(CSF::ASL + j);
        S(SSF::LAM + j) = Cf(CSF::ALAM + j);
        S(SSF::Y + j) = Cf(CSF::AY + j);
      }
      for (int i = 0; i < NX; ++i) NUd(i) = ANUd(i);
    }
    wsync(w);
  }

  // IPOPT's primal-dual system error (the soft restoration phase's measure; oracle/ipopt.py pd_error): the
  // 1-norms of the Lagrangian gradient in the reference's variables (States, S_hat, U), of the slacks'
  // stationarity -y - v_L + v_U, of the equality residuals c and d - s, and of v t - mu, at the current
  // iterate (TRIAL false) or at the trial point in buffer 1-cur with every multiplier stepped by a (the soft
  // restoration step's one step size).  Only its ratio between two points is used, so the count of terms
  // (equal at both) is not divided out.  Stage-parallel, like eval_sweep's stationarity (fp64 dynamics
  // multipliers, correction-form dd); rare (failed line searches only), so the Hessian the generated
  // dynamics code computes alongside is simply discarded.  Result in res_th.
  template <bool TRIAL>
  MR_SWEEP void pd_sweep(T a) {
    MR_UNIFORM_P();
    MR_ASSUME_LDS_STATE();
    const int k = ln, b = TRIAL ? 1 - cur : cur;
    const double ad = TRIAL ? (double)a : 0.0;
    const T at = TRIAL ? a : T(0);
    T z[NZS];
    load_z(b, z);
    T znext[NX];
    for (int i = 0; i < NX; ++i) znext[i] = wnext(w, z[i]);
    double nuk[NX];
    for (int i = 0; i < NX; ++i) nuk[i] = (own() && (k >= 1 || !MR_KKT_RESTATED)) ? NUd(i) + ad * (double)S(SSF::DNU + i) : 0.0;
    double nnd[NX];
    for (int i = 0; i < NX; ++i) nnd[i] = wnext(w, own() && k >= 1 ? nuk[i] : 0.0);
    T sum_l = T(0), rs_a = T(0), rs_b = T(0), rs_u[2] = {T(0), T(0)}, rs_p[2] = {T(0), T(0)}, rs_w[2] = {T(0), T(0)};
    if (own()) {
      T st[NZ], J[48];
      double dd[NZ];
      for (int i = 0; i < NZ; ++i) { st[i] = T(0); dd[i] = 0.0; }
      for (int i = 0; i < 48; ++i) J[i] = T(0);
      if (k < N) {
        T Hd[36], fx[6], nz[NX];
        for (int i = 0; i < NX; ++i) nz[i] = T(0);
        Dyn<T, MODEL>::fjh(P, z, z + NX, nz, fx, J, Hd);
        T c[NX];
        for (int i = 0; i < 6; ++i) c[i] = fx[i] - znext[i];
        c[6] = z[6] + z[13] - znext[6];
        c[7] = z[11] - znext[7];
        c[8] = z[12] - znext[8];
        c[9] = (k == 0 ? z[11] : z[9]) - znext[9];
        c[10] = (k == 0 ? z[12] : z[10]) - znext[10];
        for (int i = 0; i < NX; ++i) sum_l += mr_abs(c[i]);
        apply_At(J, k, nnd, dd);
        apply_Bt(J, k, nnd, dd + NX);
      }
      for (int i = 0; i < NX; ++i) dd[i] -= nuk[i];
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      stage_cost(P, I, k, z, e, sc, st, (T*)nullptr);
      T d[NI];
      int act[NI];
      row_values(k, z, e, d, act);
      T lam_j[NI], t_j[NI], y_j[NI];
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        lam_j[j] = y_j[j] = T(0);
        t_j[j] = T(1);
        if (!act[j]) continue;
        const T t = S(sf(b) + j), lam = S(SSF::LAM + j) + at * S(SSF::DLAM + j);
        lam_j[j] = lam;
        t_j[j] = t;
        sum_l += mr_abs(lam * t - mu);
        if (yslot(j)) {
          y_j[j] = S(SSF::Y + j) + at * S(SSF::DY + j);
          sum_l += mr_abs(d[j] - t);
        }
      }
#pragma unroll
      for (int r = 0; r < NROW; ++r) {
        const int j0 = 2 * r, j1 = j0 + 1;
        if (!act[j0]) continue;
        T ys;
        if (r < 2) {
          ys = y_j[j0] + y_j[j1];
          sum_l += mr_abs(-y_j[j0] - lam_j[j0]) + mr_abs(-y_j[j1] + lam_j[j1]);
        } else {
          ys = y_j[j0];
          sum_l += mr_abs(-y_j[j0] - lam_j[j0] + lam_j[j1]);
        }
#pragma unroll
        for (int q = 0; q < RN(r); ++q) st[RI(r, q)] += ys * T(RS(q));
      }
      if (lane_active(P, k)) {
        const T ys = y_j[JL];
        sum_l += mr_abs(-ys - lam_j[JL] + lam_j[JL + 1]);
        st[0] += ys * e.gC[0];
        st[1] += ys * e.gC[1];
        st[6] += ys * e.gC[2];
      }
      T sti[NZ];
      for (int i = 0; i < NZ; ++i) sti[i] = T((double)st[i] + dd[i]);
      for (int i = 0; i < 6; ++i) sum_l += mr_abs(sti[i]);  // X_k (k = 0: with the initial-state rows' nu_0)
      rs_a = sti[6];
      rs_b = k < N ? sti[13] : T(0);
      if (k < N) { rs_u[0] = sti[11]; rs_u[1] = sti[12]; }
      if (k >= 1) { rs_p[0] = sti[7]; rs_p[1] = sti[8]; rs_w[0] = sti[9]; rs_w[1] = sti[10]; }
    }
    // S_k = S_k + Delta-S_{k-1} - Delta-S_k; U_k = u_k + p_{k+1} (U_0: + every w_j), as eval_sweep
    const T bprev = wprev(w, rs_b), pn0 = wnext(w, rs_p[0]), pn1 = wnext(w, rs_p[1]);
    const T ws0 = wsum(w, rs_w[0]), ws1 = wsum(w, rs_w[1]);
    if (own()) {
      sum_l += mr_abs(rs_a + (k >= 1 ? bprev : T(0)) - rs_b);
      if (k < N) {
        sum_l += mr_abs(rs_u[0] + pn0 + (k == 0 ? ws0 : T(0)));
        sum_l += mr_abs(rs_u[1] + pn1 + (k == 0 ? ws1 : T(0)));
      }
    }
    res_th = wsum(w, sum_l);
  }

  // IPOPT's TrySoftRestoStep (oracle/ipopt.py try_soft_resto): the full primal-dual step with one step size
  // a = min(alpha_primal_max, alpha_dual_max); accepted if the filter / sufficient-decrease test against the
  // current point passes (1: "accepted by the original criterion", an h-type step), else if the primal-dual
  // error falls by soft_resto_pderror_reduction_factor (2); 0 rejected.  The trial point is in buffer 1-cur,
  // res_alpha = a.
  MR_HD int soft_resto(T th, T ph, T gphi, T th_pow, T ap, T ad) {
    const T a = mr_min(ap, ad);
    line_search<false, false>(th, ph, gphi, th_pow, a, a, a, 0, LS_FORCE, a);
    if (!(res_flags & LSR_FIN)) return 0;
    const T th_t = res_th, ph_t = res_ph;
    const LSRef<T> ref{th, ph, gphi, th_pow};
    int r = 0;
    if (th_t <= theta_max && acc_to_iterate(th_t, ph_t, ref) && filter_ok(th_t, ph_t)) {
      r = 1;
    } else {
      pd_sweep<true>(a);
      const T pd_t = res_th;
      pd_sweep<false>(T(0));
      r = pd_t <= T(IP_SOFT_RESTO_FACTOR) * res_th ? 2 : 0;
    }
    res_alpha = a;
    return r;
  }

  // IPOPT's tiny-step test (mr_solver.h Solver::tiny_step; tiny_step_tol 10 eps of double, IPOPT's): at a point
  // with primal infeasibility <= 1e-4, every step component of the reference's variables (global X, Y, S)
  // and of IPOPT's slacks below 10 eps relative to 1 + |value|.  res_flags: 1 tiny, 2 the multipliers' steps
  // also below tiny_step_y_tol (1e-2).  Lane = stage, AND-reduced.
  MR_SWEEP void tiny_check() {
    MR_UNIFORM_P();
    MR_ASSUME_LDS_STATE();
    int tiny_l = 1, ys_l = 1;
    if (own()) {
      const int k = ln;
      const T tt = T(IP_TINY_STEP_TOL);
      T z[NZS];
      load_z(cur, z);
      for (int i = 0; i < NZ; ++i) {
        if (!delta_var(i) || (k == 0 && i <= 6) || (k == N && i >= NX)) continue;
        const T org = i == 0 ? I.org[0] : (i == 1 ? I.org[1] : (i == 6 ? I.org[2] : T(0)));
        if (mr_abs(S(SSF::DZ + i)) > tt * (T(1) + mr_abs(z[i] + org))) tiny_l = 0;
      }
      Err<T> e;
      errors(I, z[0], z[1], z[6], e, false);
      T d[NI];
      int act[NI];
      row_values(k, z, e, d, act);
#pragma unroll
      for (int j = 0; j < NI; ++j) {
        if (!act[j] || !yslot(j)) continue;
        const T c = j < JL ? row_c(j / 2, z) : e.eC;
        const T sv = c - T(slot_sign(j)) * (d[j] - S(sf(cur) + j));  // IPOPT's slack value
        if (mr_abs(S(SSF::DS + j)) > tt * (T(1) + mr_abs(sv))) tiny_l = 0;
        if (!(mr_abs(S(SSF::DY + j)) < T(1e-2))) ys_l = 0;
      }
      for (int i = 0; i < NX; ++i)
        if ((i < 6 || (k == 0 && i == 6)) && !(mr_abs(S(SSF::DNU + i)) < T(1e-2))) ys_l = 0;
    }
    const int t = wall(w, tiny_l != 0), y = wall(w, ys_l != 0);
    res_flags = (t ? 1 : 0) | (y ? 2 : 0);
  }

  // ---------------- the IPM loop (wave-uniform control; mr_solver.h Solver::solve, same rules) ----------------
  MR_HD SolveOut solve() {
    MR_UNIFORM_P();
    const T kappa_eps = T(10), kappa_mu = T(0.2), theta_mu = T(1.5);
    // IPOPT's monotone update keeps mu >= min(tol, compl_inf_tol) / (barrier_tol_factor + 1)
    const T mu_min = mr_max(T(1e-11), mr_min(P.tol, T(IP_COMPL_INF_TOL)) / (kappa_eps + T(1)));
    const T g_th = T(1e-5), g_ph = T(1e-5);
    SolveOut out{2, 0, 0.0, 0.0, 0.0};
    double acc_kkt = 0.0, acc_obj = 0.0, acc_viol = 0.0;  // the stored acceptable point's measures
    T mu_prev = mu;
    int acc_count = 0, stall = 0;
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
#ifdef MR_WAVE_STATS
    long st_trials = 0, st_soc_try = 0, st_soc_ok = 0, st_resto = 0, st_wd = 0, st_fact = 0, st_lsfail = 0;
#define MR_STAT(x) (x)
#else
#define MR_STAT(x) ((void)0)
#endif
    for (it = 0;; ++it) {
      // wave-uniform mode of this iteration: the original problem, or its restoration phase
      const bool rs = wuni(w, cw()->resto != 0);
      MR_T0();
      if (rs) eval_sweep<true>(mu_prev); else eval_sweep<false>(mu_prev);
      MR_T1(0);
      const T kkt = nlp_error(rs);
      if (!(kkt == kkt) || !(fval == fval)) { out.status = 3; break; }
      if (rs) {
        // the restoration NLP converged at a point the original problem does not accept: restoration
        // failed when that point is feasible to 1e2 tol (IPOPT), else a point of local infeasibility
        out.viol = (double)mr_max(cw()->pr_o, cw()->viol);  // the restoration iterate as the original problem sees it
        if (kkt <= P.tol) { out.status = cw()->pr_o <= T(100) * P.tol ? 3 : MR_STATUS_INFEASIBLE; break; }
      } else {
        out.kkt = (double)kkt;
        out.obj = (double)(fval / sc);
        out.viol = (double)mr_max(cw()->pr_eq, cw()->viol);
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
          stall = (mu <= mu_min && mr_max(cw()->pr_eq, cw()->viol) <= T(IP_CONSTR_VIOL_TOL)) ? stall + 1 : 0;
          if (stall >= MR_F32_STALL) {
            if (cw()->have_acc) {
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
      // IPOPT's monotone barrier update; a tiny step forces a decrease (at the smallest mu: "search direction
      // becomes too small", status 3); none in the restoration phase's first iteration (MonotoneMuUpdate)
      T mu_old = mu;
      bool tflag = cw()->tiny != 0, mu_stuck = false;
      const bool skip_mu = rs && cw()->resto_first != 0;
      cw()->tiny = 0;
      cw()->resto_first = 0;
      while (!skip_mu && (barrier_error(mu) <= kappa_eps * mu || tflag)) {
        const T m1 = kappa_mu * mu, m2 = mr_exp(theta_mu * mr_log(mu));
        const T mn = mr_max(mu_min, mr_min(m1, m2));
        if (mn == mu) { mu_stuck = tflag; break; }
        mu = mn;
        tflag = false;
      }
      if (mu_stuck) { out.status = 3; break; }
      if (mu != mu_old) {  // IPOPT resets its line search with a new barrier problem: filter, watchdog, soft restoration
        nfilt = 0;
        cw()->in_wd = 0;
        cw()->wd_short = 0;
        cw()->in_soft = 0;
        cw()->soft_count = 0;
      }
      const T ph_cur = fval - mu * logs + T(IP_KAPPA_D) * mu * cw()->lins;  // barrier objective (+ damping)
      // inertia-corrected factorisation (IPOPT's PDPerturbationHandler, mr_solver.h)
      T delta = T(0);
      bool first = true, fact_ok = false;
      MR_T0();
      for (int tries = 0; tries < 200; ++tries) {
        MR_CNT(6);
#if MR_PHASE_CYCLES
        const unsigned long long tr0 = trace ? MR_CLOCK() : 0ull;
        const bool rok = rs ? riccati<true>(delta, mu)
                            : (delta > T(0) ? riccati<false, true>(delta, mu) : riccati<false, false>(delta, mu));
        if (trace && !rok) { tsub[4] += MR_CLOCK() - tr0; tsub[5] += 1; }
        if (rok) { fact_ok = true; break; }
#else
        MR_STAT(st_fact++);
        if (rs ? riccati<true>(delta, mu)
               : (delta > T(0) ? riccati<false, true>(delta, mu) : riccati<false, false>(delta, mu))) {
          fact_ok = true;
          break;
        }
#endif
        if (first) {
          delta = delta_last == T(0) ? T(1e-4) : mr_max(T(1e-20), delta_last / T(3));
          first = false;
        } else {
          delta *= (delta_last == T(0) || T(1e5) * delta_last < delta) ? T(100) : T(8);
        }
        if (delta > T(1e40)) break;
      }
      MR_T1(1);
      if (!fact_ok) {
        if (rs) { out.status = 3; break; }
        // IPOPT: no inertia-correct factorisation -> the restoration phase
        resto_enter(theta, ph_cur);
        mu_prev = mu;
        cw()->in_wd = 0;
        cw()->wd_short = 0;
        acc_count = 0;
        continue;
      }
      if (delta > T(0)) delta_last = delta;
      cw()->delta_it = delta;
      T &ap = res_ap, &ad = res_ad, &gphi = res_gphi;
      MR_T0();
      if (rs) forward_resto(ap, ad, gphi); else forward(ap, ad, gphi);
      MR_T1(2);
      T th = theta, ph = ph_cur;
      T th_pow = mr_exp(T(1.1) * mr_log(mr_max(th, T(1e-30))));
      T a_min = alpha_min_of(th, gphi);
      if (rs) {  // a restoration-phase step: its own filter, no watchdog, no second-order correction
        MR_T0();
        line_search<true, false>(th, ph, gphi, th_pow, ap, ap, a_min, 0, 0, T(0));
        MR_T1(3);
        MR_STAT((st_resto++, st_trials += res_ntr));
        if (!(res_flags & LSR_ACC)) { out.status = 3; break; }  // IPOPT: restoration failed
        cw()->fo_cur = cw()->fo;  // the accepted step's point is the last trial evaluated (no SOC here)
        if (res_flags & LSR_AUG) filter_add((T(1) - g_th) * th, ph - g_ph * th);
        if (trace && ln == 0 && it < trace_cap - MR_TRACE_RESERVED) {
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
      if (acceptable(kkt)) {  // IPOPT stores the current iterate if it is acceptable
        acc_save();
        acc_kkt = out.kkt; acc_obj = out.obj; acc_viol = out.viol;
      }
      bool take_anyway = false, accepted = false, soc_taken = false, rejf = false, tiny = false, soft_step = false,
           soft_orig = false;
      T alpha = ap;
      T uth = th, uph = ph;  // the accepting line search's reference (the filter entry on augmentation)
      int flags = 0;
      MR_T0();
      if (MR_SOFT_RESTO && wuni(w, cw()->in_soft != 0)) {
        // the soft restoration phase continues (IPOPT: max_soft_resto_iters): its step replaces the line search
        if (++cw()->soft_count <= IP_MAX_SOFT_RESTO) {
          const int sr = soft_resto(th, ph, gphi, th_pow, ap, ad);
          if (sr) {
            accepted = soft_step = true;
            soft_orig = sr == 1;
            if (soft_orig) { cw()->in_soft = 0; cw()->soft_count = 0; }
          }
        }
      } else {
#if MR_WD_TRIGGER > 0
        // IPOPT's watchdog (mr_solver.h, same rule): after watchdog_shortened_iter_trigger successive
        // shortened steps store the iterate and direction, take full steps tentatively, judged against the
        // stored point at its step size; after watchdog_trial_iter_max without an acceptable one, back to the
        // stored point and a regular backtracking line search that skips the full step
        if (!cw()->in_wd && cw()->wd_short >= MR_WD_TRIGGER) {
          wd_save();
          auto* C = cw();
          C->wd_th = th; C->wd_ph = ph; C->wd_gphi = gphi; C->wd_ap = ap; C->wd_ad = ad; C->wd_amin = a_min;
          C->wd_thpow = th_pow;
          C->in_wd = 1;
          C->wd_trial = 0;
        }
#endif
        bool ysmall = false;
        if (MR_TINY_STEP) {
          tiny_check();
          tiny = (res_flags & 1) != 0;
          ysmall = (res_flags & 2) != 0;
        }
        if (tiny) {  // IPOPT: a tiny step is taken without a line search (and, with small multiplier steps,
                     // forces a barrier decrease)
          line_search<false, false>(th, ph, gphi, th_pow, ap, ap, ap, 0, LS_FORCE, ap);
          accepted = true;
          cw()->tiny = ysmall ? 1 : 0;
        } else if (wuni(w, cw()->in_wd != 0)) {
          auto* C = cw();
          line_search<false, false>(C->wd_th, C->wd_ph, C->wd_gphi, C->wd_thpow, ap, ap, ap, 0, LS_WD, C->wd_ap);
          flags = res_flags;
          rejf |= (flags & LSR_REJF) != 0;
          uth = C->wd_th;
          uph = C->wd_ph;
          if (flags & LSR_ACC) {
            accepted = true;
            C->in_wd = 0;
            C->wd_short = 0;
          } else if (++C->wd_trial <= MR_WD_TRIAL_MAX) {
            take_anyway = true;  // the full step is taken tentatively (LS_WD stored that trial point already)
          } else {
            // back to the watchdog point: its iterate and direction, a regular backtracking line search
            // that skips the full step
            wd_restore();
            C->in_wd = 0;
            C->wd_short = 0;
            th = C->wd_th; ph = C->wd_ph; gphi = C->wd_gphi; ap = C->wd_ap; ad = C->wd_ad; a_min = C->wd_amin;
            th_pow = C->wd_thpow;
            uth = th;
            uph = ph;
            line_search<false, false>(th, ph, gphi, th_pow, T(0.5) * ap, ap, a_min, 1, LS_NOSOC, T(0));
            flags = res_flags;
            rejf |= (flags & LSR_REJF) != 0;
            accepted = (flags & LSR_ACC) != 0;
          }
        } else {
#if MR_PHASE_CYCLES
          unsigned long long tq = trace ? MR_CLOCK() : 0ull;
#define MR_TQ(q) do { if (trace) { const unsigned long long tn = MR_CLOCK(); tsub[q] += tn - tq; tq = tn; } } while (0)
#else
#define MR_TQ(q) ((void)0)
#endif
          line_search<false, false>(th, ph, gphi, th_pow, ap, ap, a_min, 0, LS_CAP, T(0));
          MR_TQ(16);
          flags = res_flags;
          rejf |= (flags & LSR_REJF) != 0;
          accepted = (flags & LSR_ACC) != 0;
          if (flags & LSR_NEED_SOC) {
            // IPOPT's TrySecondOrderCorrection: up to max_soc (4) linear corrections while theta falls by
            // kappa_soc (0.99); then, if none is accepted, the backtracking resumes at alpha / 2
            const T a_trial = res_alpha, a_test0 = res_atest;
            T th_trial = res_th, a_soc = a_trial, th_old = T(0);
#if MR_PHASE_CYCLES
            if (trace) { tsub[22] += 1; tq = MR_CLOCK(); }
#endif
            for (int count = 0; count < IP_MAX_SOC; ++count) {
              if (count > 0 && !(th_trial <= T(IP_KAPPA_SOC) * th_old)) break;
              th_old = th_trial;
              // the trial point's constraint values: captured by its own evaluation (the first trial of the
              // line search, or the previous correction's trial), accumulated by soc_backward
              MR_TQ(17);
              MR_STAT(st_soc_try++);
              MR_CNT(5);
#if MR_PHASE_CYCLES
              const unsigned long long ts0 = trace ? MR_CLOCK() : 0ull;
#endif
              soc_backward(count == 0, a_soc);
#if MR_PHASE_CYCLES
              const unsigned long long ts1 = trace ? MR_CLOCK() : 0ull;
#endif
              T aps, ads;
              forward_soc(aps, ads);
#if MR_PHASE_CYCLES
              if (trace) { tsub[6] += ts1 - ts0; tsub[7] += MR_CLOCK() - ts1; }
#endif
#if MR_PHASE_CYCLES
              if (trace) tq = MR_CLOCK();
#endif
              line_search<false, true>(th, ph, gphi, th_pow, aps, aps, aps, 0, LS_WD | LS_CAP,
                                       a_test0);
              MR_TQ(18);
              rejf |= (res_flags & LSR_REJF) != 0;
              a_soc = aps;
              if (!(res_flags & LSR_FIN)) break;
              if (res_flags & LSR_ACC) {
                soc_taken = accepted = true;
                flags = res_flags;
                ad = soc_commit();
                MR_TQ(19);
                break;
              }
              th_trial = res_th;
            }
            if (!soc_taken) {
#if MR_PHASE_CYCLES
              if (trace) { tsub[23] += 1; tq = MR_CLOCK(); }
#endif
              line_search<false, false>(th, ph, gphi, th_pow, T(0.5) * a_trial, ap, a_min, 1, LS_NOSOC, T(0));
              MR_TQ(20);
              flags = res_flags;
              rejf |= (flags & LSR_REJF) != 0;
              accepted = (flags & LSR_ACC) != 0;
            }
          }
        }
        if (MR_SOFT_RESTO && !accepted && !take_anyway) {
          // IPOPT's soft restoration phase before the restoration phase proper (TrySoftRestoStep)
#if MR_PHASE_CYCLES
          const unsigned long long tsr = trace ? MR_CLOCK() : 0ull;
#endif
          const int sr = soft_resto(th, ph, gphi, th_pow, ap, ad);
#if MR_PHASE_CYCLES
          if (trace) tsub[21] += MR_CLOCK() - tsr;
#endif
          if (sr) {
            accepted = soft_step = true;
            soft_orig = sr == 1;
            cw()->in_soft = soft_orig ? 0 : 1;
            cw()->soft_count = 0;
            uth = th;
            uph = ph;
          }
        }
      }
      MR_T1(3);
#if MR_PHASE_CYCLES
      cyc[4] += res_ntr;
#endif
      alpha = res_alpha;
      const int nls = res_nls;
      MR_STAT((st_trials += res_ntr, st_soc_ok += soc_taken, st_wd += take_anyway, st_lsfail += (!accepted && !take_anyway)));
      if (!accepted && !take_anyway) {
        // IPOPT on a failed line search (and failed soft restoration): the current point acceptable ->
        // "acceptable point reached"; almost feasible (theta <= 1e-2 tol) -> the stored acceptable point or
        // restoration failed; otherwise the restoration phase
        if (acceptable(kkt)) { out.status = 1; break; }
        if (theta <= T(1e-2) * P.tol ||
            (sizeof(T) == 4 && mr_max(cw()->pr_eq, cw()->viol) <= T(IP_CONSTR_VIOL_TOL))) {  // fp32: feasible at its resolution
          if (cw()->have_acc) {
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
        cw()->in_wd = 0;
        cw()->wd_short = 0;
        acc_count = 0;
        if (trace && ln == 0 && it < trace_cap - MR_TRACE_RESERVED) {
          double* tr = trace + 8 * it;
          tr[0] = (double)kkt; tr[1] = (double)mu; tr[2] = 0.0; tr[3] = 0.0;
          tr[4] = (double)delta; tr[5] = (double)th; tr[6] = (double)ph; tr[7] = -300.0;
        }
        continue;
      }
      if (!take_anyway && !tiny && !soft_step) cw()->wd_short = (accepted && alpha < ap) ? cw()->wd_short + 1 : 0;
#if MR_FILTER_RESET_TRIGGER > 0
      if (filt_resets < MR_MAX_FILTER_RESETS) {
        filt_rej_iters = rejf ? filt_rej_iters + 1 : 0;
        if (filt_rej_iters >= MR_FILTER_RESET_TRIGGER) {
          nfilt = 0;
          filt_resets++;
          filt_rej_iters = 0;
        }
      }
#endif
      // IPOPT augments the filter unless the step is f-type with the Armijo condition (a tiny step: never; a
      // soft restoration step: only when the regular criterion accepted it -- an h-type step)
      if (!take_anyway && (soft_step ? soft_orig : (!tiny && (flags & LSR_AUG))))
        filter_add((T(1) - g_th) * uth, uph - g_ph * uth);
      if (soft_step) ad = alpha;  // the soft restoration step moves every variable by one step size
      if (trace && ln == 0 && it < trace_cap - MR_TRACE_RESERVED) {
        double* tr = trace + 8 * it;
        tr[0] = (double)kkt; tr[1] = (double)mu; tr[2] = (double)alpha; tr[3] = (double)ad;
        tr[4] = (double)delta; tr[5] = (double)uth; tr[6] = (double)uph;
        tr[7] = (double)(take_anyway ? -100 - cw()->wd_trial : (soc_taken ? 100 + nls : nls));
      }
      alpha_p = alpha;
      alpha_d = ad;
      mu_prev = mu;
      cur = 1 - cur;
      wsync(w);  // new iterate buffer written by every lane before the next evaluation
    }
    out.iters = it;
    // a solve that ends inside the restoration phase returns the restoration iterate: its objective is the
    // original problem's there (the restoration NLP's own objective is rho |p + n| + proximity), its
    // constraint violation out.viol was set as the original problem's at the loop top
    if (wuni(w, cw()->resto != 0)) out.obj = (double)(cw()->fo_cur / sc);
#ifdef MR_WAVE_STATS
    if (ln == 0)
      printf("wave stats: status %d iters %d trials %ld soc_try %ld soc_ok %ld resto %ld wd %ld fact %ld lsfail %ld\n",
             out.status, it, st_trials, st_soc_try, st_soc_ok, st_resto, st_wd, st_fact, st_lsfail);
#endif
#undef MR_STAT
#undef MR_T0
#undef MR_T1
#undef MR_CNT
#undef MR_TQ
#if MR_PHASE_CYCLES
    if (trace && ln == 0 && trace_cap >= 2) {  // last row: cycles eval, riccati, forward, trial, #trials, #soc, #factorisations, total
      double* tr = trace + 8 * (trace_cap - 1);
      for (int q = 0; q < 7; ++q) tr[q] = (double)cyc[q];
      tr[7] = (double)(trace ? MR_CLOCK() - tstart : 0ull);
      double* tr2 = trace + 8 * (trace_cap - 2);  // sub-phases: forward seq/par, eval stage/reduce, failed factorisations (cycles, count), SOC backward / forward
      for (int q = 0; q < 8; ++q) tr2[q] = (double)tsub[q];
      if (trace_cap >= 3) {  // trial sub-phases: stage values, reductions, acceptance tests; line-search setup
        double* tr3 = trace + 8 * (trace_cap - 3);
        for (int q = 0; q < 8; ++q) tr3[q] = (double)tsub[8 + q];
      }
      if (trace_cap >= 4) {  // line-search phase split: first line search, SOC accumulation (0 since it moved
        // into soc_backward), SOC trial line searches, SOC commit, resumed backtracking, soft restoration; #SOC
        // episodes, #resumed line searches
        double* tr4 = trace + 8 * (trace_cap - 4);
        for (int q = 0; q < 8; ++q) tr4[q] = (double)tsub[16 + q];
      }
    }
#endif
    if (trace && ln == 0 && it < trace_cap - MR_TRACE_RESERVED) {
      double* tr = trace + 8 * it;
      tr[0] = (double)out.kkt; tr[1] = (double)fval; tr[2] = (double)theta; tr[3] = (double)stat_max;
      tr[4] = (double)pr_max; tr[5] = (double)sc; tr[6] = (double)mu; tr[7] = 1000.0 + out.status;
    }
    return out;
  }
  MR_HD T alpha_min_of(T th, T gphi) const {
    T a = T(1e-5);
    if (gphi < T(0)) {
      a = mr_min(a, T(1e-5) * th / (-gphi));
      if (th <= theta_min) a = mr_min(a, mr_exp(T(1.1) * mr_log(mr_max(th, T(1e-30)))) / mr_exp(T(2.3) * mr_log(-gphi)));
    }
    return T(0.05) * a;
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
// sc*f + sum nu_{k+1}.(F(x_k, u_k) - x_{k+1}) + sum y_d (d - s), Opti's is f + lam_g.g with g = X_i -
// f(X_{i-1}, U_{i-1}), so the dynamics rows are -nu/sc; every inequality row of the reference is an IPOPT row
// of the restatement (Delta-S = the u[2] box, rate rows via the previous-control state p, the i = 0 wrap rows
// via the frozen copy w at k = N-1) and its lam_g is that row's own multiplier y_d / sc -- IPOPT's y_d, which
// CasADi returns as lam_g (positive at an active upper bound; the box rows' lower halves carry -v_L), not the
// slack bound duals v_U - v_L, which equal it only where the slack stationarity -y_d - v_L + v_U vanishes;
// S_0 and X_{:,0} follow from the reference's stationarity in those variables: lam_S0 = lam_ds(1),
// lam_X0 = A_0^T lam_dyn(1).
template <typename Solver>
MR_HD void write_lam_g(Solver& S, const mr_outputs& out, int64_t B, int64_t i, int N, Wv w) {
  typedef decltype(S.mu) T;
  const int k = w.lane;
  const double isc = 1.0 / (double)S.sc;
  const int rows = 13 * N + 9;
  auto put = [&](int row, double v) { out.lam_g[(int64_t)row * B + i] = v; };
  auto yd = [&](int j) { return (double)S.S(SSF::Y + j); };  // the row multiplier of slot j (a y-slot)
  double nu1[NX];
  for (int q = 0; q < NX; ++q) nu1[q] = wshfl(w, S.own() ? S.NUd(q) : 0.0, 1);
  const double ds1 = wshfl(w, S.own() && k < N ? yd(4) * isc : 0.0, 0);
  if (k >= 1 && k <= N)
    for (int q = 0; q < 6; ++q) put(7 + 7 * (k - 1) + q, -S.NUd(q) * isc);
  if (k < N) {
    put(7 + 7 * k + 6, yd(4) * isc);  // Delta-S row of i = k + 1 (u[2] box of stage k)
    const int b = 7 + 7 * N + 6 * k;
    put(b + 0, yd(1) * isc);  // U[0,k] < d_max
    put(b + 1, yd(0) * isc);  // U[0,k] > min_throttle
    put(b + 2, yd(3) * isc);  // U[1,k] < max_steer
    put(b + 3, yd(2) * isc);  // U[1,k] > min_steer
    if (k >= 1) {
      put(b + 4, yd(6) * isc);
      put(b + 5, yd(8) * isc);
    }
    if (k == N - 1) {  // i = 0 rate rows U[:,0] - U[:,N-1]: the frozen-copy rows at stage N-1
      const int b0 = 7 + 7 * N;
      put(b0 + 4, N >= 2 ? yd(10) * isc : 0.0);
      put(b0 + 5, N >= 2 ? yd(12) * isc : 0.0);
    }
  }
  if (k == 0) {
    put(0, ds1);  // S_0 == s0
    // A_0 at the returned point (after an acceptable-point restore the record holds the abandoned one's)
    T z[NZS], J[48], Hd[36], fx[6], nz[NX];
    S.load_z(S.cur, z);
    for (int q = 0; q < NX; ++q) nz[q] = T(0);
    const ProbParams<T>& Pg = *(const ProbParams<T>*)wu_ptr(&S.P);
    Dyn<T, Solver::kModel>::fjh(Pg, z, z + NX, nz, fx, J, Hd);
    double at[NX];
    apply_At(J, 0, nu1, at);
    for (int q = 0; q < 6; ++q) put(1 + q, -at[q] * isc);  // X_{q,0} == state0
    put(rows - 2, S.I.has_thr0 ? yd(6) * isc : NAN);
    put(rows - 1, S.I.has_steer0 ? yd(8) * isc : NAN);
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
  S.ls_init();
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
    if (out.constr_viol) out.constr_viol[i] = r.viol;
  }
}

}  // namespace mr
