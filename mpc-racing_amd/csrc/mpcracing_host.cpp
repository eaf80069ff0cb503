// Host (g++) build of the solver core -- TEST HARNESS ONLY.
//
// libmpcracing_host.so runs the very same per-instance solver source as the
// gfx950 kernel (mr_wave.h), each instance as an emulated 64-lane wavefront, so that the solver logic can be checked
// against the oracle in the CPU test suite (no GPU in the build container).
// The product path (mpc-racing_amd/control/MPC.py, mpcracing.batch) never
// loads this library; it requires libmpcracing.so and a GPU.
#include <stdlib.h>
#include <string.h>
#include <vector>
#include "mr_wave.h"
#include "mr_track.h"
#include "mr_agent.h"
#include "mr_plant.h"

using namespace mr;

template <typename T, int MODEL>
struct Job {
  const ProbParams<T>* P;
  const mr_inputs* in;
  const mr_outputs* out;
  int64_t B, i;
  T* ws;
  T* lds;
};

template <typename T, int MODEL>
static void wave_body(HostWave* hw, int lane, void* arg) {
  Job<T, MODEL>* j = (Job<T, MODEL>*)arg;
  Wv w{lane, hw};
  solve_instance_wave<T, MODEL>(*j->P, *j->in, *j->out, j->B, j->i, j->ws, j->lds, w);
  wsync(w);  // final rendezvous: every lane done before the wave is torn down
}

// Each instance runs as one emulated wavefront (64 fibers, mr_wave_prims.h) on one CPU thread.
template <typename T, int MODEL>
static void run(const mr_config& c, const TyreCoef<double>& tf, const TyreCoef<double>& tr, int B,
                const mr_inputs& in, const mr_outputs& out, int nthreads) {
  ProbParams<T> P;
  fill_params<T>(c, tf, tr, P);
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
  for (int i = 0; i < B; ++i) {
    // poisoned workspace / LDS: any read-before-write shows up as NaN (device memory is not zeroed)
    std::vector<T> ws((size_t)ws_words<T>(), (T)NAN), lds((size_t)LDS_WORDS, (T)NAN);
    Job<T, MODEL> job{&P, &in, &out, (int64_t)B, (int64_t)i, ws.data(), lds.data()};
    HostWave* hw = new HostWave();
    host_wave_run(*hw, &wave_body<T, MODEL>, &job);
    delete hw;
  }
}

// The scalar C++ solver (mr_solver.h Solver: the same IPM, one instance per CPU thread, no wave
// emulation) over a batch with OpenMP -- the CPU baseline that bench.py times beside the GPU
// (SURVEY §8(d) "C++ fp64 CPU SQP twin").  Per-thread workspace of (N+1) stage records.
template <typename T, int MODEL>
static void run_scalar(const mr_config& c, const TyreCoef<double>& tf, const TyreCoef<double>& tr, int B,
                       const mr_inputs& in, const mr_outputs& out, int nthreads) {
  ProbParams<T> P;
  fill_params<T>(c, tf, tr, P);
#pragma omp parallel num_threads(nthreads > 0 ? nthreads : 1)
  {
    std::vector<T> ws((size_t)(c.N + 1) * WF::NF, (T)NAN);
#pragma omp for schedule(dynamic, 1)
    for (int i = 0; i < B; ++i) solve_instance<T, MODEL>(P, in, out, (int64_t)B, (int64_t)i, WS<T>{ws.data(), 1});
  }
}

extern "C" {

int mrh_config_default(mr_config* c) {
  fill_default_config(c);
  return 0;
}

int mrh_solve_batch(const mr_config* c, const double* a_front, double Fz_front, const double* a_back,
                    double Fz_back, int B, const mr_inputs* in, mr_outputs* out, int nthreads) {
  TyreCoef<double> tf{}, tr{};
  if (a_front) tf = pacejka_coef(a_front, Fz_front);
  if (a_back) tr = pacejka_coef(a_back, Fz_back);
  if (c->max_iter < 0 || c->max_iter > FCAP - 2) return -1;  // the line-search filter's capacity (mr_create)
#define MR_CASE(T, M) run<T, M>(*c, tf, tr, B, *in, *out, nthreads)
#define MR_MODELS(T)                                                       \
  switch (c->model) {                                                      \
    case MR_MODEL_KINEMATIC: MR_CASE(T, MODEL_KIN); break;                 \
    case MR_MODEL_DYNAMIC: MR_CASE(T, MODEL_DYN); break;                   \
    case MR_MODEL_BLENDED: MR_CASE(T, MODEL_BLEND); break;                 \
    case MR_MODEL_BLENDED_PACEJKA: MR_CASE(T, MODEL_BLEND_PACEJKA); break; \
    case MR_MODEL_DYNAMIC_PACEJKA: MR_CASE(T, MODEL_DYN_PACEJKA); break;   \
    default: return -1;                                                    \
  }
  if (c->precision == MR_PREC_FP64) { MR_MODELS(double) } else { MR_MODELS(float) }
#undef MR_CASE
  return 0;
}

int mrh_solve_batch_scalar(const mr_config* c, const double* a_front, double Fz_front, const double* a_back,
                           double Fz_back, int B, const mr_inputs* in, mr_outputs* out, int nthreads) {
  TyreCoef<double> tf{}, tr{};
  if (a_front) tf = pacejka_coef(a_front, Fz_front);
  if (a_back) tr = pacejka_coef(a_back, Fz_back);
  if (c->N < 1 || c->N > 63) return -1;
  if (c->max_iter < 0 || c->max_iter > FCAP - 2) return -1;
#define MR_CASE(T, M) run_scalar<T, M>(*c, tf, tr, B, *in, *out, nthreads)
  if (c->precision == MR_PREC_FP64) { MR_MODELS(double) } else { MR_MODELS(float) }
#undef MR_CASE
  return 0;
}

// Generated dynamics (value, Jacobian, nu-weighted Hessian) at one point, fp64.
int mrh_eval_dynamics(const mr_config* c, const double* a_front, double Fz_front, const double* a_back,
                      double Fz_back, const double* x, const double* u, const double* nu, double* f, double* J,
                      double* H) {
  TyreCoef<double> tf{}, tr{};
  if (a_front) tf = pacejka_coef(a_front, Fz_front);
  if (a_back) tr = pacejka_coef(a_back, Fz_back);
  ProbParams<double> P;
  fill_params<double>(*c, tf, tr, P);
  switch (c->model) {
    case MR_MODEL_KINEMATIC: Dyn<double, MODEL_KIN>::fjh(P, x, u, nu, f, J, H); break;
    case MR_MODEL_DYNAMIC: Dyn<double, MODEL_DYN>::fjh(P, x, u, nu, f, J, H); break;
    case MR_MODEL_BLENDED: Dyn<double, MODEL_BLEND>::fjh(P, x, u, nu, f, J, H); break;
    case MR_MODEL_BLENDED_PACEJKA: Dyn<double, MODEL_BLEND_PACEJKA>::fjh(P, x, u, nu, f, J, H); break;
    case MR_MODEL_DYNAMIC_PACEJKA: Dyn<double, MODEL_DYN_PACEJKA>::fjh(P, x, u, nu, f, J, H); break;
    default: return -1;
  }
  return 0;
}

// ---- centerline geometry (mr_track.h) on host arrays: the same functions as the gfx950 kernels ----
int mrh_track_blob_size(int nt, int n_rows) { return track_layout(nt, n_rows).total; }
int mrh_track_build(const double* t, int nt, const double* cx, const double* cy, int nc, const double* el,
                    const double* er, int n_rows, double* blob) {
  track_tables(t, nt, cx, cy, nc, el, er, n_rows, blob);
  return 0;
}
int mrh_track_eval(const double* blob, int nt, double L, int n_rows, int n, const double* s, double* out, int* span) {
  TrackView T = track_view(blob, nt, L, n_rows);
  for (int i = 0; i < n; ++i) {
    double g[6];
    int sp;
    track_eval(T, s[i], g, &sp);
    for (int c = 0; c < 6; ++c) out[(int64_t)c * n + i] = g[c];
    if (span) span[i] = sp;
  }
  return 0;
}
int mrh_track_frame(const double* blob, int nt, double L, int n_rows, int n, const double* s, double* yaw,
                    double* kappa, double* nx, double* ny, double mcla, double* meank) {
  TrackView T = track_view(blob, nt, L, n_rows);
  for (int i = 0; i < n; ++i) {
    track_frame(T, s[i], yaw + i, kappa + i, nx + i, ny + i);
    if (meank) meank[i] = track_mean_curvature(T, s[i], mcla);
  }
  return 0;
}
int mrh_track_sign(const double* blob, int nt, double L, int n_rows, int n, const double* X, const double* Y,
                   const double* s, int* sign) {
  TrackView T = track_view(blob, nt, L, n_rows);
  for (int i = 0; i < n; ++i) sign[i] = track_error_sign(T, X[i], Y[i], s[i]);
  return 0;
}
int mrh_track_polyfit(const double* blob, int nt, double L, int n_rows, int n, const double* s, const double* la,
                      double* cx, double* cy) {
  TrackView T = track_view(blob, nt, L, n_rows);
  for (int i = 0; i < n; ++i) {
    double a[5], b[5];
    track_polyfit(T, s[i], la[i], a, b);
    for (int j = 0; j < 5; ++j) { cx[(int64_t)j * n + i] = a[j]; cy[(int64_t)j * n + i] = b[j]; }
  }
  return 0;
}
int mrh_track_polyfit_deg(const double* blob, int nt, double L, int n_rows, int n, const double* s, const double* la,
                          int deg, double* cx, double* cy) {
  TrackView T = track_view(blob, nt, L, n_rows);
  for (int i = 0; i < n; ++i) {
    double a[MR_POLY_DEG_MAX + 1], b[MR_POLY_DEG_MAX + 1];
    if (!track_polyfit_deg(T, s[i], la[i], deg, a, b)) return -1;
    for (int j = 0; j <= deg; ++j) { cx[(int64_t)j * n + i] = a[j]; cy[(int64_t)j * n + i] = b[j]; }
  }
  return 0;
}
int mrh_track_lookup(const double* blob, int nt, double L, int n_rows, int n, const double* s, const double* la,
                     double* err, int* lo, int* hi, int* arg) {
  TrackView T = track_view(blob, nt, L, n_rows);
  for (int i = 0; i < n; ++i) err[i] = lane_lookup(T, s[i], la[i], lo + i, hi + i, arg + i);
  return 0;
}
int mrh_track_projection(const double* blob, int nt, double L, int n_rows, int n, const double* X, const double* Y,
                         const double* lo, const double* hi, double* s, double* dist, int* nfev) {
  TrackView T = track_view(blob, nt, L, n_rows);
  for (int i = 0; i < n; ++i) {
    s[i] = brent_projection(T, X[i], Y[i], lo[i], hi[i], nfev + i);
    dist[i] = track_dist(T, s[i], X[i], Y[i]);
  }
  return 0;
}

int mrh_spline_from_waypoints(const double* x, const double* y, int n, int close_loop, double* t, double* cx,
                              double* cy, int* n_t, double* length) {
  const int np = spline_from_waypoints(x, y, n, close_loop, t, cx, cy, length);
  if (np < 0) return np;
  *n_t = np + 4;
  return 0;
}

// lane-width table build: the serial scan of mr_track.h lane_distance (the kernel's wave scan
// visits the same samples and breaks ties the same way)
int mrh_lane_table(const double* cblob, int cnt, double cL, int c_rows, const double* lblob, int lnt, double lL,
                   int n, const double* s, double* dist, double* s_lane) {
  TrackView C = track_view(cblob, cnt, cL, c_rows), Ln = track_view(lblob, lnt, lL, 0);
#pragma omp parallel for schedule(dynamic, 16)
  for (int i = 0; i < n; ++i) dist[i] = lane_distance(C, Ln, s[i], s_lane ? s_lane + i : nullptr);
  return 0;
}

int mrh_agent_sense(const double* blob, int nt, double L, int n_rows, int n, const double* X, const double* Y,
                    const double* prev, double lookback, double lookahead, double err_offset, double* progress,
                    double* error, double* cx, double* cy, double* merr) {
  TrackView T = track_view(blob, nt, L, n_rows);
  for (int i = 0; i < n; ++i) {
    AgentSense o;
    agent_sense(T, X[i], Y[i], prev ? prev[i] : NAN, lookback, lookahead, err_offset, o);
    progress[i] = o.progress;
    error[i] = o.error;
    for (int j = 0; j < 5; ++j) { cx[(int64_t)j * n + i] = o.cx[j]; cy[(int64_t)j * n + i] = o.cy[j]; }
    merr[i] = o.max_error;
  }
  return 0;
}
int mrh_plant_step(int model, int n, const double* state, const double* cmd, double dt, double* out) {
  for (int i = 0; i < n; ++i) {
    double x[6], o[6];
    for (int j = 0; j < 6; ++j) x[j] = state[(int64_t)j * n + i];
    plant_step(model, x, cmd[i], cmd[n + i], dt, o);
    for (int j = 0; j < 6; ++j) out[(int64_t)j * n + i] = o[j];
  }
  return 0;
}

// Pacejka jet (value, d/dalpha, d2/dalpha2) in fp64 and fp32.
int mrh_pacejka(const double* a, double Fz, double alpha, int fp32, double* out3) {
  TyreCoef<double> c = pacejka_coef(a, Fz);
  if (fp32) {
    TyreCoef<float> cf{(float)c.B, (float)c.C, (float)c.E, (float)c.BCD, (float)c.K2};
    TyreJet<float> j = pacejka_jet(cf, (float)alpha);
    out3[0] = j.v; out3[1] = j.d; out3[2] = j.dd;
  } else {
    TyreJet<double> j = pacejka_jet(c, alpha);
    out3[0] = j.v; out3[1] = j.d; out3[2] = j.dd;
  }
  return 0;
}

}  // extern "C"
