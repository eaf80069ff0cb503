/*
 * mpcracing.h -- C ABI of the MI355X batched racing-MPC solver (libmpcracing.so).
 *
 * Drop-in boundary for the reference's hot path: the reference has no FFI; its
 * boundary is the Python class control.MPC.MPC (AlexGisi/mpc-racing
 * control/MPC.py:10-22 constructor, :183-184 solution()).  Each entry point
 * below replaces a piece of that class:
 *
 *   mr_config_default / mr_create   <- FixedControllerParameters (control/ControllerParameters.py:3-23),
 *                                      VehicleParameters (models/VehicleParameters.py:3-41),
 *                                      the IPOPT options dict (control/MPC.py:151-161)
 *   mr_set_tyres                    <- learned Pacejka tyres substituted into f_vehicle
 *                                      (learning/vehicle.py:79-92, :155-160)
 *   mr_solve_batch                  <- MPC.__init__ build + opti.solve() + the ret tuple
 *                                      (control/MPC.py:30-181) for B independent instances
 *   mr_last_error                   <- the RuntimeError text printed at control/MPC.py:173
 *
 * Conventions: every function returns 0 on success and a negative code on error
 * (message via mr_last_error(), thread-local).  All batch arrays are caller-owned
 * DEVICE pointers (e.g. torch tensors' data_ptr()) in structure-of-arrays layout
 * with the instance index fastest: element [c][i] of a [C][B] array is at
 * ptr[c*B + i].  All I/O is float64 regardless of the handle's compute precision.
 * Calls are ordered on the given HIP stream; a handle is bound to one device and is
 * not thread-safe.
 */
#ifndef MPCRACING_H
#define MPCRACING_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version (mr_version()): bumped whenever a struct layout or an entry point's meaning changes, so
   a caller built against another header can refuse to run (101: mr_config.dispatch_order,
   mr_outputs.lam_g / timeline, mr_config without lane_penalty (hard lane rows), status 4 = infeasible;
   102: mr_inputs.order_hint, dispatch_order 2) */
#define MR_ABI_VERSION 102

#define MR_OK 0
#define MR_ERR_ARG (-1)
#define MR_ERR_HIP (-2)
#define MR_ERR_STATE (-3)

/* dynamics models of the NLP */
#define MR_MODEL_KINEMATIC 0       /* control/MPC.py:231-260 (f_vehicle_kinematic)          */
#define MR_MODEL_DYNAMIC 1         /* control/MPC.py:186-229 (f_vehicle, the reference NLP)  */
#define MR_MODEL_BLENDED 2         /* lambda*dyn + (1-lambda)*kin, models/BlendedBicycleModel.py:22-46 */
#define MR_MODEL_BLENDED_PACEJKA 3 /* blended with learned Pacejka lateral forces            */
#define MR_MODEL_DYNAMIC_PACEJKA 4 /* dynamic with learned Pacejka lateral forces            */

/* plant models of the closed loop (the numpy simulator-side models) */
#define MR_PLANT_KINEMATIC 0 /* models/KinematicBicycleModel.py:11-48 */
#define MR_PLANT_DYNAMIC 1   /* models/DynamicBicycleModel.py:16-78   */
#define MR_PLANT_BLENDED 2   /* models/BlendedBicycleModel.py:18-58   */

#define MR_PREC_FP64 0
#define MR_PREC_FP32 1

/* per-instance solver status (replaces the try/except + breakpoint() of control/MPC.py:164-181) */
#define MR_STATUS_SOLVED 0
#define MR_STATUS_ACCEPTABLE 1
#define MR_STATUS_MAX_ITER 2
#define MR_STATUS_FAILED 3 /* non-finite values, no inertia-correct factorisation, or the restoration
                              phase's line search failed (IPOPT: Restoration_Failed) */
#define MR_STATUS_INFEASIBLE 4 /* the restoration phase converged to a minimiser of the constraint
                                  violation the original problem does not accept (IPOPT:
                                  Infeasible_Problem_Detected, "local infeasibility") */

typedef struct mr_config {
  int32_t N;           /* horizon (FixedControllerParameters.N = 30 unless the caller passes N) */
  int32_t model;       /* MR_MODEL_* */
  int32_t precision;   /* MR_PREC_* : arithmetic type of the solve */
  int32_t lane_bounds; /* 1 enables |e_C(S_i, X_i)| <= max_error, i = 1..N (the commented MPC.py:135) */
  int32_t max_batch;   /* workspace capacity (instances) */
  int32_t device;      /* HIP device ordinal */
  int32_t max_iter;    /* FixedControllerParameters.max_iter = 500 */
  int32_t acceptable_iter; /* IPOPT acceptable_iter (15); 0 disables acceptable termination */
  double Ts;           /* sampling time */
  double tol;          /* KKT tolerance of the scaled NLP (IPOPT tol) */
  double acceptable_tol;
  /* FixedControllerParameters (control/ControllerParameters.py:3-23) */
  double lambda_s, alpha_L, min_steer, max_steer, min_throttle, max_steer_delta, min_steer_delta,
      max_throttle_delta, min_throttle_delta, q_v_max, v_max, min_s_delta;
  /* VehicleParameters (models/VehicleParameters.py:3-41); max_steer_deg = VehicleParameters.max_steer */
  double m, Iz, lf, lr, Cf, Cr, T_max, r_wheel, C_wheel, R, rho, C_d, A_f, C_roll, g, max_steer_deg,
      Vblendmin, Vblendmax;
  /* workgroup dispatch order of a batch (results do not depend on it: instances are independent):
     0 = instance order; 1 = (default) a stable three-tier partition so the likely long solves start
     first: tier 0 = v >= 40 m/s, or throttle <= -0.5 at v <= 20 m/s (hard braking through a blend
     corner of the model); tier 1 = the rest outside 16.5 < v < 39; tier 2 = the others (a cold-start
     guess from the model's nonsmooth / stiff regions, for batches without history);
     2 = longest-expected-first by mr_inputs.order_hint (e.g. the previous MPC tick's iters of the same
     vehicles: LPT scheduling with a distribution-agnostic estimate); without a hint, the handle's own
     previous solve of the same batch size (its iters, kept on the device and read in stream order: calls
     on different streams must be ordered by the caller), else instance order; a uniform hint (all equal)
     gives instance order */
  int32_t dispatch_order;
} mr_config;

typedef struct mr_inputs {
  const double* state0;  /* [8][B]: x, y, yaw, v_x, v_y, yaw_dot, throttle, steer (NaN = None) */
  const double* s0;      /* [B] initial progress */
  const double* cx;      /* [5][B] centerline x polynomial, highest order first, global s */
  const double* cy;      /* [5][B] */
  const double* max_error; /* [B] lane half width (used when lane_bounds) */
  const double* runtime; /* [5][B] RuntimeControllerParameters: alpha_c, d_max, q_v_y, n, beta_delta.
                            NOTE control/MPC.py:50 reads the CLASS attribute d_max; the Python
                            drop-in passes that value here to keep the quirk. */
  const double* u_init;  /* optional [2][N][B] initial controls (already shifted last_controls,
                            control/MPC.py:120-125); NULL -> (throttle0, steer0) repeated */
  const int32_t* order_hint; /* optional [B] expected cost of each instance (larger = dispatched earlier),
                            read only with mr_config.dispatch_order = 2, before the solve starts (so the
                            previous call's mr_outputs.iters may be passed in place) */
} mr_inputs;

typedef struct mr_outputs {
  double* X;      /* [6][N+1][B] States (control/MPC.py:166) */
  double* U;      /* [2][N][B] */
  double* S;      /* [N+1][B] S_hat */
  double* eC;     /* [N][B] e_hat_C(S_hat[i], States[:, i]), i = 0..N-1 */
  double* eL;     /* [N][B] e_hat_L */
  int32_t* status; /* [B] MR_STATUS_* */
  int32_t* iters;  /* [B] interior-point iterations */
  double* obj;     /* optional [B] objective value (NULL to skip) */
  double* kkt;     /* optional [B] final scaled KKT error (NULL to skip) */
  double* trace;   /* optional [trace_cap][8] per-iteration record of instance trace_instance:
                      kkt, mu, alpha_primal, alpha_dual, delta (inertia), theta, phi, line-search trials */
  int32_t trace_instance;
  int32_t trace_cap;
  double* lam_g;   /* optional [13N+9][B]: the reference's dual = sol.value(opti.lam_g) (control/MPC.py:171)
                      in Opti row order (MPC.py:101-149): S_0, X_{:,0} (6), per i = 1..N the 6 dynamics rows and
                      the Delta-S row, per i = 0..N-1 thr < d_max, thr > min, steer < max, steer > min, the
                      throttle and steer rate rows (i = 0: against U[:, N-1]), then the state0 throttle and
                      steer rows (NaN when state0 has no throttle / steer).  CasADi convention: Lagrangian
                      f + lam_g . g, canonical row = the non-constant side (positive at an active upper
                      bound); unscaled objective.  NULL to skip. */
  int64_t* timeline; /* optional [2][B] diagnostics: device clock (s_memrealtime, 100 MHz) when instance i's
                        workgroup started and finished; NULL to skip */
  double* constr_viol; /* optional [B]: IPOPT's unscaled constraint violation of the returned point (max-norm
                          of the dynamics / initial-state rows and of the rows' bound violations; the
                          "Constraint violation" IPOPT prints on exit).  Tells a status-3 stop at an
                          almost-feasible point from a restoration failure.  NULL to skip */
} mr_outputs;

typedef struct mr_handle mr_handle;

int mr_version(void);
const char* mr_last_error(void);
int mr_config_default(mr_config* cfg);
int mr_create(mr_handle** h, const mr_config* cfg);
int mr_destroy(mr_handle* h);
/* Pacejka coefficients a[0..8] and vertical load Fz for the front and back tyre
   (state dict keys front_tire.a / front_tire.Fz / back_tire.a / back_tire.Fz).  Synchronises the
   handle's device before it replaces the constants the kernels read (solves in flight on any stream
   finish first). */
int mr_set_tyres(mr_handle* h, const double* a_front, double Fz_front, const double* a_back, double Fz_back);
int mr_solve_batch(mr_handle* h, int32_t B, const mr_inputs* in, mr_outputs* out, void* hip_stream);
/* Diagnostics: the handle's vehicle dynamics (fp64) at n points, device arrays x [n][6], u [n][2],
   nu [n][6] -> f [n][6], J [n][6*8] (d f / d(x, u)), H [n][36] (packed upper triangle of
   sum_i nu_i d2 f_i / d(x, u)^2); J == NULL evaluates the value-only variant into f.
   Replaces CasADi's evaluation of f_vehicle (control/MPC.py:186-229). */
int mr_eval_dynamics(mr_handle* h, int32_t n, const double* x, const double* u, const double* nu, double* f,
                     double* J, double* H, void* hip_stream);
/* workspace bytes used per instance for the handle's configuration */
int64_t mr_workspace_bytes_per_instance(const mr_handle* h);

/* ---- Centerline geometry: the per-tick MPC inputs, batched (csrc/mr_track.h) --------------------
 * Replaces the host geometry the reference agent runs before every solve (agent.py:156-168,
 * 271-274): splines/ParameterizedLine.py (Gx..ddGy :19-41, x_as_coeffs/y_as_coeffs :43-64,
 * projection_local :80-97, unit_tangent/curvature/mean_curvature/unit_principal_normal :107-149)
 * and splines/ParameterizedCenterline.py (lookup_error :61-80, error_sign :82-91).
 * The track is built once on the host, as ParameterizedLine.from_waypoints (:162-178) does: knots
 * t[n_t] and B-spline coefficients cx, cy[n_c] (scipy layout, k = 3), the length L, and the lane
 * table err_left/err_right[n_rows] whose row i is s = 0.5 * i (lanes/<track>_max_error.csv;
 * n_rows = 0 with NULL tables for a lane boundary, see mr_track_lane_table).
 * All query arrays are caller-owned DEVICE pointers of length n (outputs [m][n] component-major);
 * calls are ordered on hip_stream.  One lane per query. */
typedef struct mr_track mr_track;
int mr_track_create(mr_track** tr, int32_t device, const double* t, int32_t n_t, const double* cx,
                    const double* cy, int32_t n_c, double length, const double* err_left,
                    const double* err_right, int32_t n_rows);
int mr_track_destroy(mr_track* tr);
/* out [6][n] = Gx, Gy, dGx, dGy, ddGx, ddGy at s mod L; span [n] = knot interval of G (may be NULL) */
int mr_track_eval(const mr_track* tr, int32_t n, const double* s, double* out, int32_t* span, void* hip_stream);
/* unit_tangent yaw, curvature, unit_principal_normal (nx, ny); mean_curvature over [s, s + mc_lookahead]
   (N = 10) when mean_kappa != NULL; any output may be NULL */
int mr_track_frame(const mr_track* tr, int32_t n, const double* s, double* yaw, double* kappa, double* nx,
                   double* ny, double mc_lookahead, double* mean_kappa, void* hip_stream);
/* error_sign(X, Y, s) -> +1 / -1 */
int mr_track_error_sign(const mr_track* tr, int32_t n, const double* X, const double* Y, const double* s,
                        int32_t* sign, void* hip_stream);
/* x_as_coeffs / y_as_coeffs(s, lookahead, deg = 4): cx, cy [5][n], highest order first, global s */
int mr_track_polyfit(const mr_track* tr, int32_t n, const double* s, const double* lookahead, double* cx,
                     double* cy, void* hip_stream);
/* x_as_coeffs / y_as_coeffs with the reference's deg argument (splines/ParameterizedLine.py:43-64):
   0 <= deg <= 10, cx, cy [deg + 1][n], highest order first, global s (deg 4 = mr_track_polyfit) */
int mr_track_polyfit_deg(const mr_track* tr, int32_t n, const double* s, const double* lookahead, int32_t deg,
                         double* cx, double* cy, void* hip_stream);
/* lookup_error(s, lookahead) -> err [n] (NaN where the reference raises KeyError); row_lo / row_hi /
   row_arg [n]: first / last / arg-min lane-table row (-1 on KeyError; each may be NULL) */
int mr_track_lookup_error(const mr_track* tr, int32_t n, const double* s, const double* lookahead, double* err,
                          int32_t* row_lo, int32_t* row_hi, int32_t* row_arg, void* hip_stream);
/* projection_local(X, Y, bounds = (lo, hi)) -> s [n], dist [n]; nfev [n] may be NULL */
int mr_track_projection(const mr_track* tr, int32_t n, const double* X, const double* Y, const double* lo,
                        const double* hi, double* s, double* dist, int32_t* nfev, void* hip_stream);
/* The agent's tick prep fused (agent.py:156-168 after the projection of :271-274): progress
   s = projection_local(X, Y, (lo, hi)), cx, cy = x/y_as_coeffs(s - lookback, lookahead),
   max_error = lookup_error(s, lookahead) - err_offset (agent.py: car_width / 2).  Outputs s, dist [n],
   cx, cy [5][n], max_error [n]; s0 may then feed mr_solve_batch's inputs directly. */
int mr_track_prep(const mr_track* tr, int32_t n, const double* X, const double* Y, const double* lo,
                  const double* hi, double lookback, double lookahead, double err_offset, double* s,
                  double* dist, double* cx, double* cy, double* max_error, void* hip_stream);

/* Track construction (host arrays, no device work): ParameterizedLine.from_waypoints
 * (splines/ParameterizedLine.py:162-178) -- chord-length progress, not-a-knot cubic interpolation
 * (scipy make_interp_spline, k = 3) -- with ParameterizedCenterline.from_file's closing point
 * (ParameterizedCenterline.py:93-105) when close_loop.  x, y [n]; outputs t [n + 5] (capacity),
 * cx, cy [n + 1] (capacity), *n_t = knots written (coefficients: *n_t - 4), *length = L.  The
 * result feeds mr_track_create. */
int mr_spline_from_waypoints(const double* x, const double* y, int32_t n, int32_t close_loop, double* t, double* cx,
                             double* cy, int32_t* n_t, double* length);

/* ---- lane-width table build -------------------------------------------------
 * Replaces script/make_lane_width_lookup_table.py:12-16 (Pool(14) over
 * ParameterizedCenterline.get_errors(lane, s, 0), ParameterizedCenterline.py:41-58, whose
 * lane.projection with bounds None is projection_global, ParameterizedLine.py:99-105).
 * `lane` is a lane boundary built like a track (mr_track_create with its own spline from
 * lanes/<track>_{left,right}.csv, n_rows = 0, err_* NULL).  For each centerline progress s[i]:
 * dist[i] = min over u in [0, L_lane] of |lane(u) - G(s[i])|, s_lane[i] = that u (may be NULL).
 * Deterministic global search (mr_track.h lane_distance), one wavefront per query. */
int mr_track_lane_table(const mr_track* centerline, const mr_track* lane, int32_t n, const double* s, double* dist,
                        double* s_lane, void* hip_stream);

/* ---- closed loop (agent.py:138-314 with a models/ plant in place of CARLA) ---- */

/* One tick of the agent's sensing and MPC-input preparation, per vehicle:
   progress = projection(X, Y, bounds = progress_bound(prev_progress))   agent.py:80-92, 271-273,
              ParameterizedLine.py:66-105 (NaN prev_progress or bounds wider than 5 m -> global search;
              the reference's unseeded dual_annealing is replaced by the best of the bounded Brent over
              every 5 m window, first minimum wins),
   error    = dist * error_sign(X, Y, progress)                           agent.py:274,
   cx, cy   = x/y_as_coeffs(progress - lookback, lookahead)               agent.py:156-165,
   max_error = lookup_error(progress, lookahead) - err_offset             agent.py:166-168.
   Arrays [n] (cx, cy [5][n]); prev_progress may be NULL (all global). */
int mr_agent_sense(const mr_track* tr, int32_t n, const double* X, const double* Y, const double* prev_progress,
                   double lookback, double lookahead, double err_offset, double* progress, double* error, double* cx,
                   double* cy, double* max_error, void* hip_stream);
/* One plant step per vehicle: state [6][n] = (x, y, yaw, v_x, v_y, yaw_dot), cmd [2][n] = (throttle - brake,
   steer) -> out [6][n] (may alias state).  Model.step(throttle_cmd, steer_cmd, dt) of the models/ package.
   Runs on the device that owns `state` (MR_ERR_ARG if it is not a HIP device pointer). */
int mr_plant_step(int32_t model, int32_t n, const double* state, const double* cmd, double dt, double* out,
                  void* hip_stream);

#ifdef __cplusplus
}
#endif

#endif /* MPCRACING_H */
