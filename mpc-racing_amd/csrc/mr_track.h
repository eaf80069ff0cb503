// Centerline geometry on the device: the per-tick MPC inputs of the reference agent
// (agent.py:156-168, 271-274) for a batch of queries, one lane per query.
//
//   K5  cubic B-spline evaluation G, G', G''   splines/ParameterizedLine.py:19-41 (scipy BSpline:
//                                               interval search + de Boor; derivative splines by splder)
//   K6  x_as_coeffs / y_as_coeffs (deg 4)      splines/ParameterizedLine.py:43-64 (np.polyfit)
//   K7  lookup_error (lane-table window min)   splines/ParameterizedCenterline.py:61-80
//   K8  projection_local (bounded Brent)       splines/ParameterizedLine.py:80-97 (scipy
//                                               _minimize_scalar_bounded, xatol 1e-5, maxiter 500)
//   A15 tangent yaw, curvature, mean curvature, principal normal, error sign
//                                               ParameterizedLine.py:107-149, ParameterizedCenterline.py:82-91
//
// Operations follow the order the reference's libraries execute them (IEEE fp64, built without
// FP contraction), so knot-span indices, lane-table rows, spline values and the Brent step
// sequence reproduce the reference bit for bit.  The quartic fit solves the same least-squares
// problem in a centred, scaled variable (numpy's LAPACK SVD is not reproducible bit for bit);
// its parity is stated on the fitted values.
#pragma once
#include "mr_common.h"
#include <vector>

namespace mr {

// One scipy-layout B-spline (t, c, k), extrapolate=True.
struct SplineView {
  const double* t;
  const double* c;
  int nt, k;
};

// Centerline tables of one track (built once on the host, see track_tables()).
struct TrackView {
  SplineView x[3], y[3];  // G, G', G'' (k = 3, 2, 1)
  double L;               // track length: queries are taken modulo L (ParameterizedLine.py:19-25)
  const double* err_left;  // lane table, row i at s = 0.5 * i (lanes/<track>_max_error.csv)
  const double* err_right;
  int n_rows;
};

// CPython float_rem (the result takes the sign of the divisor)
MR_HD double py_mod(double x, double y) {
  double m = fmod(x, y);
  if (m != 0.0) {
    if ((y < 0) != (m < 0)) m += y;
  } else {
    m = copysign(0.0, y);
  }
  return m;
}

// Python round(x) on floats: half to even (rint in the default rounding mode)
MR_HD double py_round(double x) { return rint(x); }

// scipy _find_interval: largest l in [k, n-1] with t[l] <= x (k when none or NaN)
MR_HD int spline_span(const SplineView& s, double x) {
  const int k = s.k, n = s.nt - k - 1;
  int lo = k, hi = n - 1;  // predicate x >= t[l] is monotone in l
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (x >= s.t[mid]) lo = mid;
    else hi = mid - 1;
  }
  return lo;
}

// de Boor basis (scipy _deBoor_D, m = 0) and the coefficient sum, in scipy's order
MR_HD double spline_eval_in(const SplineView& s, double x, int ell);
MR_HD double spline_eval(const SplineView& s, double x, int* span_out = nullptr) {
  const int ell = spline_span(s, x);
  if (span_out) *span_out = ell;
  return spline_eval_in(s, x, ell);
}

// the same sum with the knot interval ell given (t[ell] <= x < t[ell + 1])
MR_HD double spline_eval_in(const SplineView& s, double x, int ell) {
  const int k = s.k;
  double h[4] = {1.0, 0.0, 0.0, 0.0}, hh[4] = {0.0, 0.0, 0.0, 0.0};
  for (int j = 1; j <= k; ++j) {
    for (int q = 0; q < j; ++q) hh[q] = h[q];
    h[0] = 0.0;
    for (int n = 1; n <= j; ++n) {
      const int ind = ell + n;
      const double xb = s.t[ind], xa = s.t[ind - j];
      if (xb == xa) {
        h[n] = 0.0;
        continue;
      }
      const double w = hh[n - 1] / (xb - xa);
      h[n - 1] += w * (xb - x);
      h[n] = w * (x - xa);
    }
  }
  double acc = 0.0;
  for (int a = 0; a <= k; ++a) acc += s.c[ell + a - k] * h[a];
  return acc;
}

// Gx, Gy, dGx, dGy, ddGx, ddGy at s mod L; span = knot interval of G
MR_HD void track_eval(const TrackView& T, double s, double* out6, int* span) {
  const double m = py_mod(s, T.L);
  out6[0] = spline_eval(T.x[0], m, span);
  out6[1] = spline_eval(T.y[0], m);
  out6[2] = spline_eval(T.x[1], m);
  out6[3] = spline_eval(T.y[1], m);
  out6[4] = spline_eval(T.x[2], m);
  out6[5] = spline_eval(T.y[2], m);
}

// dist(s) = sqrt((Gx(s) - X)**2 + (Gy(s) - Y)**2)  (ParameterizedLine.py:95)
MR_HD double track_dist(const TrackView& T, double s, double X, double Y) {
  const double m = py_mod(s, T.L);
  const double dx = spline_eval(T.x[0], m) - X, dy = spline_eval(T.y[0], m) - Y;
  return sqrt(dx * dx + dy * dy);
}

// scipy.optimize._minimize_scalar_bounded, step for step; returns the minimiser
MR_HD double brent_projection(const TrackView& T, double X, double Y, double x1, double x2, int* nfev) {
  const double xatol = 1e-5;
  const int maxiter = 500;
  const double sqrt_eps = 1.4832396974191326e-08;  // math.sqrt(2.2e-16)
  const double golden_mean = 0.3819660112501051;   // 0.5 * (3.0 - math.sqrt(5.0))
  double a = x1, b = x2;
  double fulc = a + golden_mean * (b - a);
  double nfc = fulc, xf = fulc;
  double rat = 0.0, e = 0.0;
  double fx = track_dist(T, xf, X, Y);
  int num = 1;
  double ffulc = fx, fnfc = fx;
  double xm = 0.5 * (a + b);
  double tol1 = sqrt_eps * fabs(xf) + xatol / 3.0;
  double tol2 = 2.0 * tol1;
  while (fabs(xf - xm) > (tol2 - 0.5 * (b - a))) {
    bool golden = true;
    if (fabs(e) > tol1) {
      golden = false;
      double r = (xf - nfc) * (fx - ffulc);
      double q = (xf - fulc) * (fx - fnfc);
      double p = (xf - fulc) * q - (xf - nfc) * r;
      q = 2.0 * (q - r);
      if (q > 0.0) p = -p;
      q = fabs(q);
      r = e;
      e = rat;
      if (fabs(p) < fabs(0.5 * q * r) && p > q * (a - xf) && p < q * (b - xf)) {
        rat = (p + 0.0) / q;
        const double x = xf + rat;
        if ((x - a) < tol2 || (b - x) < tol2) {
          const double d = xm - xf;
          const double si = (d > 0 ? 1.0 : (d < 0 ? -1.0 : 0.0)) + (xm == xf ? 1.0 : 0.0);
          rat = tol1 * si;
        }
      } else {
        golden = true;
      }
    }
    if (golden) {
      e = (xf >= xm) ? (a - xf) : (b - xf);
      rat = golden_mean * e;
    }
    const double si = (rat > 0 ? 1.0 : (rat < 0 ? -1.0 : 0.0)) + (rat == 0 ? 1.0 : 0.0);
    const double x = xf + si * (fabs(rat) > tol1 ? fabs(rat) : tol1);
    const double fu = track_dist(T, x, X, Y);
    num += 1;
    if (fu <= fx) {
      if (x >= xf) a = xf;
      else b = xf;
      fulc = nfc; ffulc = fnfc;
      nfc = xf; fnfc = fx;
      xf = x; fx = fu;
    } else {
      if (x < xf) a = x;
      else b = x;
      if (fu <= fnfc || nfc == xf) {
        fulc = nfc; ffulc = fnfc;
        nfc = x; fnfc = fu;
      } else if (fu <= ffulc || fulc == xf || fulc == nfc) {
        fulc = x; ffulc = fu;
      }
    }
    xm = 0.5 * (a + b);
    tol1 = sqrt_eps * fabs(xf) + xatol / 3.0;
    tol2 = 2.0 * tol1;
    if (num >= maxiter) break;
  }
  if (nfev) *nfev = num;
  return xf;
}

// ---- Lane-width table build ----
// script/make_lane_width_lookup_table.py:12-16 computes, for every centerline sample
// s = 0.5 i, ParameterizedCenterline.get_errors(lane, s, 0) (ParameterizedCenterline.py:41-58):
// the distance from G(s) to the lane spline, through lane.projection with bounds None, i.e.
// projection_global (ParameterizedLine.py:99-105, scipy dual_annealing over [0, L_lane],
// unseeded).  Deterministic restatement of that global minimum: the lane spline is sampled at
// the start and the midpoint of every knot interval and at L_lane (sample m: interval
// k + m / 2, fraction (m & 1) / 2); the nearest sample m* (smallest m on ties) brackets the
// minimiser in [u_(m*-1), u_(m*+1)] and the bounded Brent (scipy's, as projection_local)
// refines it there.  The lanes' waypoints are ~0.25 m apart, so the bracket holds the global
// minimiser; the result matches the reference's committed tables to 1e-4 m (tests).
MR_HD int lane_n_samples(const TrackView& lane) { return 2 * (lane.x[0].nt - 2 * lane.x[0].k - 1) + 1; }

MR_HD double lane_sample_u(const TrackView& lane, int m, int* ell) {
  const SplineView& S = lane.x[0];
  const int nspan = S.nt - 2 * S.k - 1;
  if (m >= 2 * nspan) { *ell = S.k + nspan - 1; return S.t[S.k + nspan]; }
  const int l = S.k + (m >> 1);
  *ell = l;
  return (m & 1) ? S.t[l] + 0.5 * (S.t[l + 1] - S.t[l]) : S.t[l];
}

MR_HD double lane_sample_d2(const TrackView& lane, int m, double X, double Y) {
  int ell;
  const double u = lane_sample_u(lane, m, &ell);
  const double dx = spline_eval_in(lane.x[0], u, ell) - X, dy = spline_eval_in(lane.y[0], u, ell) - Y;
  return dx * dx + dy * dy;
}

// Brent refinement in the bracket of sample mbest; returns the distance, *s_lane = minimiser
MR_HD double lane_refine(const TrackView& lane, double X, double Y, int mbest, double* s_lane) {
  const int M = lane_n_samples(lane);
  int e;
  const double lo = lane_sample_u(lane, mbest > 0 ? mbest - 1 : 0, &e);
  const double hi = lane_sample_u(lane, mbest + 1 < M ? mbest + 1 : M - 1, &e);
  const double u = brent_projection(lane, X, Y, lo, hi, nullptr);
  if (s_lane) *s_lane = u;
  return track_dist(lane, u, X, Y);
}

// centerline point G(s mod L) (ParameterizedCenterline.get_errors: self.Gx(s), self.Gy(s))
MR_HD void centerline_point(const TrackView& C, double s, double* X, double* Y) {
  const double m = py_mod(s, C.L);
  *X = spline_eval(C.x[0], m);
  *Y = spline_eval(C.y[0], m);
}

// serial form (host build, one lane per query): the same samples, scan order and ties
MR_HD double lane_distance(const TrackView& C, const TrackView& lane, double s, double* s_lane) {
  double X, Y;
  centerline_point(C, s, &X, &Y);
  const int M = lane_n_samples(lane);
  double best = 1e300;
  int mb = 0;
  for (int m = 0; m < M; ++m) {
    const double d2 = lane_sample_d2(lane, m, X, Y);
    if (d2 < best) { best = d2; mb = m; }
  }
  return lane_refine(lane, X, Y, mb, s_lane);
}

// lookup_error: min over the 0.5 m rows of [s, s + lookahead) of min(left, right); rows keyed
// by round-half-even(2 (q mod L)) / 2.  NaN when a key is outside the table (the reference's
// KeyError); row_lo / row_hi / row_arg = first, last, arg-min row (-1 then).
MR_HD double lane_lookup(const TrackView& T, double s, double lookahead, int* row_lo, int* row_hi, int* row_arg) {
  const double s_round = py_round(s * 2) / 2;
  const double la = py_round(lookahead * 2) / 2;
  const double stop = s + la;
  const double span = ceil((stop - s_round) / 0.5);  // numpy.arange length
  const int n = span > 0 ? (int)span : 0;
  double left_min = 10000, right_min = 10000;
  int arg_left = -1, arg_right = -1, lo = -1, hi = -1;
  for (int i = 0; i < n; ++i) {
    const double q = s_round + i * 0.5;
    const double key = py_round(py_mod(q, T.L) * 2) / 2;
    const int row = (int)(key * 2);
    if (row < 0 || row >= T.n_rows) {
      if (row_lo) *row_lo = -1;
      if (row_hi) *row_hi = -1;
      if (row_arg) *row_arg = -1;
      return NAN;
    }
    if (i == 0) lo = row;
    hi = row;
    const double left = T.err_left[row], right = T.err_right[row];
    if (left < left_min) { left_min = left; arg_left = row; }
    if (right < right_min) { right_min = right; arg_right = row; }
  }
  if (row_lo) *row_lo = lo;
  if (row_hi) *row_hi = hi;
  const bool take_left = left_min < right_min;  // Python min(right_min, left_min)
  if (row_arg) *row_arg = take_left ? arg_left : arg_right;
  return take_left ? left_min : right_min;
}

// unit_tangent yaw, curvature |x'y'' - y'x''|, unit principal normal (t_y, -t_x)
MR_HD void track_frame(const TrackView& T, double s, double* yaw, double* kappa, double* nx, double* ny) {
  double g[6];
  track_eval(T, s, g, nullptr);
  const double nrm = sqrt(g[2] * g[2] + g[3] * g[3]);
  const double ux = g[2] / nrm, uy = g[3] / nrm;
  *yaw = atan2(uy, ux);
  *kappa = fabs(g[2] * g[5] - g[3] * g[4]);
  *nx = uy;
  *ny = -ux;
}

// mean_curvature(s, lookahead, N=10): (1/N) * sum of curvature on linspace(s, s + lookahead, N)
MR_HD double track_mean_curvature(const TrackView& T, double s, double lookahead) {
  const int NS = 10;
  const double stop = s + lookahead;
  const double step = (stop - s) / (NS - 1);
  double sum = 0.0;
  for (int i = 0; i < NS; ++i) {
    const double q = i == NS - 1 ? stop : i * step + s;
    double g[6];
    track_eval(T, q, g, nullptr);
    sum += fabs(g[2] * g[5] - g[3] * g[4]);
  }
  return (1.0 / NS) * sum;
}

// error_sign: +1 if |d - n| < |d + n| else -1, d = (X - Gx, Y - Gy), n the principal normal
MR_HD int track_error_sign(const TrackView& T, double X, double Y, double s) {
  double g[6], yaw, kappa, nx, ny;
  track_eval(T, s, g, nullptr);
  track_frame(T, s, &yaw, &kappa, &nx, &ny);
  const double dx = X - g[0], dy = Y - g[1];
  const double a = sqrt((dx - nx) * (dx - nx) + (dy - ny) * (dy - ny));
  const double b = sqrt((dx + nx) * (dx + nx) + (dy + ny) * (dy + ny));
  return a < b ? 1 : -1;
}

// x_as_coeffs / y_as_coeffs(s, lookahead, deg) (ParameterizedLine.py:43-64): least-squares polynomial of
// degree D through the 50 samples of G on numpy.linspace(0, lookahead, 50) + s, in GLOBAL s, highest
// order first (np.polyfit).  Normal equations in u = (s' - mid) / h (moments of a well-conditioned
// basis), Cholesky, then the exact binomial expansion back to powers of s'.  D = 4 is the agent's fit
// (agent.py:140); the others serve the drop-in's deg argument (D <= MR_POLY_DEG_MAX).
constexpr int MR_POLY_DEG_MAX = 10;
template <int D>
MR_HD void track_polyfit_t(const TrackView& T, double s, double lookahead, double* cx, double* cy) {
  constexpr int K = D + 1;
  const int M = 50;
  const double h = lookahead > 0 ? 0.5 * lookahead : 1.0;
  const double mid = s + 0.5 * lookahead;
  const double step = lookahead / (M - 1);
  double mom[2 * D + 1], rx[K], ry[K];
  for (int j = 0; j <= 2 * D; ++j) mom[j] = 0.0;
  for (int j = 0; j < K; ++j) { rx[j] = 0.0; ry[j] = 0.0; }
  for (int i = 0; i < M; ++i) {
    const double q = (i == M - 1 ? lookahead : i * step) + s;
    const double m = py_mod(q, T.L);
    const double yx = spline_eval(T.x[0], m), yy = spline_eval(T.y[0], m);
    const double u = (q - mid) / h;
    double p = 1.0;
    for (int j = 0; j <= 2 * D; ++j) {
      mom[j] += p;
      if (j < K) { rx[j] += p * yx; ry[j] += p * yy; }
      p *= u;
    }
  }
  double L[K][K];
  for (int i = 0; i < K; ++i)
    for (int j = 0; j < K; ++j) L[i][j] = 0.0;
  for (int j = 0; j < K; ++j) {
    double d = mom[2 * j];
    for (int q = 0; q < j; ++q) d -= L[j][q] * L[j][q];
    L[j][j] = sqrt(d);
    for (int i = j + 1; i < K; ++i) {
      double v = mom[i + j];
      for (int q = 0; q < j; ++q) v -= L[i][q] * L[j][q];
      L[i][j] = v / L[j][j];
    }
  }
  double ax[K], ay[K];
  for (int i = 0; i < K; ++i) {  // L y = r
    double vx = rx[i], vy = ry[i];
    for (int q = 0; q < i; ++q) { vx -= L[i][q] * ax[q]; vy -= L[i][q] * ay[q]; }
    ax[i] = vx / L[i][i];
    ay[i] = vy / L[i][i];
  }
  for (int i = K - 1; i >= 0; --i) {  // L^T a = y
    double vx = ax[i], vy = ay[i];
    for (int q = i + 1; q < K; ++q) { vx -= L[q][i] * ax[q]; vy -= L[q][i] * ay[q]; }
    ax[i] = vx / L[i][i];
    ay[i] = vy / L[i][i];
  }
  // sum_j a_j ((s' - mid) / h)^j  ->  ascending powers of s'
  double gx[K], gy[K];
  for (int j = 0; j < K; ++j) { gx[j] = 0.0; gy[j] = 0.0; }
  double hj = 1.0;
  for (int j = 0; j < K; ++j) {
    const double sx = ax[j] / hj, sy = ay[j] / hj;
    double bin = 1.0;  // C(j, i), from i = j down
    double pm = 1.0;   // (-mid)^(j - i)
    for (int i = j; i >= 0; --i) {
      gx[i] += sx * bin * pm;
      gy[i] += sy * bin * pm;
      bin = bin * (double)i / (double)(j - i + 1);
      pm *= -mid;
    }
    hj *= h;
  }
  for (int j = 0; j < K; ++j) {
    cx[j] = gx[D - j];
    cy[j] = gy[D - j];
  }
}
MR_HD void track_polyfit(const TrackView& T, double s, double lookahead, double* cx, double* cy) {
  track_polyfit_t<4>(T, s, lookahead, cx, cy);
}
// any degree 0..MR_POLY_DEG_MAX (false otherwise); cx, cy hold deg + 1 coefficients
MR_HD bool track_polyfit_deg(const TrackView& T, double s, double lookahead, int deg, double* cx, double* cy) {
  switch (deg) {
    case 0: track_polyfit_t<0>(T, s, lookahead, cx, cy); return true;
    case 1: track_polyfit_t<1>(T, s, lookahead, cx, cy); return true;
    case 2: track_polyfit_t<2>(T, s, lookahead, cx, cy); return true;
    case 3: track_polyfit_t<3>(T, s, lookahead, cx, cy); return true;
    case 4: track_polyfit_t<4>(T, s, lookahead, cx, cy); return true;
    case 5: track_polyfit_t<5>(T, s, lookahead, cx, cy); return true;
    case 6: track_polyfit_t<6>(T, s, lookahead, cx, cy); return true;
    case 7: track_polyfit_t<7>(T, s, lookahead, cx, cy); return true;
    case 8: track_polyfit_t<8>(T, s, lookahead, cx, cy); return true;
    case 9: track_polyfit_t<9>(T, s, lookahead, cx, cy); return true;
    case 10: track_polyfit_t<10>(T, s, lookahead, cx, cy); return true;
  }
  return false;
}

// Host: the device tables of one track from the scipy spline (t, c, k = 3): G's coefficients
// padded to len(t), then splder's rule twice, exactly as scipy BSpline.derivative() computes it
// (the reference rebuilds the derivative spline on every call, ParameterizedLine.py:27-41).
// Blob layout: t | cx | cy | t1 | dcx | dcy | t2 | ddcx | ddcy | err_left | err_right.
struct TrackLayout {
  int nt, off_t, off_cx, off_cy, off_t1, off_dcx, off_dcy, off_t2, off_ddcx, off_ddcy, off_el, off_er, total;
};
inline TrackLayout track_layout(int nt, int n_rows) {
  TrackLayout L;
  L.nt = nt;
  int o = 0;
  L.off_t = o; o += nt;
  L.off_cx = o; o += nt;
  L.off_cy = o; o += nt;
  L.off_t1 = o; o += nt - 2;
  L.off_dcx = o; o += nt - 2;
  L.off_dcy = o; o += nt - 2;
  L.off_t2 = o; o += nt - 4;
  L.off_ddcx = o; o += nt - 4;
  L.off_ddcy = o; o += nt - 4;
  L.off_el = o; o += n_rows;
  L.off_er = o; o += n_rows;
  L.total = o;
  return L;
}
// splder on (t, c[len(t)], k): returns c' of length len(t) - 2 (knots t[1:-1], degree k - 1)
inline void splder_coeffs(const double* t, const double* c, int nt, int k, double* out) {
  const int m = nt - k - 2;  // len(dt)
  for (int i = 0; i < m; ++i) {
    const double dt = t[i + k + 1] - t[i + 1];
    out[i] = ((c[i + 1] - c[i]) * (double)k) / dt;
  }
  for (int i = m; i < nt - 2; ++i) out[i] = 0.0;
}
// ---- Track construction, host side of the library ----
// ParameterizedLine.from_waypoints (ParameterizedLine.py:162-178): chord-length progress
// accumulated with the reference's euclidean (splines/util.py:3-4), then scipy
// make_interp_spline(s, x) (k = 3, not-a-knot: knots [s0]*4 + s[2:-2] + [sL]*4).  The
// ParameterizedCenterline.from_file closing point (ParameterizedCenterline.py:93-105:
// midpoint(last, first, alpha = 0.9) when they are more than 0.1 m apart) when close_loop.
// The collocation system is a B-spline collocation matrix (totally positive), solved by
// banded Gaussian elimination without pivoting; scipy's gbsv pivots, so coefficients agree
// to rounding (~1e-12 relative), knots and the arc length bit for bit.
// Returns the number of points used (n or n + 1); t gets np + 4 knots, cx / cy np coefficients.
// Python's float ** 2 is libm pow(x, 2.0), which is not always x * x; called through a volatile
// pointer so the compiler cannot rewrite it into a multiply (splines/util.py:3-4 bit for bit).
inline double py_square(double x) {
  static double (*volatile libm_pow)(double, double) = ::pow;
  return libm_pow(x, 2.0);
}

inline int spline_from_waypoints(const double* x, const double* y, int n, int close_loop, double* t, double* cx,
                                 double* cy, double* length) {
  const int k = 3;
  if (n < 4) return -1;
  std::vector<double> px(x, x + n), py(y, y + n);
  if (close_loop) {
    const double gx = px[n - 1] - px[0], gy = py[n - 1] - py[0];
    if (sqrt(py_square(gx) + py_square(gy)) > 0.1) {
      const double dx = (px[0] - px[n - 1]) * 0.9, dy = (py[0] - py[n - 1]) * 0.9;
      px.push_back(dx + px[n - 1]);
      py.push_back(dy + py[n - 1]);
    }
  }
  const int np = (int)px.size();
  std::vector<double> s(np);
  double cum = 0.0;
  s[0] = 0.0;
  for (int i = 0; i + 1 < np; ++i) {
    const double ax = px[i] - px[i + 1], ay = py[i] - py[i + 1];
    cum += sqrt(py_square(ax) + py_square(ay));
    s[i + 1] = cum;
  }
  *length = cum;
  const int nt = np + 4;
  for (int i = 0; i <= k; ++i) { t[i] = s[0]; t[nt - 1 - i] = s[np - 1]; }
  for (int i = 2; i < np - 2; ++i) t[i + 2] = s[i];
  // collocation rows: B_j(s_i), j = l - 3 .. l; band storage A[i][j - i + KL], KL = KU = 3
  const int KL = 3, W = 7;
  std::vector<double> A((size_t)np * W, 0.0), bx(px), by(py);
  SplineView sv{t, nullptr, nt, k};
  for (int i = 0; i < np; ++i) {
    const int l = spline_span(sv, s[i]);
    double h[4] = {1.0, 0.0, 0.0, 0.0}, hh[4] = {0.0, 0.0, 0.0, 0.0};
    for (int j = 1; j <= k; ++j) {  // de Boor basis, as spline_eval_in
      for (int q = 0; q < j; ++q) hh[q] = h[q];
      h[0] = 0.0;
      for (int m = 1; m <= j; ++m) {
        const double xb = t[l + m], xa = t[l + m - j];
        if (xb == xa) { h[m] = 0.0; continue; }
        const double w = hh[m - 1] / (xb - xa);
        h[m - 1] += w * (xb - s[i]);
        h[m] = w * (s[i] - xa);
      }
    }
    for (int a = 0; a <= k; ++a) {
      const int col = l - k + a, off = col - i + KL;
      if (off < 0 || off >= W) return -2;  // outside the band (cannot happen for distinct s)
      A[(size_t)i * W + off] = h[a];
    }
  }
  for (int j = 0; j < np; ++j) {  // banded LU, no pivoting
    const double piv = A[(size_t)j * W + KL];
    if (piv == 0.0) return -3;
    for (int i = j + 1; i <= j + KL && i < np; ++i) {
      const double f = A[(size_t)i * W + (j - i + KL)] / piv;
      if (f == 0.0) continue;
      for (int c = j; c <= j + KL && c < np; ++c) A[(size_t)i * W + (c - i + KL)] -= f * A[(size_t)j * W + (c - j + KL)];
      bx[i] -= f * bx[j];
      by[i] -= f * by[j];
    }
  }
  for (int j = np - 1; j >= 0; --j) {
    double vx = bx[j], vy = by[j];
    for (int c = j + 1; c <= j + KL && c < np; ++c) {
      vx -= A[(size_t)j * W + (c - j + KL)] * cx[c];
      vy -= A[(size_t)j * W + (c - j + KL)] * cy[c];
    }
    cx[j] = vx / A[(size_t)j * W + KL];
    cy[j] = vy / A[(size_t)j * W + KL];
  }
  return np;
}

inline void track_tables(const double* t, int nt, const double* cx, const double* cy, int nc, const double* el,
                         const double* er, int n_rows, double* blob) {
  const TrackLayout L = track_layout(nt, n_rows);
  for (int i = 0; i < nt; ++i) {
    blob[L.off_t + i] = t[i];
    blob[L.off_cx + i] = i < nc ? cx[i] : 0.0;
    blob[L.off_cy + i] = i < nc ? cy[i] : 0.0;
  }
  for (int i = 0; i < nt - 2; ++i) blob[L.off_t1 + i] = t[i + 1];
  splder_coeffs(blob + L.off_t, blob + L.off_cx, nt, 3, blob + L.off_dcx);
  splder_coeffs(blob + L.off_t, blob + L.off_cy, nt, 3, blob + L.off_dcy);
  for (int i = 0; i < nt - 4; ++i) blob[L.off_t2 + i] = t[i + 2];
  splder_coeffs(blob + L.off_t1, blob + L.off_dcx, nt - 2, 2, blob + L.off_ddcx);
  splder_coeffs(blob + L.off_t1, blob + L.off_dcy, nt - 2, 2, blob + L.off_ddcy);
  for (int i = 0; i < n_rows; ++i) {
    blob[L.off_el + i] = el[i];
    blob[L.off_er + i] = er[i];
  }
}
inline TrackView track_view(const double* blob, int nt, double length, int n_rows) {
  const TrackLayout L = track_layout(nt, n_rows);
  TrackView T;
  T.x[0] = {blob + L.off_t, blob + L.off_cx, nt, 3};
  T.y[0] = {blob + L.off_t, blob + L.off_cy, nt, 3};
  T.x[1] = {blob + L.off_t1, blob + L.off_dcx, nt - 2, 2};
  T.y[1] = {blob + L.off_t1, blob + L.off_dcy, nt - 2, 2};
  T.x[2] = {blob + L.off_t2, blob + L.off_ddcx, nt - 4, 1};
  T.y[2] = {blob + L.off_t2, blob + L.off_ddcy, nt - 4, 1};
  T.L = length;
  T.err_left = blob + L.off_el;
  T.err_right = blob + L.off_er;
  T.n_rows = n_rows;
  return T;
}

}  // namespace mr
