// The reference agent's per-tick sensing and MPC-input preparation (agent.py:80-92, 138-168,
// 271-274), one lane per vehicle, on the centerline tables of mr_track.h.
#pragma once
#include "mr_track.h"

namespace mr {

// ParameterizedLine.projection_global (ParameterizedLine.py:99-105) uses scipy dual_annealing,
// unseeded and therefore not reproducible.  Deterministic restatement (the same one as the drop-in
// splines.ParameterizedCenterline): the bounded Brent over every 5 m window
// [5w, min(5w + 5, L)] of the track, first best distance wins.
MR_HD double global_projection(const TrackView& T, double X, double Y) {
  double best_s = 0.0, best_d = 1e300;
  for (double lo = 0.0; lo < T.L; lo += 5.0) {
    const double hi = lo + 5.0 < T.L ? lo + 5.0 : T.L;
    const double s = brent_projection(T, X, Y, lo, hi, nullptr);
    const double d = track_dist(T, s, X, Y);
    if (d < best_d) { best_d = d; best_s = s; }
  }
  return best_s;
}

// agent.progress_bound (agent.py:80-92) + ParameterizedLine.projection dispatch (:66-78):
// no previous progress (NaN) or bounds wider than 5 m -> global search, else local Brent.
MR_HD double agent_projection(const TrackView& T, double X, double Y, double prev_progress) {
  if (prev_progress != prev_progress) return global_projection(T, X, Y);
  const double lower = py_mod(prev_progress - 2, T.L), upper = py_mod(prev_progress + 2, T.L);
  const double lo = lower < upper ? lower : upper, hi = lower < upper ? upper : lower;
  if (5 < fabs(hi - lo)) return global_projection(T, X, Y);
  return brent_projection(T, X, Y, lo, hi, nullptr);
}

struct AgentSense {
  double progress, error, cx[5], cy[5], max_error;
};

// One tick of agent.run_step's sensing (:271-274) and run_mpc's inputs (:156-168):
// progress, signed centerline error, quartic coefficients over [progress - lookback,
// progress - lookback + lookahead], and lookup_error(progress, lookahead) - err_offset.
MR_HD void agent_sense(const TrackView& T, double X, double Y, double prev_progress, double lookback,
                       double lookahead, double err_offset, AgentSense& o) {
  const double p = agent_projection(T, X, Y, prev_progress);
  o.progress = p;
  o.error = track_dist(T, p, X, Y) * (double)track_error_sign(T, X, Y, p);
  track_polyfit(T, p - lookback, lookahead, o.cx, o.cy);
  o.max_error = lane_lookup(T, p, lookahead, nullptr, nullptr, nullptr) - err_offset;
}

}  // namespace mr
