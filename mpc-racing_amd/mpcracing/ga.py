"""Batched fitness evaluation of controller-parameter populations.

The reference's GA (GA/mpcGA.py:16-62) scores each individual -- a RuntimeControllerParameters
vector (alpha_c, d_max, q_v_y, n, beta_delta) -- by its time over a track segment
(splines/TrackSegments.py:7-35 splits the lap into ``num_checkpoints`` equal-time segments),
rewards it with ``exp(-kT (segment_time - average_time))`` and updates the segment's running
average ``lambda_T * segment_time + (1 - lambda_T) * average_time`` (mpcGA.py:18-23).  The
reference's loop has a random placeholder where the segment time should come from driving;
here every (individual, segment) pair is one vehicle of a batched closed loop
(mpcracing.ClosedLoop): population x segments vehicles start at their segment's first point,
are MPC-controlled from the first tick, and the segment time is the first tick at which their
progress passes the segment end (linear interpolation inside the tick; ``inf`` if not reached).
"""
import numpy as np
import torch

from .closed_loop import ClosedLoop

KT, KC, LAMBDA_T = 4.0, 0.5, 0.3  # GA/mpcGA.py:11-13


def compute_reward(segment_time, average_time):
    return np.exp(-KT * (segment_time - average_time))   # mpcGA.py:18-20


def compute_avg_time(segment_time, average_time):
    return LAMBDA_T * segment_time + (1 - LAMBDA_T) * average_time   # mpcGA.py:22-23


def segment_times(records, s_start, s_end, length, dt):
    """First crossing time of s_end [B] by the progress records (track wrap handled)."""
    prog = np.stack([r["progress"].cpu().numpy() for r in records])          # [T][B]
    travelled = np.mod(prog - s_start[None, :], length)                      # distance along the lap
    # the first ticks may sit slightly behind the start (projection): treat > L/2 as negative
    travelled = np.where(travelled > 0.5 * length, travelled - length, travelled)
    need = np.mod(s_end - s_start, length)
    B = prog.shape[1]
    out = np.full(B, np.inf)
    for b in range(B):
        hit = np.nonzero(travelled[:, b] >= need[b])[0]
        if len(hit) and hit[0] > 0:
            k = hit[0]
            a, c = travelled[k - 1, b], travelled[k, b]
            out[b] = dt * ((k - 1) + (need[b] - a) / (c - a))
    return out


def evaluate_population(track, population, bounds, ticks, v0=15.0, N=15, precision="fp64", plant="blend",
                        dt=0.05, d_max_class_attribute=True, **solver_kw):
    """Segment times [P][K] of P individuals ([P][5] runtime vectors) on K segments (bounds [K+1]).

    d_max_class_attribute: the reference's NLP ignores the runtime d_max (MPC.py:50 reads the
    class attribute 0.85); True reproduces that."""
    pop = np.asarray(population, dtype=np.float64).reshape(-1, 5)
    P, K = pop.shape[0], len(bounds) - 1
    starts = np.asarray(bounds[:-1], dtype=np.float64)
    ends = np.asarray(bounds[1:], dtype=np.float64)
    rt = np.repeat(pop, K, axis=0).T.copy()             # [5][P*K], vehicle = individual * K + segment
    if d_max_class_attribute:
        rt[1] = 0.85
    s0 = np.tile(starts, P)
    loop = ClosedLoop(track, B=P * K, N=N, plant=plant, precision=precision, dt=dt, start_control_at=1,
                      runtime=rt, **solver_kw)
    x0 = ClosedLoop.start_states(loop.track, s0, v0=v0)
    loop.reset(x0)
    recs = loop.run(ticks)
    torch.cuda.synchronize(loop.dev)
    t = segment_times(recs, s0, np.tile(ends, P), loop.track.length, dt)
    return t.reshape(P, K), recs


def rewards(times, avg_times):
    """Per-individual reward sum and the updated segment averages, in the order of mpcGA.py:40-56
    (individual i on its segment, averages updated as the individuals are scored)."""
    avg = np.array(avg_times, dtype=np.float64)
    P, K = times.shape
    r = np.zeros(P)
    for i in range(P):
        for k in range(K):
            a = avg[k]
            avg[k] = compute_avg_time(times[i, k], a)
            r[i] += compute_reward(times[i, k], a)
    return r, avg


# splines/TrackSegments.py:7-35, the drop-in module (host quadrature, reference formulas)
from splines.TrackSegments import TrackSegments  # noqa: E402,F401
