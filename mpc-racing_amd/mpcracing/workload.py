"""Benchmark configurations and synthetic MPC instance batches.

BASELINE.json ``configs``:
  C1 kinematic, N=20, one instance (script/test_mpc.py:18-39 inputs; Ts 0.1, lookahead 75)
  C2 kinematic, N=20, B=1024, fp64, Shanghai
  C3 dynamic + lane-bound rows, N=40, B=8192, fp64, t1_triple
  C4 blended, N=40, B=65536 over 8 GPUs (8192 per GPU), fp32, Shanghai
  C5 blended + learned Pacejka (pacejka-2), N=60, B=131072 over 8 GPUs (16384 per GPU), fp32, Shanghai

A batch is K track-segment offsets x M randomised states: s0_k = (k + 0.5) L / K;
lateral offset e ~ U(-w/2, w/2) with w = lookup_error(s0, lookahead) - car_width/2
(as script/test_mpc.py:137); heading = tangent yaw + N(0, 0.02); vx ~ U(5, 45);
vy ~ N(0, 1) clipped to +-3; r ~ N(0, 0.5) clipped to +-1.5; throttle0 ~ U(-1, 0.85);
steer0 ~ U(-0.3, 0.3).  Fit window: lookback 5 m, lookahead N*Ts*v_max + 25 m
(ParameterizedLine.x_as_coeffs, deg 4).  Segment k draws from
numpy.random.default_rng([1000 + config#, k]) so any shard of the batch is
reproducible independently of the number of GPUs.

Sharding (SURVEY §8(e), weak scaling): the global batch of a config is fixed --
K segments in lap order x M states (C4: 512 x 128 = 65 536).  It splits into
``n_shards = B / per_gpu`` disjoint shards of per_gpu instances (C4: 8 x 8 192);
shard r holds segments r, r + n_shards, r + 2 n_shards, ... so every shard spans
the whole lap (the same instance mix, hence balanced ranks).  Rank r of a world of
W <= n_shards GPUs solves shard r: the 1-GPU bench line is rank 0's shard of the
8-GPU run, and the 8 shards union to the full batch.
"""
import json
import os

import numpy as np

from .track import Track, CAR_WIDTH

HERE = os.path.dirname(os.path.abspath(__file__))

CONFIGS = {
    "C1": dict(model="kin", N=20, precision="fp64", B=1, per_gpu=1, K=1, M=1, track="shanghai_intl_circuit",
               lane=False, Ts=0.1, seed=1001, tyres=None),
    "C2": dict(model="kin", N=20, precision="fp64", B=1024, per_gpu=1024, K=64, M=16,
               track="shanghai_intl_circuit", lane=False, Ts=0.05, seed=1002, tyres=None),
    "C3": dict(model="dyn", N=40, precision="fp64", B=8192, per_gpu=8192, K=128, M=64, track="t1_triple",
               lane=True, Ts=0.05, seed=1003, tyres=None),
    "C4": dict(model="blend", N=40, precision="fp32", B=65536, per_gpu=8192, K=512, M=128,
               track="shanghai_intl_circuit", lane=False, Ts=0.05, seed=1004, tyres=None),
    "C5": dict(model="blend_pacejka", N=60, precision="fp32", B=131072, per_gpu=16384, K=1024, M=128,
               track="shanghai_intl_circuit", lane=False, Ts=0.05, seed=1005, tyres="pacejka-2"),
}

RUNTIME_DEFAULT = (1000.0, 0.85, 50.0, 2.0, 5000.0)  # RuntimeControllerParameters (alpha_c, d_max, q_v_y, n, beta_delta)
V_MAX = 50.0

_tracks = {}


def track(name):
    if name not in _tracks:
        _tracks[name] = Track(name)
    return _tracks[name]


def tyre_coeffs(name):
    """Learned tyre coefficients exported from learning/models/<name>/model (weights only)."""
    with open(os.path.join(HERE, "..", "data", "tyres.json")) as f:
        t = json.load(f)[name]
    return (t["front_tire.a"], t["front_tire.Fz"][0]), (t["back_tire.a"], t["back_tire.Fz"][0])


def segment_instances(cfg, k, K, M):
    """The M instances of segment k (of K)."""
    tr = track(cfg["track"])
    N, Ts = cfg["N"], cfg["Ts"]
    rng = np.random.default_rng([cfg["seed"], k])
    L = tr.length
    s0 = (k + 0.5) * L / K
    la = N * Ts * V_MAX + 25.0
    cx, cy = tr.xy_coeffs(s0 - 5.0, la)
    w = tr.lookup_error(s0, la) - CAR_WIDTH / 2
    nx, ny = tr.unit_principal_normal(s0)
    yaw0 = float(tr.unit_tangent_yaw(s0))
    gx, gy = float(tr.Gx(s0)), float(tr.Gy(s0))
    e = rng.uniform(-w / 2, w / 2, M)
    st = np.zeros((8, M))
    st[0] = gx + e * nx
    st[1] = gy + e * ny
    st[2] = yaw0 + rng.normal(0.0, 0.02, M)
    st[3] = rng.uniform(5.0, 45.0, M)
    st[4] = np.clip(rng.normal(0.0, 1.0, M), -3.0, 3.0)
    st[5] = np.clip(rng.normal(0.0, 0.5, M), -1.5, 1.5)
    st[6] = rng.uniform(-1.0, 0.85, M)
    st[7] = rng.uniform(-0.3, 0.3, M)
    return dict(state0=st, s0=np.full(M, s0), cx=np.repeat(cx[:, None], M, 1), cy=np.repeat(cy[:, None], M, 1),
                max_error=np.full(M, w))


def config1_instance():
    """C1: script/test_mpc.py:18-39 (s0 = 69.6, Ts = 0.1, lookahead 75), N overridden to 20."""
    tr = track("shanghai_intl_circuit")
    s0 = 69.6
    cx, cy = tr.xy_coeffs(s0 - 5, 75.0)
    max_err = tr.lookup_error(s0, 75.0) - CAR_WIDTH / 2
    st = np.array([171.0, 91.8, -0.219, 20.0, 0.48, -0.059, 0.19, 0.63])[:, None]
    return dict(state0=st, s0=np.array([s0]), cx=cx[:, None], cy=cy[:, None], max_error=np.array([max_err]))


def shard_segments(name, rank=0, world=1, per_gpu=None):
    """(segment indices of ``rank``'s shard, K total segments, n_shards) -- see the module doc."""
    cfg = CONFIGS[name]
    M = cfg["M"]
    per = per_gpu or cfg["per_gpu"]
    if per % M:
        raise ValueError(f"per_gpu ({per}) must be a multiple of M = {M} states per segment")
    n_shards = max(1, cfg["B"] // per)
    if world > n_shards:
        raise ValueError(f"{name}: {world} ranks but only {n_shards} shards of {per} instances "
                         f"(global batch {cfg['B']}); lower per_gpu")
    if not 0 <= rank < world:
        raise ValueError("rank out of range")
    K = n_shards * (per // M)
    return list(range(rank, K, n_shards)), K, n_shards


def make_batch(name, rank=0, world=1, per_gpu=None, limit=None):
    """The shard of config ``name`` owned by ``rank`` (weak scaling: per_gpu instances per rank)."""
    cfg = CONFIGS[name]
    if name == "C1":
        if world != 1:
            raise ValueError("C1 is a single instance")
        parts = [config1_instance()]
    else:
        M = cfg["M"]
        segs, K, _ = shard_segments(name, rank, world, per_gpu)
        if limit is not None:
            segs = segs[:max(1, -(-limit // M))]
        parts = [segment_instances(cfg, k, K, M) for k in segs]
    b = {key: np.concatenate([p[key] for p in parts], axis=-1) for key in parts[0]}
    if limit is not None:
        b = {key: v[..., :limit] for key, v in b.items()}
    B = b["s0"].shape[0]
    b["runtime"] = np.repeat(np.array(RUNTIME_DEFAULT)[:, None], B, 1)
    b["u_init"] = None
    return {k: (np.ascontiguousarray(v, dtype=np.float64) if v is not None else None) for k, v in b.items()}


def instance_dicts(batch):
    """Per-instance (state0 dict, s0, cx, cy, max_error) views of a batch (for the oracle)."""
    out = []
    names = ["x", "y", "yaw", "v_x", "v_y", "yaw_dot", "throttle", "steer"]
    for i in range(batch["s0"].shape[0]):
        st = {n: float(batch["state0"][j, i]) for j, n in enumerate(names)}
        for n in ("throttle", "steer"):
            if st[n] != st[n]:
                st[n] = None
        out.append(dict(state0=st, s0=float(batch["s0"][i]), cx=batch["cx"][:, i].tolist(),
                        cy=batch["cy"][:, i].tolist(), max_error=float(batch["max_error"][i])))
    return out
