"""Multi-rank path of bench.py on CPU (gloo): ``bench.py --gpus 2`` spawns its two rank processes itself
(WORLD_SIZE unset, the driver's plain invocation), each builds its shard, and the counters go through
the real ``reduce_counters`` (the run's only collective; RCCL "nccl" on the GPU box).  Checks: the
right number of ranks, disjoint shards that span the lap and union to the config's batch, and the
reduced totals."""
import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(*argv):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), *argv, "--cpu-check"], env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("world", [2, 4])
def test_spawned_ranks_shard_the_batch(world):
    per = 256
    out = _run("--gpus", str(world), "--config", "C4", "--per-gpu", str(per))
    assert out["n_gpus"] == world and out["instances"] == per * world
    segs = out["segments"]
    assert len(segs) == world
    flat = [k for s in segs for k in s]
    assert len(flat) == len(set(flat))                        # disjoint
    n_shards = out["n_shards"]
    assert n_shards == 65536 // per and out["K"] == n_shards * (per // 128)
    for r, s in enumerate(segs):
        assert s == list(range(r, out["K"], n_shards))        # every shard spans the lap
    assert out["elapsed_max"] == float(world)                  # max over ranks of 1 + rank
    sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
    from mpcracing import workload as wl
    tot = sum(float(wl.make_batch("C4", rank=r, world=world, per_gpu=per)["state0"][3].sum()) for r in range(world))
    assert abs(out["vx_sum"] - tot) <= 1e-9 * tot


def test_single_rank_is_rank0_of_eight():
    """The 1-GPU bench shard is rank 0's shard of the 8-GPU run (same instances)."""
    sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
    from mpcracing import workload as wl
    a = wl.make_batch("C4", rank=0, world=1, per_gpu=1024)
    b = wl.make_batch("C4", rank=0, world=8, per_gpu=1024)
    for k in ("state0", "s0", "cx", "cy", "max_error"):
        assert np.array_equal(a[k], b[k])
    with pytest.raises(ValueError):
        wl.make_batch("C4", rank=0, world=128, per_gpu=1024)  # more ranks than shards


def test_bench_world2_real_path_with_gloo():
    """bench.py's own world > 1 branch (not --cpu-check): init_process_group (gloo via
    MR_BENCH_BACKEND), per-rank shards of the real path, reduce_counters and the JSON line -- the solves
    skipped (--dry-run, no GPU here).  The line must report 2 GPUs and the union of the two shards."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MR_BENCH_BACKEND"] = "gloo"
    r = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--per-gpu", "8192",
                        "--steps", "2", "--warmup", "0", "--dry-run"], env=env, capture_output=True, text=True,
                       timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads(r.stdout.strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["dry_run"] is True
    assert line["config"]["global_batch"] == 16384 and line["config"]["parallelism"] == "dp2 (instance shards)"
    assert line["status_hist"]["solved"] == 16384 and line["scaling"] == "weak"
