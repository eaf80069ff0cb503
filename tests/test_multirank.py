"""Multi-rank path of bench.py on CPU (gloo, world_size 2): contiguous instance shards per rank
with no data-path collective, and the one counter all-reduce (SUM) / wall-clock max of the run.
The same code runs over RCCL ("nccl") with one process per MI355X on the GPU box."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, per, q):
    sys.path.insert(0, REPO)
    sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from mpcracing import workload as wl
    b = wl.make_batch("C4", rank=rank, world=world, per_gpu=per)
    B = b["s0"].shape[0]
    # stand-in per-rank counters (the GPU solve is not run here): instances, a checksum of the
    # shard, and a status histogram
    counts = torch.tensor([B, float(b["state0"][3].sum()), 0.0, B, 0, 0, 0, 0], dtype=torch.float64)
    tot, tmax = bench.reduce_counters(counts, elapsed=1.0 + rank, world=world)
    q.put((rank, b["s0"].tolist(), tot.tolist(), tmax))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_shards_and_counter_reduce(world):
    per = 256
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, per, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
    from mpcracing import workload as wl
    full = wl.make_batch("C4", rank=0, world=1, per_gpu=per * world)
    # the shards are contiguous and partition the weak-scaled batch exactly
    assert np.array_equal(np.concatenate([np.asarray(r[1]) for r in res]), full["s0"])
    for _, _, tot, tmax in res:
        assert tot[0] == per * world and tot[3] == per * world
        assert abs(tot[1] - full["state0"][3].sum()) < 1e-6 * abs(full["state0"][3].sum())
        assert tmax == float(world)  # max over ranks of 1 + rank
