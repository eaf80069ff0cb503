"""Developer probe: per-phase shader cycles of single instances (trace instance, last
trace row) and B=1 wall latency; writes gpurun_out/phase_probe.json.

Needs a diagnostic build with the cycle counters compiled in (the product build has none):
  python -c "import sys; sys.path.insert(0,'mpc-racing_amd'); from mpcracing import build; \
             build.build_hip(force=True, out='variants/lib_cycles.so', \
             flags=build.DEFAULT_FLAGS + ['-DMR_PHASE_CYCLES=1'])"
  MR_PRODUCT_LIB=variants/lib_cycles.so python mpc-racing_amd/tools/phase_probe.py C4"""
import json
import os
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
from mpcracing import workload as wl  # noqa: E402
from mpcracing.batch import solver_for_config  # noqa: E402

NAMES = ["eval", "riccati", "forward", "trial", "n_trials", "n_soc_tries", "n_fact", "total"]
# the fourth diagnostics row (mr_wave.h MR_PHASE_CYCLES): the line-search phase by call
LS_SPLIT = ["ls_first", "soc_prep_acc", "ls_soc", "soc_commit", "ls_resume", "soft_resto", "n_soc_episodes",
            "n_ls_resume"]


def _solver(name, B):
    """AGENT: the reference agent's call (agent.py:154,171-183; bench.py agent_call): N = 15, dynamic model,
    fp64, Ts 0.05, the reference's IPOPT options, on C2 instances."""
    if name == "AGENT":
        from mpcracing.batch import BatchSolver
        return BatchSolver(15, "dyn", "fp64", False, 0.05, max_batch=B, tol=1e-4, acceptable_tol=1e-2,
                           acceptable_iter=15)
    return solver_for_config(name, B)


def _batch(name):
    return wl.make_batch("C2", limit=100) if name == "AGENT" else wl.make_batch(name)


def one(name, b, i, cap=520):
    sub = {k: (v[..., i:i + 1].copy() if v is not None else None) for k, v in b.items()}
    s = _solver(name, 1)
    out = s.solve(sub, trace_instance=0, trace_cap=cap)
    torch.cuda.synchronize()
    lat = []
    d = s.to_device(sub)
    o = s.alloc_outputs(1)
    for _ in range(3):
        torch.cuda.synchronize()
        t = time.perf_counter()
        s.launch(d, o)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t)
    tr = out["trace"].cpu().numpy()
    it = int(out["iters"][0])
    row = dict(zip(NAMES, tr[-1].tolist()))
    row.update(dict(zip(["fwd_seq", "fwd_par", "socf_chain", "socf_par", "fact_failed_cycles", "n_fact_failed",
                        "soc_backward", "soc_forward"], tr[-2][:8].tolist())))
    row.update(dict(zip(["trial_stage", "trial_reduce", "trial_accept", "ls_setup", "socb_grad", "socb_pre", "socb_chain",
                          "socb_post"], tr[-3][:8].tolist())))
    row.update(dict(zip(LS_SPLIT, tr[-4][:8].tolist())))
    row.update(instance=i, iters=it, status=int(out["status"][0]), wall_ms=1e3 * min(lat),
               cycles_per_iter=row["total"] / max(it, 1))
    return row


def main():
    names = sys.argv[1].split(",") if len(sys.argv) > 1 else ["C4"]
    res = {}
    for name in names:
        b = _batch(name)
        B = b["s0"].shape[0]
        s = _solver(name, B)
        o = {k: v.cpu().numpy() for k, v in s.solve(b).items()}
        it = o["iters"]
        order = np.argsort(it)
        picks = [int(order[len(order) // 2]), int(order[-1]), int(order[-2])]
        if len(sys.argv) > 2:  # explicit instances: python phase_probe.py C4 395,4387
            picks = [int(x) for x in sys.argv[2].split(",")]
        res[name] = [one(name, b, i) for i in picks]
        # the same instances traced inside the full batch launch (memory system and SIMD shared with
        # the other 8 191 solves): which phases the contention slows
        for i in picks:
            o = s.solve(b, trace_instance=i, trace_cap=520)
            tr = o["trace"].cpu().numpy()
            it_i = int(o["iters"][i])
            row = dict(zip(NAMES, tr[-1].tolist()))
            row.update(dict(zip(["fwd_seq", "fwd_par", "socf_chain", "socf_par", "fact_failed_cycles",
                                 "n_fact_failed", "soc_backward", "soc_forward"], tr[-2][:8].tolist())))
            row.update(dict(zip(["trial_stage", "trial_reduce", "trial_accept", "ls_setup", "socb_grad", "socb_pre", "socb_chain",
                          "socb_post"], tr[-3][:8].tolist())))
            row.update(dict(zip(LS_SPLIT, tr[-4][:8].tolist())))
            row.update(instance=i, iters=it_i, status=int(o["status"][i]), in_batch=True,
                       cycles_per_iter=row["total"] / max(it_i, 1))
            res[name].append(row)
        for r in res[name]:
            print(name, json.dumps(r), flush=True)
    os.makedirs(os.path.join(REPO, "gpurun_out"), exist_ok=True)
    with open(os.path.join(REPO, "gpurun_out", "phase_probe.json"), "w") as f:
        json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
