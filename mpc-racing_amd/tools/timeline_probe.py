"""Timeline probe (GPU): when every instance of one batched solve started and finished.

Writes gpurun_out/timeline_<cfg>_d<order>.npz (start/end in ms from the first start, iterations,
status) and prints a JSON summary: makespan, slot utilisation, per-iteration time of the longest
solves in the batch vs alone, and when the longest solves started.
usage: python mpc-racing_amd/tools/timeline_probe.py [C4] [dispatch_order]
"""
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
from mpcracing import workload as wl  # noqa: E402
from mpcracing.batch import solver_for_config  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "C4"
    order = int(sys.argv[2]) if len(sys.argv) > 2 else 1
    b = wl.make_batch(name)
    B = b["s0"].shape[0]
    s = solver_for_config(name, B, dispatch_order=order)
    d = s.to_device(b)
    o = s.alloc_outputs(B)
    s.launch(d, o)  # warm-up
    torch.cuda.synchronize()
    if order == 2:  # longest-expected-first by the warm-up solve's iterations (the ideal LPT hint)
        d["order_hint"] = o["iters"].clone()
    o["timeline"] = torch.zeros((2, B), dtype=torch.int64, device=s.device)
    s.launch(d, o)
    torch.cuda.synchronize()
    tl = o["timeline"].cpu().numpy().astype(np.float64) / 1e5  # 100 MHz -> ms
    t0 = tl[0].min()
    st, en = tl[0] - t0, tl[1] - t0
    it = o["iters"].cpu().numpy()
    status = o["status"].cpu().numpy()
    dur = en - st
    mk = float(en.max())
    long_ = np.argsort(-it)[:20]
    # solo time of the 5 longest (B = 1 launches)
    solo = []
    for i in long_[:3]:
        s1 = solver_for_config(name, 1)
        sub = {k: (v[..., i:i + 1].copy() if v is not None else None) for k, v in b.items()}
        d1, o1 = s1.to_device(sub), s1.alloc_outputs(1)
        o1["timeline"] = torch.zeros((2, 1), dtype=torch.int64, device=s1.device)
        s1.launch(d1, o1)
        torch.cuda.synchronize()
        t = o1["timeline"].cpu().numpy()[:, 0].astype(np.float64) / 1e5
        solo.append(float(t[1] - t[0]))
    slots = 1024 * (2 if wl.CONFIGS[name]["precision"] == "fp32" else 1)  # 256 CUs x 4 SIMDs x waves/SIMD
    rec = {"config": name, "dispatch_order": order, "B": int(B), "makespan_ms": mk,
           "sum_instance_ms": float(dur.sum()), "slot_utilisation": float(dur.sum() / (slots * mk)),
           "ms_per_iter_batch_median": float(np.median(dur / np.maximum(it, 1))),
           "ms_per_iter_batch_mean": float(dur.sum() / max(int(it.sum()), 1)),
           "iters_total": int(it.sum()),
           "longest": [{"i": int(i), "iters": int(it[i]), "status": int(status[i]), "start_ms": float(st[i]),
                        "dur_ms": float(dur[i])} for i in long_[:8]],
           "longest_solo_ms": solo,
           "last_to_end": [{"i": int(i), "iters": int(it[i]), "status": int(status[i]), "start_ms": float(st[i]),
                            "end_ms": float(en[i])} for i in np.argsort(-en)[:8]],
           "end_of_bulk_ms_p99": float(np.quantile(en, 0.99)), "end_p999": float(np.quantile(en, 0.999))}
    os.makedirs("gpurun_out", exist_ok=True)
    np.savez_compressed(f"gpurun_out/timeline_{name}_d{order}.npz", start=st, end=en, iters=it, status=status)
    print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
