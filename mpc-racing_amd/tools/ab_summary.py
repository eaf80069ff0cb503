"""Summarise A/B runs of tools/gpu_flags_ab.sh: gpurun_out/ab_<v>.log (bench.py JSON line) and
gpurun_out/abtl_<v>.log (timeline_probe.py JSON line) -> one JSON object per variant."""
import json
import os
import sys


def last_json(p):
    if not os.path.exists(p):
        return None
    lines = [ln for ln in open(p) if ln.startswith("{")]
    return json.loads(lines[-1]) if lines else None


out = {}
d = os.path.dirname(sys.argv[1]) if len(sys.argv) > 1 else "gpurun_out"
for v in sys.argv[2:] if len(sys.argv) > 2 else []:
    b, t = last_json(os.path.join(d, f"ab_{v}.log")), last_json(os.path.join(d, f"abtl_{v}.log"))
    r = {}
    if b:
        r.update(ms_per_step=b["ms_per_step"], solves_per_s=b["value"], iters_mean=b["iters_mean"],
                 status_hist=b["status_hist"], frac=b["roofline"]["frac"])
    if t:
        r.update(makespan_ms=t["makespan_ms"], ms_per_iter_batch_mean=t.get("ms_per_iter_batch_mean"),
                 ms_per_iter_batch_median=t["ms_per_iter_batch_median"], end_of_bulk_ms_p99=t["end_of_bulk_ms_p99"],
                 longest_solo_ms=t["longest_solo_ms"], slot_utilisation=t["slot_utilisation"],
                 last_to_end=t["last_to_end"][:3])
    out[v] = r
print(json.dumps(out, indent=1))
