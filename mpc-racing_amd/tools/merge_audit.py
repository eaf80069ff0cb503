"""Merge convergence_audit.py shard outputs (same config / n): python merge_audit.py a.json b.json ... > out.json"""
import json
import sys

recs = [json.load(open(p)) for p in sys.argv[1:]]
out = {k: v for k, v in recs[0].items() if k not in ("unsolved", "shard", "cpu_s")}
out["unsolved"] = sorted((e for r in recs for e in r["unsolved"]), key=lambda e: e["i"])
out["shards"] = len(recs)
print(json.dumps(out, indent=1))
