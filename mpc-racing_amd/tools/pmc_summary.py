"""Summarise rocprofv3 outputs of a bench run into profiles/ (developer tool).

usage: pmc_summary.py <stats_csv> <fetch_counter_csv> <write_counter_csv> <out_json> [kernel_substr] [B] [config]

B / config are recorded so bench.py can match the summary to its own batch (it reports
`traffic` only when B agrees).

HBM traffic per launch of the dominant kernel, corrected as MI355X_MICROARCH.md §HBM prescribes:
FETCH_SIZE (KiB) reports half of the bytes of wide coalesced reads on gfx950 -> x2; WRITE_SIZE
(KiB) as is.  Only the dispatches with the largest grid (the bench batch, not the B = 1
latency probe) are averaged.
"""
import csv
import hashlib
import json
import os
import sys

LIB = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "csrc", "libmpcracing.so")


def rows(path):
    with open(path) as f:
        return list(csv.DictReader(f))


def counter_per_launch(path, name, ksub):
    per = {}
    grid = {}
    for r in rows(path):
        if ksub not in r.get("Kernel_Name", ""):
            continue
        if r.get("Counter_Name") != name:
            continue
        d = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[d] = per.get(d, 0.0) + float(r["Counter_Value"])
        grid[d] = int(float(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0))
    if not per:
        return None, 0
    gmax = max(grid.values())
    vals = [v for d, v in per.items() if grid[d] == gmax]
    return sum(vals) / len(vals), len(vals)


def main():
    stats, fetch, write, out = sys.argv[1:5]
    ksub = sys.argv[5] if len(sys.argv) > 5 else "mr_wave_kernel"
    res = {"kernel": ksub}
    for r in rows(stats):
        if ksub in r["Name"]:
            res["stats"] = {k: r[k] for k in ("Name", "Calls", "AverageNs", "MinNs", "MaxNs", "Percentage")}
    f, nf = counter_per_launch(fetch, "FETCH_SIZE", ksub)
    w, nw = counter_per_launch(write, "WRITE_SIZE", ksub)
    res["fetch_kib_raw_per_launch"] = f
    res["write_kib_per_launch"] = w
    if f is not None and w is not None:
        res["hbm_bytes_per_launch"] = (2.0 * f + w) * 1024.0
    res["dispatches"] = [nf, nw]
    with open(os.environ.get("MR_PRODUCT_LIB") or LIB, "rb") as f:  # bench.py reports traffic only for this build
        res["lib_sha"] = hashlib.sha256(f.read()).hexdigest()[:16]
    if len(sys.argv) > 6:
        res["B"] = int(sys.argv[6])
    if len(sys.argv) > 7:
        res["config"] = sys.argv[7]
        res["command"] = ("rocprofv3 --pmc FETCH_SIZE|WRITE_SIZE (separate passes) -- python bench.py --config "
                          f"{sys.argv[7]} --steps 1 --warmup 0 --no-cpu-baseline --no-latency")
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
