"""Summarise rocprofv3 outputs of a bench run into profiles/ (developer tool).

usage: pmc_summary.py <stats_csv> <fetch_counter_csv> <write_counter_csv> <out_json> [kernel_substr] [B] [config]
                      [sq_counter_csv]

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


SIMDS, CUS = 1024, 256  # MI355X: 256 CUs x 4 SIMDs (MI355X_MICROARCH.md)


def compute_side(path, ksub):
    """The compute side of the kernel's roofline from one SQ + GRBM pass (MI355X_MICROARCH.md §PMC):
    kernel cycles = GRBM_GUI_ACTIVE / 8 (summed over the 8 XCDs); SQ_ACTIVE_INST_* and SQ_WAVE_CYCLES are
    quad-cycles summed over waves, SQ_VALU_MFMA_BUSY_CYCLES cycles summed over SIMDs.  Fractions are of
    the chip's issue capacity over the kernel's duration: VALU busy = active VALU cycles / (cycles x 1024
    SIMDs), MFMA busy likewise, LDS = LDS instructions per CU-cycle (one per cycle per CU peak), and the
    wave-cycle split (parked on a wait / issue-stalled / issuing)."""
    g = {}
    for n in ("GRBM_GUI_ACTIVE", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY",
              "SQ_VALU_MFMA_BUSY_CYCLES", "SQ_INSTS_LDS", "SQ_INSTS_VALU", "SQ_WAIT_ANY", "SQ_WAIT_INST_ANY"):
        v, _ = counter_per_launch(path, n, ksub)
        if v is not None:
            g[n] = v
    out = {"counters_per_launch": g}
    cyc = g.get("GRBM_GUI_ACTIVE", 0.0) / 8.0
    if cyc > 0:
        out["kernel_cycles"] = cyc
        if "SQ_ACTIVE_INST_VALU" in g:
            out["valu_busy_frac"] = 4.0 * g["SQ_ACTIVE_INST_VALU"] / (cyc * SIMDS)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in g:
            out["mfma_busy_frac"] = g["SQ_VALU_MFMA_BUSY_CYCLES"] / (cyc * SIMDS)
        if "SQ_INSTS_LDS" in g:
            out["lds_insts_per_cu_cycle"] = g["SQ_INSTS_LDS"] / (cyc * CUS)
    if g.get("SQ_WAVE_CYCLES"):
        w = g["SQ_WAVE_CYCLES"]
        out["wave_cycles_split"] = {"waiting": g.get("SQ_WAIT_ANY", 0.0) / w,
                                    "issue_stalled": g.get("SQ_WAIT_INST_ANY", 0.0) / w,
                                    "issuing": g.get("SQ_ACTIVE_INST_ANY", 0.0) / w}
    return out


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
    if len(sys.argv) > 8 and os.path.exists(sys.argv[8]):
        res["compute"] = compute_side(sys.argv[8], ksub)
    with open(out, "w") as fo:
        json.dump(res, fo, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
