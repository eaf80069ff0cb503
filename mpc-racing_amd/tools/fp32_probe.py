"""fp32 accuracy probe (GPU): fp32 vs fp64 solves on the same instances, and both against the oracle.

Prints one JSON line per config with the distribution of |U32 - U64|, |X32 - X64|, statuses, and the
oracle comparison of a few instances -- the data behind the fp32 tolerances of tests/test_gpu.py
(DESIGN.md §4).  Usage: python mpc-racing_amd/tools/fp32_probe.py [n] [n_oracle]
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, ".."))
sys.path.insert(0, os.path.join(HERE, "..", ".."))


def main():
    from mpcracing import workload as wl
    from mpcracing.batch import BatchSolver
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 256
    n_or = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    for name in ("C4", "C5"):
        cfg = wl.CONFIGS[name]
        tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
        b = wl.make_batch(name, limit=n)
        s64 = BatchSolver(cfg["N"], cfg["model"], "fp64", max_batch=n, tyres=tyres, tol=1e-10, acceptable_iter=0)
        s32 = BatchSolver(cfg["N"], cfg["model"], "fp32", max_batch=n, tyres=tyres)
        # fp64 with the reference's own IPOPT termination (tol 1e-4, acceptable 1e-2 x 15) -- what the
        # fp32 solve uses: separates the termination tolerance from fp32 rounding
        s64r = BatchSolver(cfg["N"], cfg["model"], "fp64", max_batch=n, tyres=tyres, tol=1e-4, acceptable_tol=1e-2,
                           acceptable_iter=15)
        o64 = {k: v.cpu().numpy() for k, v in s64.solve(b).items()}
        o32 = {k: v.cpu().numpy() for k, v in s32.solve(b).items()}
        o64r = {k: v.cpu().numpy() for k, v in s64r.solve(b).items()}
        ok = (o64["status"] == 0) & (o32["status"] <= 1)
        dU = np.abs(o64["U"] - o32["U"])[:, :-1, :][:, :, ok]
        dX = np.abs(o64["X"] - o32["X"])[:, :-1, :][:, :, ok]
        dS = np.abs(o64["S"] - o32["S"])[:, ok]
        per_inst = dU.max(axis=(0, 1))
        rec = {"config": name, "n": n, "ok": int(ok.sum()),
               "st64": np.bincount(o64["status"], minlength=5).tolist(),
               "st32": np.bincount(o32["status"], minlength=5).tolist(),
               "it64": float(o64["iters"].mean()), "it32": float(o32["iters"].mean()),
               "dU_q50_q90_q99_max": [float(np.quantile(dU, q)) for q in (0.5, 0.9, 0.99)] + [float(dU.max())],
               "dU_inst_q50_q90_max": [float(np.quantile(per_inst, q)) for q in (0.5, 0.9)] + [float(per_inst.max())],
               "dU_solved_only_max": float(np.abs(o64["U"] - o32["U"])[:, :-1, :][:, :, ok & (o32["status"] == 0)].max()),
               "dX_q50_q99_max": [float(np.quantile(dX, q)) for q in (0.5, 0.99)] + [float(dX.max())],
               "dS_max": float(dS.max()), "kkt32_q50_max": [float(np.median(o32["kkt"])), float(o32["kkt"].max())]}
        okr = ok & (o64r["status"] <= 1)
        dUr = np.abs(o64["U"] - o64r["U"])[:, :-1, :][:, :, okr].max(axis=(0, 1))
        dU32 = np.abs(o64["U"] - o32["U"])[:, :-1, :][:, :, okr].max(axis=(0, 1))
        loc = lambda o: o["obj"] + 300.0 * b["s0"]  # noqa: E731  objective without the constant -lambda_s*s0
        gap32 = (loc(o32) - loc(o64))[okr] / np.abs(loc(o64)[okr])
        gapr = (loc(o64r) - loc(o64))[okr] / np.abs(loc(o64)[okr])
        rec.update({"st64_reftol": np.bincount(o64r["status"], minlength=5).tolist(),
                    "dU_inst_64reftol_q50_q90_max": [float(np.quantile(dUr, q)) for q in (0.5, 0.9)] + [float(dUr.max())],
                    "dU32_over_dU64reftol_q50_q90_max": [float(np.quantile(dU32 / np.maximum(dUr, 1e-6), q))
                                                         for q in (0.5, 0.9)] + [float((dU32 / np.maximum(dUr, 1e-6)).max())],
                    "objgap32_q50_q99_max": [float(np.quantile(gap32, q)) for q in (0.5, 0.99)] + [float(gap32.max())],
                    "objgap64reftol_q50_q99_max": [float(np.quantile(gapr, q)) for q in (0.5, 0.99)] + [float(gapr.max())],
                    "objgap32_min": float(gap32.min())})
        if n_or:
            sys.path.insert(0, os.path.join(HERE, "..", ".."))
            from oracle.nlp import MPCProblem, solve_ipm
            errs = []
            for i, inst in enumerate(wl.instance_dicts(b)[:n_or]):
                p = MPCProblem(inst["state0"], inst["s0"], inst["cx"], inst["cy"], inst["max_error"], N=cfg["N"],
                               Ts=cfg["Ts"], model=cfg["model"], tyres=tyres)
                r = solve_ipm(p, tol=1e-10)
                X, U, S, eC, eL = p.unpack(r.w)
                e32 = np.abs(U - o32["U"][:, :, i])[:, :-1].max()
                e64 = np.abs(U - o64["U"][:, :, i])[:, :-1].max()
                errs.append([int(o32["status"][i]), float(e32), float(e64)])
            rec["oracle_vs_32_64"] = errs
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
