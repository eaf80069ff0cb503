"""Developer probe: does the C5 accuracy test's solve (tests/test_gpu.py test_fp32_accuracy_vs_reference_tolerance)
depend on what ran before it in the process?  The test's three solves (fp64 tol 1e-10, fp32, fp64 at the
reference's options, 512 instances) run before and after the GPU tests that precede it in the suite (in-process,
pytest.main); every output is compared bitwise and the test's objective-gap quantiles printed for both.

Usage: python mpc-racing_amd/tools/suite_order_probe.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(HERE, ".."))


def triple(name="C5", n=512):
    from mpcracing import workload as wl
    from mpcracing.batch import BatchSolver
    cfg = wl.CONFIGS[name]
    tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
    b = wl.make_batch(name, limit=n)
    mk = lambda prec, **kw: BatchSolver(cfg["N"], cfg["model"], prec, max_batch=n, tyres=tyres, **kw)  # noqa: E731
    np_ = lambda o: {k: v.cpu().numpy() for k, v in o.items()}  # noqa: E731
    return b, {"o64": np_(mk("fp64", tol=1e-10, acceptable_iter=0).solve(b)), "o32": np_(mk("fp32").solve(b)),
               "oref": np_(mk("fp64", tol=1e-4, acceptable_tol=1e-2, acceptable_iter=15).solve(b))}


def gaps(b, r):
    o64, o32, oref = r["o64"], r["o32"], r["oref"]
    ok = (o64["status"] == 0) & (o32["status"] <= 1) & (oref["status"] <= 1)
    loc = lambda o: (o["obj"] + 300.0 * b["s0"])[ok]  # noqa: E731
    g32 = (loc(o32) - loc(o64)) / np.abs(loc(o64))
    gref = (loc(oref) - loc(o64)) / np.abs(loc(o64))
    return {"ok": int(ok.sum()), "g32_q90": float(np.quantile(g32, 0.9)), "gref_q90": float(np.quantile(gref, 0.9)),
            "status32": np.bincount(o32["status"], minlength=5).tolist(),
            "statusref": np.bincount(oref["status"], minlength=5).tolist()}


def main():
    import pytest
    b, A = triple()
    print(json.dumps({"before": gaps(b, A)}), flush=True)
    pre = ["tests/test_c3_sample.py", "tests/test_duals.py", "tests/test_edge_cases.py",
           "tests/test_gpu.py::test_c2_full_batch_matches_host_build", "tests/test_gpu.py::test_c4_full_batch_fp32_properties",
           "tests/test_gpu.py::test_c3_full_batch_lane_rows", "tests/test_gpu.py::test_fp32_accuracy_vs_reference_tolerance"]
    rc = pytest.main([os.path.join(ROOT, p) for p in pre] + ["-m", "gpu", "-q", "-p", "no:cacheprovider"])
    print(json.dumps({"pytest_rc": int(rc)}), flush=True)
    _, B = triple()
    print(json.dumps({"after": gaps(b, B)}), flush=True)
    for s in A:
        for k in A[s]:
            x, y = A[s][k], B[s][k]
            if not np.array_equal(x, y, equal_nan=True):
                cols = np.nonzero(np.any((x != y).reshape(-1, x.shape[-1]), axis=0))[0]
                print(json.dumps({"solve": s, "field": k, "n_instances": int(cols.size), "first": cols[:12].tolist()}),
                      flush=True)
    print(json.dumps({"done": True}), flush=True)


if __name__ == "__main__":
    main()
