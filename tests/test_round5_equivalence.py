"""Round-5 rewrites that claim bit-identical iterates, pinned on the host build.

The kernel source's compile-time switches MR_SOC_CAPTURE (a second-order correction accumulates the
constraint values its trial evaluation captured, instead of evaluating the trial point again) and
MR_LS_BRANCHFREE (the trial evaluation's slot loop without per-slot branches) change how the work is
done, not what is computed.  This test builds the host twin of the same
source with both off (the round-4 forms) and requires every output -- statuses, iteration counts,
iterates, objective, KKT error, constraint violation -- to be bitwise equal to the default build on C4
(fp32, second-order corrections frequent) and C3 (fp64, lane rows and the restoration phase).
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import host_twin as ht
from mpcracing import workload as wl

HERE = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(HERE, "..", "mpc-racing_amd", "csrc")

_RUN = r"""
import sys, numpy as np
sys.path.insert(0, {tests!r}); sys.path.insert(0, {pkg!r})
import host_twin as ht
from mpcracing import workload as wl
name, prec, n, out = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4]
cfg = wl.CONFIGS[name]
tyres = wl.tyre_coeffs(cfg["tyres"]) if cfg["tyres"] else None
b = wl.make_batch(name, limit=n)
o = ht.solve(ht.config(cfg["N"], cfg["model"], prec, cfg["lane"], cfg["Ts"], tol=1e-4, acceptable_tol=1e-2,
                       acceptable_iter=15), b, tyres=tyres, nthreads=8)
np.savez(out, **o)
"""


def _solve(name, prec, n, lib, out):
    env = dict(os.environ, MR_HOST_TWIN_LIB=lib) if lib else dict(os.environ)
    code = _RUN.format(tests=HERE, pkg=os.path.join(HERE, "..", "mpc-racing_amd"))
    subprocess.run([sys.executable, "-c", code, name, prec, str(n), out], check=True, env=env, timeout=900)
    return dict(np.load(out))


@pytest.fixture(scope="module")
def round4_forms(tmp_path_factory):
    d = tmp_path_factory.mktemp("r4forms")
    lib = str(d / "libmpcracing_host_r4forms.so")
    subprocess.run(["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-fPIC", "-shared", "-fopenmp",
                    "-DMR_SOC_CAPTURE=0", "-DMR_LS_BRANCHFREE=0", "-o", lib,
                    os.path.join(CSRC, "mpcracing_host.cpp")], check=True, timeout=900)
    return lib, d


@pytest.mark.parametrize("name,prec,n", [("C4", "fp32", 48), ("C3", "fp64", 16)])
def test_soc_capture_and_branchfree_trials_are_bit_identical(round4_forms, name, prec, n):
    lib, d = round4_forms
    ref = _solve(name, prec, n, lib, str(d / f"{name}_r4.npz"))
    new = _solve(name, prec, n, None, str(d / f"{name}_r5.npz"))
    for k in ref:
        assert np.array_equal(ref[k], new[k], equal_nan=True), k
