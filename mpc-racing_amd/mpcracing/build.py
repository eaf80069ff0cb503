"""In-tree builds of the native libraries (no JIT cache: the .so files travel with the repo).

* libmpcracing.so       -- the product: gfx950 kernels + C ABI (hipcc --offload-arch=gfx950)
* libmpcracing_host.so  -- TEST-ONLY g++ build of the same solver source (CPU test suite)
"""
import os
import subprocess

from .abi import CSRC, PRODUCT_LIB, HOST_TWIN_LIB

HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
SOURCES = ["mpcracing.hip", "mr_batch.h", "mr_solver.h", "mr_common.h", "gen_dynamics.h", "mr_wave.h", "mr_wave_prims.h", "mr_track.h", "mr_agent.h", "mr_plant.h"]
INCLUDE = os.path.abspath(os.path.join(CSRC, "..", "..", "include"))


def _stale(target, deps):
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(d) > t for d in deps)


DEFAULT_FLAGS = ["-ffp-contract=fast-honor-pragmas", "-fgpu-flush-denormals-to-zero", "-fno-slp-vectorize"]


def build_hip(force=False, verbose=True, out=None, flags=None):
    """Build libmpcracing.so (or a developer A/B variant at ``out`` with ``flags`` replacing the
    default code-generation flags; load it with MR_PRODUCT_LIB)."""
    out = out or PRODUCT_LIB
    deps = [os.path.join(CSRC, s) for s in SOURCES] + [os.path.join(INCLUDE, "mpcracing.h"), __file__]
    if not force and not _stale(out, deps):
        return out
    # FMA contraction on (-ffp-contract=fast): the round-1 note about "huge defects at iteration 0" with
    # contraction came from the old lane-per-instance kernel (deleted); the wave kernel with contraction
    # passes every fp64 parity test against the oracle and the GPU-vs-host-build status tests, and is
    # 2.7 % faster on C4 (profiles/r02_fma_ab.json).  The host twin stays -ffp-contract=off (IEEE
    # reference for the CPU tests).  "fast-honor-pragmas" (not "fast", which fuses in the backend
    # regardless of source pragmas): the centerline / sensing / plant kernels below the
    # `#pragma clang fp contract(off)` in mpcracing.hip stay bit-exact with the host build.
    # fp32 kernels use the hardware reciprocal / square root / transcendentals (v_rcp, v_sqrt, v_sin,
    # v_exp, v_log: a few ulp) instead of the correctly rounded library sequences -- the fp32 solve is
    # instruction-latency bound and its KKT noise floor (~1e-3) is far above these errors; fp64 stays IEEE.
    # fp32 denormals flush to zero (-fgpu-flush-denormals-to-zero): every fp32 division / log otherwise
    # carries a frexp/ldexp range-scaling sequence (~4 extra VALU ops each); no fp32 quantity of the
    # solve lives near 1e-38.  fp64 (the centerline kernels, fp64 solves) keeps IEEE denormals.
    # No SLP vectorisation (-fno-slp-vectorize): the v_pk_* pairs it formed in the generated dynamics
    # code cost more register moves than they saved (eval sweep 4 975 -> 3 939 VALU instructions, its
    # scratch spills gone).  A/B on C4: profiles/r03_flags_ab.json (tools/gpu_flags_ab.sh).
    cg = flags if flags is not None else DEFAULT_FLAGS
    cmd = [HIPCC, "--offload-arch=gfx950", "-O3", *cg, "-std=c++17", "-fPIC", "-shared",
           "-Wno-unused-result", "-fno-hip-fp32-correctly-rounded-divide-sqrt", "-fgpu-approx-transcendentals",
           "-o", out, os.path.join(CSRC, "mpcracing.hip")]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return out


def build_host_twin(force=False, verbose=True):
    deps = [os.path.join(CSRC, s) for s in ["mpcracing_host.cpp"] + SOURCES[1:]] + \
           [os.path.join(INCLUDE, "mpcracing.h")]
    if not force and not _stale(HOST_TWIN_LIB, deps):
        return HOST_TWIN_LIB
    cmd = ["g++", "-O2", "-ffp-contract=off", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-o", HOST_TWIN_LIB,
           os.path.join(CSRC, "mpcracing_host.cpp")]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.run(cmd, check=True)
    return HOST_TWIN_LIB
