"""Developer A/B builds of the code-generation defaults (mpcracing/build.py DEFAULT_FLAGS, the fp32 launch
bounds of mpcracing.hip): variants/lib_<name>.so, run by tools/gpu_flags_ab.sh on the GPU box.

  base     the product flags
  denorm   fp32 denormals kept (no -fgpu-flush-denormals-to-zero)
  slp      SLP vectorisation on (no -fno-slp-vectorize)
  w1       fp32 solve kernel at 1 wave per SIMD (MR_WAVES_PER_SIMD_F32=1, 512 VGPRs)
  cyc      per-sweep shader-cycle counters of the trace instance (tools/phase_probe.py)
  nofma    no floating-point contraction (-ffp-contract=off: the host build's arithmetic, no FMA)
  inline   the sweeps force-inlined into the solve kernel (MR_SWEEP_INLINE: one register allocation, no call ABI)
  wspad    64 Ki unused words after each instance's workspace (an out-of-range write would land there)
  poisonP  LDS and workspace filled with pattern P (1 NaN, 2 zero, 3 -1e30) at kernel start (determinism_probe.py)
"""
import os
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, os.path.join(REPO, "mpc-racing_amd"))
from mpcracing.build import DEFAULT_FLAGS, build_hip  # noqa: E402

VARIANTS = {
    "base": DEFAULT_FLAGS,
    "denorm": [f for f in DEFAULT_FLAGS if f != "-fgpu-flush-denormals-to-zero"],
    "slp": [f for f in DEFAULT_FLAGS if f != "-fno-slp-vectorize"],
    "w1": DEFAULT_FLAGS + ["-DMR_WAVES_PER_SIMD_F32=1"],
    "cyc": DEFAULT_FLAGS + ["-DMR_PHASE_CYCLES=1"],
    "nofma": ["-ffp-contract=off"] + [f for f in DEFAULT_FLAGS if not f.startswith("-ffp-contract")],
    "poison1": DEFAULT_FLAGS + ["-DMR_POISON=1"],
    "poison2": DEFAULT_FLAGS + ["-DMR_POISON=2"],
    "poison3": DEFAULT_FLAGS + ["-DMR_POISON=3"],
    "inline": DEFAULT_FLAGS + ["-DMR_SWEEP_INLINE=1"],
    "wspad": DEFAULT_FLAGS + ["-DMR_WS_PAD=65536"],
}


def main():
    names = sys.argv[1:] or list(VARIANTS)
    os.makedirs(os.path.join(REPO, "variants"), exist_ok=True)
    with ThreadPoolExecutor(len(names)) as ex:
        futs = [ex.submit(build_hip, True, True, os.path.join(REPO, "variants", f"lib_{n}.so"), VARIANTS[n])
                for n in names]
        for f in futs:
            print(f.result(), flush=True)


if __name__ == "__main__":
    main()
