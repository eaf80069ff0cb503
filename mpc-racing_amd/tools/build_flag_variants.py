"""Developer A/B builds of the code-generation defaults (mpcracing/build.py DEFAULT_FLAGS, the fp32 launch
bounds of mpcracing.hip): variants/lib_<name>.so, run by tools/gpu_flags_ab.sh on the GPU box.

  base     the product flags
  denorm   fp32 denormals kept (no -fgpu-flush-denormals-to-zero)
  slp      SLP vectorisation on (no -fno-slp-vectorize)
  w1       fp32 solve kernel at 1 wave per SIMD (MR_WAVES_PER_SIMD_F32=1, 512 VGPRs)
  ric3     Riccati operand gathers three stages ahead instead of two (MR_RIC_AHEAD=3)
  s464     a 464-word record stride (the footprint the rejected paired factorisation needed, git e417017)
  s336     the 336-word record stride of the build that still stored p1 / k1 (git 60d581f)
  prio60   waves past iteration 60 raise their issue priority (s_setprio 3)
  cyc      per-sweep shader-cycle counters of the trace instance (tools/phase_probe.py)
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
    "ric3": DEFAULT_FLAGS + ["-DMR_RIC_AHEAD=3"],
    "s464": DEFAULT_FLAGS + ["-DMR_RC_STRIDE_FORCE=464"],
    "s336": DEFAULT_FLAGS + ["-DMR_RC_STRIDE_FORCE=336"],
    "prio60": DEFAULT_FLAGS + ["-DMR_PRIO_ITER=60"],
    "cyc": DEFAULT_FLAGS + ["-DMR_PHASE_CYCLES=1"],
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
