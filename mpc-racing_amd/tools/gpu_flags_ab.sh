#!/bin/bash
# A/B of code-generation / kernel options (tools/build_flag_variants.py builds variants/lib_<v>.so on the
# CPU side): per variant one C4 bench line and one timeline (the batch time is set by a few tail solves
# whose iterates change with any fp32 rounding change, so the timeline's mean in-batch time per
# instance-iteration is the variant-insensitive throughput figure).  Each step time-limited; stop on the
# first failure.  Summary: python mpc-racing_amd/tools/ab_summary.py gpurun_out/x base denorm ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
[ $# -eq 0 ] && set -- base denorm slp w1
for v in "$@"; do
  MR_PRODUCT_LIB=variants/lib_$v.so timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-latency > gpurun_out/ab_$v.log 2>&1 || exit $?
  MR_PRODUCT_LIB=variants/lib_$v.so timeout -k 10 300 python -u mpc-racing_amd/tools/timeline_probe.py C4 1 > gpurun_out/abtl_$v.log 2>&1 || exit $?
  echo "$v done"
done
