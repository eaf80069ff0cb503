#!/bin/bash
# A/B session: bench lines per variant (gpu_ab.sh), the named variant's parity subset, timelines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
cand=$1; shift
MR_PRODUCT_LIB=variants/lib_$cand.so timeout -k 10 400 python -u -m pytest tests/test_gpu.py -k "fp64_vs_oracle or c4_full or c4_fp64 or accuracy" -x -q --timeout 300 --timeout-method thread > gpurun_out/parity_$cand.log 2>&1
echo "parity $cand rc=$?"
bash mpc-racing_amd/tools/gpu_ab.sh "$@" || exit $?
for v in "$@"; do
  MR_PRODUCT_LIB=variants/lib_$v.so timeout -k 10 200 python -u mpc-racing_amd/tools/timeline_probe.py C4 1 > gpurun_out/timeline_$v.log 2>&1 || exit $?
done
