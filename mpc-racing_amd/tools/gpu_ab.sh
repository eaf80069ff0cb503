#!/bin/bash
# A/B of library variants on the C4 bench line: for each given .so (MR_PRODUCT_LIB), bench.py without the
# CPU baseline, STEPS timed steps (default 3); the list is run ROUNDS times (default 1, interleaved, so
# drift hits every variant alike); lines to gpurun_out/<tag>_ab_<name>[_r<round>].json.  Stops at the first
# crash/timeout.
# Usage: [STEPS=n] [ROUNDS=r] gpu_ab.sh TAG lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
TAG=$1; shift
STEPS=${STEPS:-3}
ROUNDS=${ROUNDS:-1}
for r in $(seq 1 "$ROUNDS"); do
  for lib in "$@"; do
    n=$(basename "$lib" .so)
    [ "$ROUNDS" -gt 1 ] && n=${n}_r$r
    MR_PRODUCT_LIB=$lib timeout -k 10 300 python bench.py --steps "$STEPS" --warmup 1 --no-cpu-baseline --pipeline 0 > gpurun_out/${TAG}_ab_$n.json 2> gpurun_out/${TAG}_ab_$n.err
    rc=$?
    echo "$n rc=$rc" >> gpurun_out/${TAG}_ab.log
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
