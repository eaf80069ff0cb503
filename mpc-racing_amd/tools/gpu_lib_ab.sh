#!/bin/bash
# A/B of library variants on the B = 1 agent call and the C2 / C4 bench lines: for each given .so
# (MR_PRODUCT_LIB), tools/agent_probe.py 100, then bench.py --config C2 and C4 without the CPU baseline.
# Lines to gpurun_out/<tag>_<name>_{agent,C2,C4}.json; stops at the first crash / timeout.
# Usage: gpu_lib_ab.sh TAG lib1.so lib2.so ...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
TAG=$1; shift
for lib in "$@"; do
  n=$(basename "$lib" .so)
  MR_PRODUCT_LIB=$lib timeout -k 10 300 python -u mpc-racing_amd/tools/agent_probe.py 100 > gpurun_out/${TAG}_${n}_agent.json 2> gpurun_out/${TAG}_${n}_agent.err || exit $?
  for c in C2 C4; do
    MR_PRODUCT_LIB=$lib timeout -k 10 300 python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-latency \
      > gpurun_out/${TAG}_${n}_$c.json 2> gpurun_out/${TAG}_${n}_$c.err || exit $?
  done
  echo "$n done" >> gpurun_out/${TAG}_ab.log
done
