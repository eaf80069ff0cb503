#!/bin/bash
# A/B of library builds (variants/lib_<v>.so, built on the CPU side): one bench line per
# argument <variant>[:<config>] (config default C4).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for a in "$@"; do
  v=${a%%:*}; c=C4; [ "$a" != "$v" ] && c=${a#*:}
  MR_PRODUCT_LIB=variants/lib_$v.so timeout -k 10 300 python -u bench.py --config $c --no-cpu-baseline --no-latency > gpurun_out/ab_${v}_$c.log 2>&1
  rc=$?
  echo "$v $c rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
for lib in variants/lib_cyc*.so; do
  [ -f "$lib" ] || continue
  v=$(basename "$lib" .so); v=${v#lib_}
  MR_PRODUCT_LIB=$lib timeout -k 10 300 python -u mpc-racing_amd/tools/phase_probe.py C4 > gpurun_out/phase_$v.log 2>&1
  rc=$?
  echo "phase $v rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
