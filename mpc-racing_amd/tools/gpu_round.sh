#!/bin/bash
# One GPU session: parity tests, smoke, bench, rocprofv3 kernel trace.  Each GPU step has its
# own time limit; a crash / timeout (rc >= 124) ends the session, test failures (rc 1) do not.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name: $*" >> gpurun_out/session.log
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> gpurun_out/session.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
what=${1:-all}
if [ "$what" = all ] || [ "$what" = tests ]; then
  step pytest_gpu 1100 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
fi
if [ "$what" = all ] || [ "$what" = bench ]; then
  step bench 900 python bench.py
  step prof 900 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency
fi
if [ "$what" = all ] || [ "$what" = bench ] || [ "$what" = timeline ]; then
  step timeline 300 python -u mpc-racing_amd/tools/timeline_probe.py C4 1
fi
if [ "$what" = probe ]; then
  step fp32_probe 600 python -u mpc-racing_amd/tools/fp32_probe.py 256 4
fi
if [ "$what" = pmc ]; then
  step pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline
  step pmc_write 900 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline
fi
