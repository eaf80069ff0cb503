#!/bin/bash
# GPU parity tests + smoke + one bench line (no CPU baseline) on the in-tree build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > gpurun_out/pytest_t.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_t.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_t.log 2>&1 &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_t.log 2>&1
rc2=$?
echo "smoke/bench rc=$rc2"; tail -1 gpurun_out/smoke_t.log; tail -1 gpurun_out/bench_t.log | cut -c1-300
exit $rc2
