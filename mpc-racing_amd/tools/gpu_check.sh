#!/bin/bash
# Developer GPU session: parity tests, then the iteration/timing probe.  Each GPU step is
# time-limited; a crash or timeout (rc >= 124) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {
  local name=$1 lim=$2; shift 2
  echo "== $name: $*" >> gpurun_out/session.log
  timeout -k 10 "$lim" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> gpurun_out/session.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -rA
step probe 400 python -u mpc-racing_amd/tools/iter_probe.py ${PROBE:-C4,C3}
