#!/bin/bash
# A development GPU session: the named steps in order, each under its own time limit; the session stops
# at the first crash / timeout (test failures, rc 1, do not stop it).  Logs under gpurun_out/<tag>_<step>.*
#   tests   python -m pytest tests -m gpu
#   smoke   __graft_entry__.smoke()
#   bench   bench.py (default line)
#   prof    rocprofv3 --kernel-trace --stats of the C4 bench command
#   phase   tools/phase_probe.py on the C4 tail instances (cycle-counter build in variants/)
#   tl      tools/timeline_probe.py C4
#   c2 c3 c5  bench.py --config Cx --no-cpu-baseline
#   agent   tools/agent_probe.py (the B = 1 agent call alone)
#   agent_ic  the same under one PMC pass: instruction-cache hits / misses and wave wait cycles
# Usage: gpu_session.sh TAG step...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=$1; shift
step() {  # name limit cmd...
  local name=$1 lim=$2; shift 2
  echo "== $name: $*" >> gpurun_out/${TAG}_session.log
  timeout -k 10 "$lim" "$@" > "gpurun_out/${TAG}_$name.log" 2>&1
  local rc=$?
  echo "== $name rc=$rc" >> gpurun_out/${TAG}_session.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    tests) step tests 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    bench) step bench 600 python bench.py ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency ;;
    phase) step phase 600 env MR_PRODUCT_LIB=variants/lib_cycles.so python -u mpc-racing_amd/tools/phase_probe.py C4 ;;
    tl) step tl 300 python -u mpc-racing_amd/tools/timeline_probe.py C4 1 ;;
    agent) step agent 300 python -u mpc-racing_amd/tools/agent_probe.py 100 ;;
    agent_ic) step agent_ic 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQC_ICACHE_HITS SQC_ICACHE_MISSES -d gpurun_out/${TAG}_agent_ic -o run --output-format csv -- python -u mpc-racing_amd/tools/agent_probe.py 10 ;;
    c2|c3|c5) C=$(echo $s | tr a-z A-Z); step bench_$C 600 python bench.py --config $C --no-cpu-baseline ;;
    *) echo "unknown step $s" >> gpurun_out/${TAG}_session.log ;;
  esac
done
