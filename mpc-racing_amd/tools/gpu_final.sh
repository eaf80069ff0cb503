#!/bin/bash
# Round-end GPU session on the committed build: parity tests, smoke, bench line, rocprofv3 kernel stats,
# the two PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs) and their summary, the PMC calibration
# (tools/pmc_calib.hip: 1 GiB read / written at 4 and 8 B per lane), the C4 timeline and the other
# configurations' bench lines.  Every GPU step has its own time limit; the session stops at the first
# crash / timeout (test failures, rc 1, do not stop it).
# Usage: gpu_final.sh [A|B|AB]   A: tests, smoke, C4 profile / PMC / bench / timeline; B: the other
# configurations' bench lines, kernel statistics and PMC (C2, C3, C5); default AB (one call may not fit).
set -u
PART=${1:-AB}
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
B=$(python -c "import sys; sys.path.insert(0,'mpc-racing_amd'); from mpcracing import workload as wl; print(wl.CONFIGS['C4']['per_gpu'])")
if [[ $PART == *A* ]]; then
step pytest_gpu 900 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread
step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency
step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-latency
step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-latency
step pmc_sq 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-latency
step pmc_sum 120 python mpc-racing_amd/tools/pmc_summary.py gpurun_out/prof/run_kernel_stats.csv gpurun_out/pmc_fetch/run_counter_collection.csv gpurun_out/pmc_write/run_counter_collection.csv gpurun_out/pmc_C4.json mr_wave_kernel $B C4 gpurun_out/pmc_sq/run_counter_collection.csv
# the bench line's roofline.traffic comes from profiles/pmc_C4.json when its library hash is this build's
[ -s gpurun_out/pmc_C4.json ] && cp gpurun_out/pmc_C4.json profiles/pmc_C4.json
step bench 600 python bench.py
if [ -x variants/pmc_calib ]; then
  step calib_fetch 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/calib_fetch -o run --output-format csv -- variants/pmc_calib
  step calib_write 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/calib_write -o run --output-format csv -- variants/pmc_calib
fi
step timeline 300 python -u mpc-racing_amd/tools/timeline_probe.py C4 1
fi
if [[ $PART == *B* ]]; then
for c in C2 C3 C5; do
  step bench_$c 600 python bench.py --config $c --no-cpu-baseline
done
# kernel statistics and HBM traffic of C2, C3 and C5 (same passes as C4's; C5 also the SQ pass)
for c in C2 C3 C5; do
  BC=$(python -c "import sys; sys.path.insert(0,'mpc-racing_amd'); from mpcracing import workload as wl; print(wl.CONFIGS['$c']['per_gpu'])")
  step prof_$c 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$c -o run --output-format csv -- python bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline --no-latency
  step pmc_fetch_$c 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$c -o run --output-format csv -- python bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-latency
  step pmc_write_$c 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$c -o run --output-format csv -- python bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-latency
  SQ=""
  if [ "$c" = C5 ]; then
    step pmc_sq_$c 300 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq_$c -o run --output-format csv -- python bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline --no-latency
    SQ=gpurun_out/pmc_sq_$c/run_counter_collection.csv
  fi
  step pmc_sum_$c 120 python mpc-racing_amd/tools/pmc_summary.py gpurun_out/prof_$c/run_kernel_stats.csv gpurun_out/pmc_fetch_$c/run_counter_collection.csv gpurun_out/pmc_write_$c/run_counter_collection.csv gpurun_out/pmc_$c.json mr_wave_kernel $BC $c $SQ
  [ -s gpurun_out/pmc_$c.json ] && cp gpurun_out/pmc_$c.json profiles/pmc_$c.json
done
fi
