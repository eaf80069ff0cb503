#!/bin/bash
# Profiles of the product build: rocprofv3 kernel stats of bench.py, the two PMC passes (HBM bytes),
# their summary (gpurun_out/pmc_C4.json), then the per-phase probe (variants/lib_cyc.so) if present.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$(python -c "import sys; sys.path.insert(0,'mpc-racing_amd'); from mpcracing import workload as wl; print(wl.CONFIGS['C4']['per_gpu'])")
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency > gpurun_out/prof.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-latency > gpurun_out/pmc_fetch.log 2>&1 || exit $?
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-latency > gpurun_out/pmc_write.log 2>&1 || exit $?
python mpc-racing_amd/tools/pmc_summary.py gpurun_out/prof/run_kernel_stats.csv gpurun_out/pmc_fetch/run_counter_collection.csv gpurun_out/pmc_write/run_counter_collection.csv gpurun_out/pmc_C4.json mr_wave_kernel $B C4 > gpurun_out/pmc_sum.log 2>&1 || exit $?
if [ -f variants/lib_cyc.so ]; then
  MR_PRODUCT_LIB=variants/lib_cyc.so timeout -k 10 300 python -u mpc-racing_amd/tools/phase_probe.py C4 > gpurun_out/phase_cyc.log 2>&1 || exit $?
fi
