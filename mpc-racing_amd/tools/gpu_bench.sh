#!/bin/bash
# Developer GPU session: bench line, rocprofv3 kernel stats, and the two PMC passes
# (FETCH_SIZE / WRITE_SIZE in separate runs).  Each step time-limited; stop on the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-C4}
timeout -k 10 300 python -u bench.py --config $CFG > gpurun_out/bench_$CFG.json 2> gpurun_out/bench_$CFG.err &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$CFG -o run --output-format csv -- python bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-latency > gpurun_out/prof_$CFG.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch_$CFG -o run --output-format csv -- python bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-latency > gpurun_out/pmc_fetch_$CFG.log 2>&1 &&
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write_$CFG -o run --output-format csv -- python bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-latency > gpurun_out/pmc_write_$CFG.log 2>&1
echo "rc=$?" >> gpurun_out/bench_$CFG.err
