set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B=$(python -c "import sys; sys.path.insert(0,'mpc-racing_amd'); from mpcracing import workload as wl; print(wl.CONFIGS['C4']['per_gpu'])")
timeout -k 10 700 python -u -m pytest tests -m gpu -v -rA --timeout 300 --timeout-method thread > gpurun_out/pytest_r2e.log 2>&1
echo "pytest rc=$?" >> gpurun_out/pytest_r2e.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_r2e.log 2>&1 &&
timeout -k 10 600 python -u bench.py > gpurun_out/bench_r2e.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r2e -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-latency > gpurun_out/prof_r2e.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-latency > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-latency > gpurun_out/pmc_write.log 2>&1 &&
python mpc-racing_amd/tools/pmc_summary.py gpurun_out/prof_r2e/run_kernel_stats.csv gpurun_out/pmc_fetch/run_counter_collection.csv gpurun_out/pmc_write/run_counter_collection.csv gpurun_out/pmc_C4.json mr_wave_kernel $B C4 > gpurun_out/pmc_sum.log 2>&1 &&
cp gpurun_out/pmc_C4.json profiles/pmc_C4.json &&
timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-latency > gpurun_out/bench_r2e_pmc.log 2>&1 &&
timeout -k 10 300 python -u mpc-racing_amd/tools/timeline_probe.py C4 1 > gpurun_out/timeline_r2e.log 2>&1 &&
timeout -k 10 300 python -u mpc-racing_amd/tools/phase_probe.py C4 > gpurun_out/phase_r2e.log 2>&1
echo "rc=$?" >> gpurun_out/pmc_sum.log
