set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u mpc-racing_amd/tools/fp32_probe.py 512 0 > gpurun_out/probe2.log 2>&1 &&
MR_PRODUCT_LIB=$PWD/mpc-racing_amd/csrc/libmpcracing_fma.so timeout -k 10 300 python -u bench.py --no-cpu-baseline > gpurun_out/bench_fma.log 2>&1 &&
MR_PRODUCT_LIB=$PWD/mpc-racing_amd/csrc/libmpcracing_fma.so timeout -k 10 600 python -u -m pytest tests/test_gpu.py -m gpu -v -rA --timeout 300 --timeout-method thread > gpurun_out/pytest_fma.log 2>&1
echo "rc=$?" >> gpurun_out/probe2.log
