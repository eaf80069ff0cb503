set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > gpurun_out/counters.txt 2>&1
grep -o "TA_[A-Z_]*\|TD_[A-Z_]*\|TCP_[A-Z_]*" gpurun_out/counters.txt | sort -u > gpurun_out/counters_tatd.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu.py tests/test_duals.py -m gpu -v -rA --timeout 300 --timeout-method thread > gpurun_out/pytest_r2b.log 2>&1
echo "rc=$?" >> gpurun_out/pytest_r2b.log
