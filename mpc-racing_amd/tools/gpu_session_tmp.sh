set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_gpu.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
bash mpc-racing_amd/tools/gpu_flags_ab.sh head new s336
