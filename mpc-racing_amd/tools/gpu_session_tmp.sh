set -u
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu.py tests/test_gpu_closed_loop.py -x -v --timeout 300 --timeout-method thread -s > gpurun_out/pytest_sel.log 2>&1; rc=$?; echo "rc=$rc" >> gpurun_out/pytest_sel.log; if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 300 python -u mpc-racing_amd/tools/timeline_probe.py C4 2 > gpurun_out/tl_order2.log 2>&1 || exit $?
timeout -k 10 600 python -u mpc-racing_amd/tools/closed_loop_bench.py 4096 40 > gpurun_out/clbench.log 2>&1 || exit $?
