set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for v in W1 W2 F; do
  MR_PRODUCT_LIB=variants/lib_$v.so timeout -k 5 120 python -u bench.py --config C5 --steps 1 --warmup 0 --no-cpu-baseline --no-latency > gpurun_out/c5_$v.log 2>&1
  rc=$?
  echo "$v rc=$rc $(tail -1 gpurun_out/c5_$v.log | cut -c1-200)"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
