#!/bin/bash
# fp32 accuracy / parity subset per library variant: variants/lib_<v>.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for v in "$@"; do
  MR_PRODUCT_LIB=variants/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu.py -k "fp64_vs_oracle or c4_full or c5_full or c4_fp64 or accuracy" -q -rA --timeout 300 --timeout-method thread > gpurun_out/parity_$v.log 2>&1
  rc=$?
  echo "parity $v rc=$rc"
  if [ $rc -gt 1 ]; then exit $rc; fi
done
