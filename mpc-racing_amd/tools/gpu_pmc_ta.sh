#!/bin/bash
# Memory-pipeline and issue PMC passes over one C4 bench step of a library variant ($1 = path):
# TA/TD busy (is the vector-memory pipeline the shared limit?) and SQ wave-cycle split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/pmcta
export TMPDIR=/tmp
export MR_PRODUCT_LIB=$1
CMD="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-latency"
i=0
for P in "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "TD_TD_BUSY_sum TD_TC_STALL_sum" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM SQ_INSTS_LDS" \
         "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/pmcta/p$i -o run --output-format csv -- $CMD > gpurun_out/pmcta/p$i.log 2>&1
  rc=$?
  echo "pass $i [$P] rc=$rc"
  if [ $rc -ne 0 ]; then exit $rc; fi
done
