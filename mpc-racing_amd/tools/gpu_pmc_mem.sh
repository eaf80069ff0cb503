#!/bin/bash
# Memory-pipeline PMC passes over one C4 bench step (each pass its own rocprofv3 run, <= 2 TA/TD,
# <= 4 TCP, <= 8 SQ counters): is the vector-memory pipeline (TA/TD/TCP) the shared bottleneck?
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out/pmcmem
export TMPDIR=/tmp
CMD="python bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-latency"
i=0
for P in "TA_TA_BUSY_sum GRBM_GUI_ACTIVE" "TD_TD_BUSY_sum TD_TC_STALL_sum" "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" \
         "TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM SQ_ACTIVE_INST_VMEM SQ_IFETCH" \
         "SQC_ICACHE_MISSES SQC_ICACHE_HITS"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmcmem/p$i -o run --output-format csv -- $CMD > gpurun_out/pmcmem/p$i.log 2>&1
  rc=$?
  echo "pass $i [$P] rc=$rc" >> gpurun_out/pmcmem/summary.log
  if [ $rc -ne 0 ]; then exit $rc; fi
done
