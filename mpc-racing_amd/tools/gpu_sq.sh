#!/bin/bash
# SQ counter passes (one rocprofv3 --pmc run each, <= 8 SQ counters) over one C4 bench step:
# where the wave kernel's cycles go (issue vs waits, VALU vs VMEM vs LDS instruction counts).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
CFG=${CFG:-C4}
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA -d gpurun_out/sq_a_$CFG -o run --output-format csv -- python bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-latency > gpurun_out/sq_a_$CFG.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_WAVES -d gpurun_out/sq_b_$CFG -o run --output-format csv -- python bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline --no-latency > gpurun_out/sq_b_$CFG.log 2>&1
echo "rc=$?" >> gpurun_out/sq_a_$CFG.log
