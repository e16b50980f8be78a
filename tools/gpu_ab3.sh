#!/bin/bash
# batched MAC: variants 0/2/3 offline A/B, SQ counters of variant 3, ahead2 kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-ab3}
timeout -k 10 200 python tools/batchbench.py c5 5 96 NEO_HIP_BATCH_VAR=0 NEO_HIP_BATCH_VAR=2 NEO_HIP_BATCH_VAR=3 > $O/ab_c5_$TAG.log 2>&1 && \
timeout -k 10 200 python tools/batchbench.py c4 5 96 NEO_HIP_BATCH_VAR=0 NEO_HIP_BATCH_VAR=2 NEO_HIP_BATCH_VAR=3 > $O/ab_c4_$TAG.log 2>&1 && \
cd /tmp && export TMPDIR=/tmp && \
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE --output-format csv -d $O/pmc_sq_$TAG -o run -- python3 $R/tools/batchbench.py c5 1 64 NEO_HIP_BATCH_VAR=3 > $O/pmc_sq_$TAG.log 2>&1 && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace_c5_$TAG -o run -- python3 $R/bench.py --steps 64 --warmup 4 --no-cpu-baseline --no-offline > $O/trace_c5_$TAG.log 2>&1
echo ab-exit=$?
