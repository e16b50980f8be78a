#!/bin/bash
# Is the T=32 batched MAC compute- or memory-bound? Cache-resident shape vs C5, T=16 vs 32, clocks
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-ab5}
timeout -k 10 200 python tools/batchbench.py 256x512x32768 5 96 NEO_HIP_BATCH_VAR=0 NEO_HIP_BATCH_VAR=2 NEO_HIP_BATCH_VAR=3 > $O/ab_res_$TAG.log 2>&1 && \
timeout -k 10 200 python tools/batchbench.py c5 5 96 NEO_HIP_BATCH_VAR=3 NEO_HIP_BATCH_T=16,NEO_HIP_BATCH_VAR=0 > $O/ab_t16_$TAG.log 2>&1 && \
(timeout -k 10 200 python tools/batchbench.py c5 40 96 NEO_HIP_BATCH_T=32,NEO_HIP_BATCH_VAR=3 > $O/ab_long_$TAG.log 2>&1 &
 sleep 25; timeout 20 rocm-smi --showclocks --showpower > $O/smi_$TAG.log 2>&1; wait)
echo ab-exit=$?
