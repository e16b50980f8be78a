#!/bin/bash
# A/B of the batched MAC variants (NEO_HIP_BATCH_VAR) offline and in the streaming bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-ab}
timeout -k 10 200 python tools/batchbench.py c5 5 96 NEO_HIP_BATCH_VAR=0 NEO_HIP_BATCH_VAR=1 NEO_HIP_BATCH_VAR=2 > $O/ab_c5_$TAG.log 2>&1 && \
timeout -k 10 200 python tools/batchbench.py c4 5 96 NEO_HIP_BATCH_VAR=0 NEO_HIP_BATCH_VAR=1 NEO_HIP_BATCH_VAR=2 > $O/ab_c4_$TAG.log 2>&1 && \
for V in 0 2; do NEO_HIP_BATCH_VAR=$V timeout -k 10 200 python bench.py --no-cpu-baseline --no-offline > $O/bench_var${V}_$TAG.json 2>&1 || exit $?; done
echo ab-ok
