#!/bin/bash
# batched-pass workgroup target: streaming bench vs offline batchbench on one box
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-ab7}
timeout -k 10 200 python tools/batchbench.py c5 5 96 NEO_HIP_BATCH_WGS=512 NEO_HIP_BATCH_WGS=1024 > $O/ab_c5_$TAG.log 2>&1 && \
for W in 512 1024; do NEO_HIP_BATCH_WGS=$W timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_w${W}_$TAG.json 2>&1 || exit $?; done
timeout -k 10 200 python tools/batchbench.py c5 5 96 NEO_HIP_BATCH_WGS=512 NEO_HIP_BATCH_WGS=1024 > $O/ab_c5b_$TAG.log 2>&1
echo ab-exit=$?
