#!/bin/bash
# after removing the spilling cacheable-row select: offline A/B + streaming bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-ab8}
timeout -k 10 300 python -u -m pytest tests/test_upols_gpu.py -m gpu -x -q -k "batch or ahead" --timeout 120 --timeout-method thread > $O/pytest_$TAG.log 2>&1 && \
timeout -k 10 200 python tools/batchbench.py c5 5 96 NEO_HIP_BATCH_WGS=512 NEO_HIP_BATCH_WGS=1024 NEO_HIP_BATCH_VAR=2,NEO_HIP_BATCH_WGS=512 > $O/ab_c5_$TAG.log 2>&1 && \
timeout -k 10 200 python tools/batchbench.py c4 5 96 NEO_HIP_BATCH_WGS=512 NEO_HIP_BATCH_WGS=1024 NEO_HIP_BATCH_VAR=2,NEO_HIP_BATCH_WGS=512 > $O/ab_c4_$TAG.log 2>&1 && \
for W in 512 1024; do NEO_HIP_BATCH_WGS=$W timeout -k 10 200 python bench.py --no-cpu-baseline > $O/bench_w${W}_$TAG.json 2>&1 || exit $?; done
echo ab-exit=$?
