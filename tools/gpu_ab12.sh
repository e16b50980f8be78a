#!/bin/bash
# batched MAC with cacheable filter rows (first pcb rows per channel) vs all nontemporal
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-ab12}
timeout -k 10 300 python -u -m pytest tests/test_upols_gpu.py -m gpu -x -q -k "ahead or batch" --timeout 120 --timeout-method thread > $O/pytest_$TAG.log 2>&1 && \
timeout -k 10 200 python tools/batchbench.py c5 5 96 NEO_HIP_BATCH_CACHE_ROWS=0 NEO_HIP_BATCH_CACHE_ROWS=206 NEO_HIP_BATCH_CACHE_ROWS=400 > $O/ab_c5_$TAG.log 2>&1 && \
for V in 0 206; do NEO_HIP_BATCH_CACHE_ROWS=$V timeout -k 10 200 python bench.py --no-cpu-baseline --no-offline > $O/bench_c5_pc${V}_$TAG.json 2>&1 || exit $?; done && \
for V in 0 412; do NEO_HIP_BATCH_CACHE_ROWS=$V timeout -k 10 200 python bench.py --workload c4 --no-cpu-baseline --no-offline > $O/bench_c4_pc${V}_$TAG.json 2>&1 || exit $?; done
echo ab-exit=$?
