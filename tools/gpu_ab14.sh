#!/bin/bash
# batched MAC: paired units per 8-wave workgroup (var 3) vs var 2
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-ab14}
timeout -k 10 300 python -u -m pytest tests/test_upols_gpu.py -m gpu -x -q -k "ahead or batch" --timeout 120 --timeout-method thread > $O/pytest_$TAG.log 2>&1 && \
timeout -k 10 200 python tools/batchbench.py c5 5 96 NEO_HIP_BATCH_VAR=2 NEO_HIP_BATCH_VAR=3 > $O/ab_c5_$TAG.log 2>&1 && \
timeout -k 10 200 python tools/batchbench.py c4 5 96 NEO_HIP_BATCH_VAR=2 NEO_HIP_BATCH_VAR=3 > $O/ab_c4_$TAG.log 2>&1 && \
timeout -k 10 120 python tools/probebench.py c5 > $O/probe_$TAG.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --no-offline > $O/bench_c5_$TAG.json 2>&1 && \
timeout -k 10 200 python bench.py --workload c4 --no-cpu-baseline --no-offline > $O/bench_c4_$TAG.json 2>&1
echo ab-exit=$?
