#!/bin/bash
# batched MAC: co-resident workgroups trading issue priority vs not
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-ab13}
timeout -k 10 300 python -u -m pytest tests/test_upols_gpu.py -m gpu -x -q -k "ahead or batch" --timeout 120 --timeout-method thread > $O/pytest_$TAG.log 2>&1 && \
timeout -k 10 200 python tools/batchbench.py c5 5 96 NEO_HIP_BATCH_PRIO=0 NEO_HIP_BATCH_PRIO=1 > $O/ab_c5_$TAG.log 2>&1 && \
timeout -k 10 200 python tools/batchbench.py c4 5 96 NEO_HIP_BATCH_PRIO=0 NEO_HIP_BATCH_PRIO=1 > $O/ab_c4_$TAG.log 2>&1 && \
timeout -k 10 120 python tools/probebench.py c5 > $O/probe_$TAG.log 2>&1 && \
for V in 0 1; do NEO_HIP_BATCH_PRIO=$V timeout -k 10 200 python bench.py --no-cpu-baseline --no-offline > $O/bench_c5_p${V}_$TAG.json 2>&1 || exit $?; done
echo ab-exit=$?
