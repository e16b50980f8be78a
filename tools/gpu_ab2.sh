#!/bin/bash
# ahead2 parity + A/B (k_upols_ahead vs k_upols_ahead2), VALU FMA rate microbenchmark
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-ab2}
timeout -k 10 60 tools/valubench/valubench > $O/valubench_$TAG.log 2>&1 && \
timeout -k 10 300 python -u -m pytest tests/test_upols_gpu.py -m gpu -x -q -k ahead --timeout 120 --timeout-method thread > $O/pytest_ahead_$TAG.log 2>&1 && \
for W in c5 c4 c3; do for K in 1 2; do
  NEO_HIP_AHEAD_KERNEL=$K timeout -k 10 200 python bench.py --workload $W --no-cpu-baseline --no-offline > $O/bench_${W}_k${K}_$TAG.json 2>&1 || exit $?
done; done
echo ab-ok
