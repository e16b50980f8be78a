#!/bin/bash
# LDS-DMA batched MAC variants: parity (batched + lookahead tests) and offline A/B
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-ab4}
for V in 4 5; do
  NEO_HIP_BATCH_VAR=$V timeout -k 10 300 python -u -m pytest tests/test_upols_gpu.py -m gpu -x -q -k "batch or ahead" --timeout 120 --timeout-method thread > $O/pytest_var${V}_$TAG.log 2>&1 || exit $?
done
timeout -k 10 200 python tools/batchbench.py c5 5 96 NEO_HIP_BATCH_VAR=2 NEO_HIP_BATCH_VAR=3 NEO_HIP_BATCH_VAR=4 NEO_HIP_BATCH_VAR=5 > $O/ab_c5_$TAG.log 2>&1 && \
timeout -k 10 200 python tools/batchbench.py c4 5 96 NEO_HIP_BATCH_VAR=2 NEO_HIP_BATCH_VAR=3 NEO_HIP_BATCH_VAR=4 NEO_HIP_BATCH_VAR=5 > $O/ab_c4_$TAG.log 2>&1
echo ab-exit=$?
