#!/bin/bash
# direct-head block step: parity, then same-box A/B against the transform path
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-ab16}
timeout -k 10 300 python -u -m pytest tests/test_upols_gpu.py -m gpu -x -q -k "ahead or batch" --timeout 120 --timeout-method thread > $O/pytest_$TAG.log 2>&1 || exit $?
bash tools/gpu_ab15.sh ${TAG}a NEO_HIP_AHEAD_DIRECT=0 NEO_HIP_AHEAD_DIRECT=1 && \
W=c3 bash tools/gpu_ab15.sh ${TAG}b NEO_HIP_AHEAD_DIRECT=0 NEO_HIP_AHEAD_DIRECT=1 && \
W=c4 bash tools/gpu_ab15.sh ${TAG}c NEO_HIP_AHEAD_DIRECT=0 NEO_HIP_AHEAD_DIRECT=1
echo ab-exit=$?
