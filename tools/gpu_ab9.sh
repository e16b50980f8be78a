#!/bin/bash
# overlap of a batched MAC pass (stream a) with lookahead block steps (stream b)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-ab9}
( timeout -k 10 120 python tools/overlapbench.py c5 && \
  timeout -k 10 120 python tools/overlapbench.py c5 NEO_HIP_BATCH_LDS=90000 && \
  timeout -k 10 120 python tools/overlapbench.py c4 NEO_HIP_BATCH_LDS=90000 ) > $O/overlap_$TAG.log 2>&1
echo ab-exit=$?
