#!/bin/bash
# kernel trace of overlapbench (B-only block steps: durations and gaps)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O
TAG=${1:-ab10}
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace_ov_$TAG -o run -- python3 $R/tools/overlapbench.py c5 > $O/trace_ov_$TAG.log 2>&1
echo ab-exit=$?
