#!/bin/bash
# Kernel timeline of a short bench run (tag $1, workload $2, step group $3): rocprofv3 kernel trace
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
T=${1:-tr}; W=${2:-c5}; G=${3:-4}
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_${W}_g${G}_$T -o run -- python3 $R/bench.py --workload $W --steps 64 --warmup 5 --step-group $G --no-cpu-baseline --no-fft --no-offline --no-host-io --no-parity > $O/trace_${W}_g${G}_$T.log 2>&1
