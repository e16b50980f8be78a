#!/bin/bash
# Kernel timeline of a short bench run (tag $1, workload $2, step group $3, steps $4): rocprofv3
# kernel trace, marker kernels around the first timed region (NEO_BENCH_MARK)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
mkdir -p $O
T=${1:-tr}; W=${2:-c5}; G=${3:-4}; S=${4:-20}
cd /tmp && export TMPDIR=/tmp && export NEO_BENCH_MARK=1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace_${W}_g${G}_$T -o run -- python3 $R/bench.py --workload $W --steps $S --warmup 5 --step-group $G --no-cpu-baseline --no-fft --no-offline --no-host-io --no-parity > $O/trace_${W}_g${G}_$T.log 2>&1
