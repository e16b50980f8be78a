#!/bin/bash
# rocprofv3 kernel trace + stats of the c5 (or $1) bench; summary -> gpurun_out/prof_$2
set -o pipefail
W=${1:-c5}; TAG=${2:-r2}
R=$(pwd); O=$R/gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${W}_$TAG -o run -- python3 $R/bench.py --workload $W --steps 128 --warmup 10 --no-cpu-baseline --no-offline --no-parity --no-fft > $O/prof_${W}_$TAG.json 2> $O/prof_${W}_$TAG.err || { echo "rocprof rc=$?"; tail -5 $O/prof_${W}_$TAG.err; exit 1; }
find $O/prof_${W}_$TAG -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/prof_${W}_${TAG}_kernel_stats.csv
find $O/prof_${W}_$TAG -name "*kernel_trace.csv" | head -1 | xargs -I{} cp {} $O/prof_${W}_${TAG}_kernel_trace.csv
echo ok
