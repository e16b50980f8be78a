#!/bin/bash
# C4 (two-level lookahead on by default there) bench + kernel stats, and the default C5 bench.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; cd "$R"; O=$R/gpurun_out; mkdir -p $O; TAG=${1:-r1j}
timeout -k 10 300 python bench.py --workload c4 --steps 128 --no-cpu-baseline > $O/bench_c4_$TAG.json 2> $O/bench_c4_$TAG.err && \
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench_c5_$TAG.json 2> $O/bench_c5_$TAG.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4_$TAG -o run -- python3 $R/bench.py --workload c4 --steps 128 --no-cpu-baseline --no-offline > $O/prof_c4_$TAG.log 2>&1
echo "c4far exit=$?"
