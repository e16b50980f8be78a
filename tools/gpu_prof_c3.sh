#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_$1 -o run -- python3 $R/bench.py --workload c3 --steps 200 --no-cpu-baseline > $O/prof_c3_$1.log 2>&1
