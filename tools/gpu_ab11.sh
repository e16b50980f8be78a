#!/bin/bash
# lookahead block step: parity, per-phase stamps (diagnostic build), streaming bench
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-ab11}
timeout -k 10 300 python -u -m pytest tests/test_upols_gpu.py -m gpu -x -q -k "ahead or batch" --timeout 120 --timeout-method thread > $O/pytest_$TAG.log 2>&1 && \
timeout -k 10 120 python tools/probebench.py c5 > $O/probe_c5_$TAG.log 2>&1 && \
timeout -k 10 200 python bench.py --no-cpu-baseline --no-offline > $O/bench_c5_$TAG.json 2>&1 && \
timeout -k 10 200 python bench.py --workload c4 --no-cpu-baseline --no-offline > $O/bench_c4_$TAG.json 2>&1
echo ab-exit=$?
