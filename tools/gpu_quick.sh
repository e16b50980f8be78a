#!/bin/bash
# Quick check after a step-kernel change, tag $1: the level / far GPU parity tests, then the
# headline bench line (driver flags) and the c5 / c4 lines. Stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-q}
timeout -k 10 600 python -u -m pytest tests/test_upols_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "level or far or full_size or ahead or multi or before_any" > $O/pytest_quick_$T.log 2>&1 && \
echo tests-ok && \
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c5full_$T.json 2> $O/bench_c5full_$T.err && \
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --no-fft > $O/bench_c5_$T.json 2> $O/bench_c5_$T.err && \
timeout -k 10 300 python bench.py --workload c4 --steps 128 --no-cpu-baseline --no-fft > $O/bench_c4_$T.json 2> $O/bench_c4_$T.err && \
echo benches-ok
st=$?; tail -3 $O/pytest_quick_$T.log; exit $st
