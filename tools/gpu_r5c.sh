#!/bin/bash
# Round 5, first session: GPU tests after the latency-mode / setup fixes, then the bring-up and
# group-frame diagnostics (HIP call costs, bench_create, bench_group with the probe build).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-r5c}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest_gpu_$T.log 2>&1; rc=$?
echo "pytest exit=$rc" >> $O/pytest_gpu_$T.log; tail -3 $O/pytest_gpu_$T.log
[ $rc -lt 124 ] || exit $rc

timeout -k 10 300 tests/cpp/bin/bench_create 256 > $O/create_$T.json 2>&1 && \
LD_LIBRARY_PATH=$R/tools/ab/gprobe timeout -k 10 300 tests/cpp/bin/bench_group 256 64 > $O/group256_$T.json 2> $O/group256_$T.err && \
LD_LIBRARY_PATH=$R/tools/ab/gprobe timeout -k 10 300 tests/cpp/bin/bench_group 2048 16 > $O/group2048_$T.json 2> $O/group2048_$T.err
echo "diag exit=$?"
timeout -k 10 300 tests/cpp/bin/bench_group 256 64 > $O/group256m_$T.json 2> $O/group256m_$T.err && \
timeout -k 10 300 tests/cpp/bin/bench_group 2048 16 > $O/group2048m_$T.json 2> $O/group2048m_$T.err
echo "main exit=$?"
