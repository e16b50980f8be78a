#!/bin/bash
# Group checks: the group GPU tests, the C++ group test, the frame benches at 256 / 2048 members.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-grp}
timeout -k 10 600 python -u -m pytest tests/test_group_gpu.py tests/test_cpp_api.py -v --timeout 300 \
  --timeout-method thread -m gpu > $O/pytest_grp_$T.log 2>&1; rc=$?
tail -12 $O/pytest_grp_$T.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tests/cpp/bin/bench_group 256 64 > $O/group256_$T.json && \
timeout -k 10 600 tests/cpp/bin/bench_group 2048 16 > $O/group2048_$T.json && cat $O/group256_$T.json $O/group2048_$T.json
