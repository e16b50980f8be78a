#!/bin/bash
# Round 4 check: the new GPU tests (latency mode, groups, C++ groups), then (LIBS set) a
# same-box A/B of builds.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-r4a}
timeout -k 10 900 python -u -m pytest tests/test_persist_gpu.py tests/test_group_gpu.py tests/test_cpp_api.py -v \
  --timeout 300 --timeout-method thread -m gpu > $O/pytest_new_$T.log 2>&1; rc=$?
tail -25 $O/pytest_new_$T.log
[ $rc -lt 124 ] || exit $rc  # crash or time limit: nothing more on the GPU
[ -n "$LIBS" ] || exit $rc
bash tools/gpu_abn.sh $T
