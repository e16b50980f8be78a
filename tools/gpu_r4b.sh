#!/bin/bash
# Round 4, second evidence call: the new GPU tests (paced, latency mode, groups, C++), the
# profiles / PMC / calibration part of the round script, the group frame benches.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-r4}
timeout -k 10 900 python -u -m pytest tests/test_paced_gpu.py tests/test_persist_gpu.py tests/test_group_gpu.py \
  tests/test_cpp_api.py -v --timeout 300 --timeout-method thread -m gpu > $O/pytest_new_$T.log 2>&1; rc=$?
tail -4 $O/pytest_new_$T.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 tests/cpp/bin/bench_group 256 64 > $O/group256_$T.json && \
timeout -k 10 600 tests/cpp/bin/bench_group 2048 16 > $O/group2048_$T.json && \
PART=2 bash tools/gpu_round.sh $T
