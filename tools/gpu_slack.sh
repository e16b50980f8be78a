#!/bin/bash
# A/B of a library build under tools/ab/$V: its streaming-level GPU tests first (the library
# the Python tests load: NEO_HIP_LIBRARY), then interleaved bench lines against the main build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
V=${V:-slack2}
T=${1:-slk}
NEO_HIP_LIBRARY=$R/tools/ab/$V/libneo_hip.so timeout -k 10 900 python -u -m pytest tests/test_upols_gpu.py \
  tests/test_paced_gpu.py tests/test_group_gpu.py -x -q -m gpu --timeout 120 --timeout-method thread $DESEL \
  > $O/pytest_${V}_$T.log 2>&1; rc=$?
tail -4 $O/pytest_${V}_$T.log
[ $rc = 0 ] || exit $rc
LIBS="main $V" REPS=${REPS:-3} bash tools/gpu_abn.sh $T
