#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out; mkdir -p $O; T=${1:-r5g}
timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest_gpu_$T.log 2>&1; rc=$?
tail -3 $O/pytest_gpu_$T.log; [ $rc -lt 124 ] || exit $rc
timeout -k 10 300 tests/cpp/bin/bench_create 512 > $O/create_$T.json 2>&1 && \
timeout -k 10 300 tests/cpp/bin/bench_group 2048 16 > $O/group2048_$T.json 2> $O/group2048_$T.err && \
timeout -k 10 300 tests/cpp/bin/bench_group 2048 16 > $O/group2048b_$T.json 2> $O/group2048b_$T.err && \
timeout -k 10 300 tests/cpp/bin/bench_group 256 64 > $O/group256_$T.json 2> $O/group256_$T.err
echo "exit=$?"
cat $O/create_$T.json
for f in group2048 group2048b group256; do python -c "import json; d=json.load(open('$O/${f}_$T.json')); print('$f', d['frame_p50_us'], d['frame_p99_us'], d['setup_s'], d['shared_scratch']['switch_frame_us'])"; done
