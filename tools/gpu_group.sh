#!/bin/bash
# The plugin boundary (convolver groups): their GPU tests, then tests/cpp/bench_group at 2048 and 256
# channels with the probe build (tools/ab/gprobe: SRC=upols_group tools/build_variant.sh gprobe
# -DNEO_GROUP_PROBE; the per-phase medians on stderr) and with the main build.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out; mkdir -p $O; T=${1:-grp}
timeout -k 10 600 python -u -m pytest tests/test_group_gpu.py tests/test_cpp_api.py -q -rf --timeout 300 --timeout-method thread > $O/pytest_$T.log 2>&1; rc=$?
tail -3 $O/pytest_$T.log; [ $rc -lt 124 ] || exit $rc
LD_LIBRARY_PATH=$R/tools/ab/gprobe timeout -k 10 300 tests/cpp/bin/bench_group 2048 16 > $O/group2048p_$T.json 2> $O/group2048p_$T.err && \
LD_LIBRARY_PATH=$R/tools/ab/gprobe timeout -k 10 300 tests/cpp/bin/bench_group 256 64 > $O/group256p_$T.json 2> $O/group256p_$T.err && \
timeout -k 10 300 tests/cpp/bin/bench_group 2048 16 > $O/group2048_$T.json 2> $O/group2048_$T.err && \
timeout -k 10 300 tests/cpp/bin/bench_group 256 64 > $O/group256_$T.json 2> $O/group256_$T.err
echo "exit=$?"
for f in group2048p group256p group2048 group256; do grep -v amdgpu $O/${f}_$T.err; python -c "import json; d=json.load(open('$O/${f}_$T.json')); print('$f', d['frame_p50_us'], d['frame_p99_us'], d['setup_s'], d['shared_scratch']['switch_frame_us'])"; done
