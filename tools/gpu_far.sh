#!/bin/bash
# Two-level lookahead (NEO_HIP_FAR): parity tests, then same-box benches with it off and on.
# Stops at any GPU fault / abort / timeout (exit codes other than 0 and pytest's 1).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out; mkdir -p $O; TAG=${1:-far}
ok() { [ $1 -eq 0 ] || [ $1 -eq 1 ]; }
timeout -k 10 400 python -u -m pytest tests/test_upols_gpu.py -m gpu -x -q -k "far or ahead" --timeout 120 --timeout-method thread > $O/far_pytest_$TAG.log 2>&1; rc=$?; echo "pytest rc=$rc" >> $O/far_pytest_$TAG.log
ok $rc || exit $rc
for w in c5 c4; do
  timeout -k 10 200 python bench.py --workload $w --steps 128 --no-cpu-baseline --no-offline > $O/far_off_${w}_$TAG.json 2> $O/far_off_${w}_$TAG.err || exit $?
  NEO_HIP_FAR=1 timeout -k 10 200 python bench.py --workload $w --steps 128 --no-cpu-baseline --no-offline > $O/far_on_${w}_$TAG.json 2> $O/far_on_${w}_$TAG.err || exit $?
done
cd /tmp && export TMPDIR=/tmp && export NEO_HIP_FAR=1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/far_prof_c5_$TAG -o run -- python3 $R/bench.py --steps 128 --warmup 5 --no-cpu-baseline --no-offline > $O/far_prof_c5_$TAG.log 2>&1
echo "far exit=$?"
