#!/bin/bash
# Same-box A/B of the group path: bench_group with the current library and with tools/ab/grpold.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
for rep in 1 2; do
  for L in new old; do
    if [ $L = old ]; then export LD_LIBRARY_PATH=$R/tools/ab/grpold; else unset LD_LIBRARY_PATH; fi
    timeout -k 10 300 tests/cpp/bin/bench_group 256 48 > $O/gab_256_${L}_$rep.json || exit 1
    timeout -k 10 300 tests/cpp/bin/bench_group 2048 8 > $O/gab_2048_${L}_$rep.json || exit 1
    python3 -c "import json,sys
for c in (256, 2048):
    d = json.load(open('$O/gab_%d_${L}_$rep.json' % c))
    print(c, '$L', d['frame_p50_us'], d['frame_mean_us'], d['shared_scratch']['per_channel_block_p50_us'], d['shared_scratch']['switch_frame_us'])"
  done
done
