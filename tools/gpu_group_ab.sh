#!/bin/bash
# same-box A/B of tests/cpp/bench_group: the main build vs tools/ab/$ALT, alternating, two repetitions
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out; mkdir -p $O; T=${1:-gab}
for rep in 1 2; do for L in main ${ALT:-grpold}; do for C in 2048 256; do
  NF=$([ $C = 2048 ] && echo 16 || echo 64)
  if [ $L = main ]; then LP=""; else LP=$R/tools/ab/$L; fi
  LD_LIBRARY_PATH=$LP timeout -k 10 300 tests/cpp/bin/bench_group $C $NF > $O/${T}_${L}_${C}_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$O/${T}_${L}_${C}_$rep.json')); print('$L $C $rep', d['frame_p50_us'], d['frame_p99_us'])"
done; done; done
