#!/bin/bash
# same-box A/B of tests/cpp/bench_group over the frame promises (mode 0 plain, 1 stable, 2 in place):
# the builds in LIBS (main = the tree's own, else tools/ab/<name>), alternating, REPS repetitions,
# channel counts CHS; then one run of each PROBES build (NEO_GROUP_PROBE: where a frame's host time
# goes) per mode, its stderr kept
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out; mkdir -p $O; T=${1:-gmode}
for rep in $(seq 1 ${REPS:-2}); do for C in ${CHS:-2048}; do for M in ${MODES:-0 1 2}; do for L in ${LIBS:-main gpfw2}; do
  if [ $L = main ]; then LP=""; else LP=$R/tools/ab/$L; fi
  NF=$([ $C -ge 1024 ] && echo 32 || echo 64)
  LD_LIBRARY_PATH=$LP timeout -k 10 120 tests/cpp/bin/bench_group $C $NF 512 480000 $M > $O/${T}_${L}_${C}_m${M}_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('$O/${T}_${L}_${C}_m${M}_$rep.json')); print('$L $C mode $M rep $rep', d['frame_p50_us'], d['frame_p99_us'])"
done; done; done; done
for L in ${PROBES:-}; do for M in ${MODES:-0 1 2}; do
  LD_LIBRARY_PATH=$R/tools/ab/$L timeout -k 10 120 tests/cpp/bin/bench_group 2048 32 512 480000 $M > $O/${T}_${L}_m${M}.json 2> $O/${T}_${L}_m${M}.err || exit 1
  echo "$L mode $M $(grep group_probe $O/${T}_${L}_m${M}.err)"
done; done
