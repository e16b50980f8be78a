#!/bin/bash
# Timelines of the step kernel (tools/timeline.py) for the workloads in $WL, tag $1, with the
# timeline builds under tools/ab/ given in $LIBS (default "tl").
set -o pipefail
R0=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R0"
T=${1:-tl}
for L in ${LIBS:-tl}; do
  for w in ${WL:-c4 c5 c5full}; do
    echo "== $L $w"
    NEO_HIP_LIBRARY=$R0/tools/ab/$L/libneo_hip.so timeout -k 10 240 python tools/timeline.py --workload $w --steps 200 \
      --json gpurun_out/timeline_${L}_${w}_$T.json 2> gpurun_out/timeline_${L}_${w}_$T.err || { tail -5 gpurun_out/timeline_${L}_${w}_$T.err; exit 1; }
  done
done
