#!/bin/bash
# Per-workgroup timelines (tools/timeline.py, NEO_TIMELINE build tools/ab/tl from
# tools/build_timeline.sh) of the step groups' slices launch (part 2) and block launch (part 1)
# for the workloads in $WL.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out; T=${1:-tl}
for w in ${WL:-c4 c5}; do for p in 2 1; do
  echo "== $w part $p"
  NEO_HIP_LIBRARY=$PWD/tools/ab/tl/libneo_hip.so timeout -k 10 240 python tools/timeline.py --workload $w --steps 64 --part $p \
    --json gpurun_out/${T}_${w}_p$p.json 2> gpurun_out/${T}_${w}_p$p.err || { tail -5 gpurun_out/${T}_${w}_p$p.err; exit 1; }
done; done
