#!/bin/bash
# Same-box A/B of k_off_mac builds (tools/ab/<name>/libneo_hip.so; main = this tree's library):
# tools/off_bench.py at the workloads in WL, repetitions alternating.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out; T=${1:-offab}
for rep in 1 2 3; do for L in ${LIBS:-main pf1 pf2}; do
  if [ $L = main ]; then unset NEO_HIP_LIBRARY; else export NEO_HIP_LIBRARY=$PWD/tools/ab/$L/libneo_hip.so; fi
  for w in ${WL:-c5full c5}; do
    timeout -k 10 300 python tools/off_bench.py --workload $w > gpurun_out/${T}_${L}_${w}_$rep.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/${T}_${L}_${w}_$rep.json')); print('$L $w $rep', round(d['msamples_s']), round(d['mac_ms'],3))"
  done
done; done
unset NEO_HIP_LIBRARY
