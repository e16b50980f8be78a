#!/bin/bash
# same-box A/B of the host-buffer boundary (bench.py --host-io) between the main build and tools/ab/$ALT
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out; T=${1:-hio}
for rep in 1 2; do for L in main ${ALT:-ownst}; do
  if [ $L = main ]; then unset NEO_HIP_LIBRARY; else export NEO_HIP_LIBRARY=$PWD/tools/ab/$L/libneo_hip.so; fi
  for w in c5full c5; do
    timeout -k 10 300 python bench.py --workload $w --host-io --steps 200 > gpurun_out/${T}_${L}_${w}_$rep.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/${T}_${L}_${w}_$rep.json')); h=d['host_io']; print('$L $w $rep', {k:(round(v['p50_us'],1), round(v['p99_us'],1)) for k,v in h.items() if isinstance(v,dict) and 'p50_us' in v})"
  done
done; done
