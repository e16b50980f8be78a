#!/bin/bash
# same-box A/B of diagnostic builds (tools/ab/<name>): 128-step bench lines at c5full, c5, c4
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out; T=${1:-ab5}
for rep in 1 2; do for L in ${LIBS:-main pad ord1 ord2 hpol}; do
  if [ $L = main ]; then unset NEO_HIP_LIBRARY; else export NEO_HIP_LIBRARY=$PWD/tools/ab/$L/libneo_hip.so; fi
  for w in ${WL:-c5full c5 c4}; do
    timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-128} --warmup 5 --no-cpu-baseline --no-fft --no-host-io --no-offline --no-paced --no-parity > gpurun_out/${T}_${L}_${w}_$rep.json 2>/dev/null || exit 1
    python -c "import json; d=json.load(open('gpurun_out/${T}_${L}_${w}_$rep.json')); print('$L $w $rep', round(d['value']), round(d['ms_per_step']*1e3,2))"
  done
done; done
unset NEO_HIP_LIBRARY
