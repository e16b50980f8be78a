#!/bin/bash
# step-group sweep (bench.py --step-group) at the 256-channel shapes, two repetitions, 128 and 20 steps
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out; T=${1:-sgs}
for rep in 1 2; do for w in c4 c5; do for G in 4 2 8; do for S in 128 20; do
  timeout -k 10 300 python bench.py --workload $w --steps $S --warmup 5 --step-group $G --no-cpu-baseline --no-fft --no-host-io --no-offline --no-paced --no-parity > gpurun_out/${T}_${w}_g${G}_s${S}_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/${T}_${w}_g${G}_s${S}_$rep.json')); print('$w G=$G steps=$S rep $rep', round(d['value']), round(d['ms_per_step']*1e3,2))"
done; done; done; done
