#!/bin/bash
# Same-box A/B of whole trees (the round-4 and round-5 final trees as git worktrees under tools/ab,
# built in place, against this tree): c5full bench lines at the driver's 20 steps and the 128-step
# full far window, repetitions alternating. TREES="head r5tree r4tree" by default.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R; mkdir -p gpurun_out; T=${1:-abt}
for rep in 1 2 3; do for tr in ${TREES:-head r5tree r4tree}; do
  D=$R; [ $tr = head ] || D=$R/tools/ab/$tr
  for st in 20 128; do
    (cd $D && timeout -k 10 300 python bench.py --workload ${WL:-c5full} --steps $st --warmup 5 --no-cpu-baseline --no-fft \
      --no-host-io --no-offline --no-paced --no-parity) > gpurun_out/${T}_${tr}_${st}_$rep.json 2> gpurun_out/${T}_${tr}_${st}_$rep.err || exit 1
    python -c "import json; d=json.load(open('gpurun_out/${T}_${tr}_${st}_$rep.json')); print('$tr $st $rep', round(d['value']), round(d['ms_per_step']*1e3,2))"
  done
done; done
