#!/bin/bash
# same-box A/B of lookahead options in the streaming bench (alternating runs)
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}; O=$R/gpurun_out; mkdir -p $O; cd $R
TAG=${1:-ab15}; shift
W=${W:-c5}
for rep in 1 2; do
  for SPEC in "$@"; do
    env $SPEC timeout -k 10 200 python bench.py --workload $W --no-cpu-baseline --no-offline > $O/b_${TAG}.json 2>&1 || exit $?
    python -c "import json; d=json.loads(open('$O/b_${TAG}.json').read().splitlines()[-1]); print('$SPEC', round(d['value'],1), round(d['ms_per_step']*1e3,2), 'us/step, pass', round(d['roofline']['kernel_avg_ms'],4))" >> $O/ab_$TAG.log
  done
done
echo ab-exit=$?
