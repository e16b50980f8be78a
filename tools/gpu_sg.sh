#!/bin/bash
# Same-box A/B of step group sizes ($GS) at $WL: bench lines at the driver's 20 steps (each with
# its 128-step steady sub-line), $REPS repetitions, tag $1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-sg}
for rep in $(seq 1 ${REPS:-2}); do
  for W in ${WL:-c5full c5 c4}; do
    for G in ${GS:-4 8}; do
      timeout -k 10 300 python bench.py --workload $W --steps 20 --warmup 5 --step-group $G --no-cpu-baseline \
        --no-fft --no-offline --no-parity --no-host-io --no-paced > $O/sg_${T}_${W}_${G}_$rep.json 2> $O/sg_${T}_${W}_${G}_$rep.err || exit 1
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'G', sys.argv[3], round(d['value'],1), 'steady', round(d['steady']['value'],1))" $O/sg_${T}_${W}_${G}_$rep.json $W $G
    done
  done
done
