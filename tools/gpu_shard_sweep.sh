#!/bin/bash
# The per-GPU shapes of the driver's N-GPU strong-scaling run (bench.py --shard-of N: rank 0's
# channels of the 2048, measured alone on one GPU), the automatic code-path choices against the
# far window group's alternative; 128 steps, two repetitions, same box.
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out; T=${1:-shs}
for rep in $(seq 1 ${REPS:-2}); do for N in ${NS:-2 4 8}; do for FG in ${FGS:-0 2 3}; do
  timeout -k 10 300 python bench.py --shard-of $N --far-group $FG --steps ${STEPS:-128} --warmup 5 --no-cpu-baseline --no-fft \
    --no-host-io --no-offline --no-paced --no-parity > gpurun_out/${T}_n${N}_fg${FG}_s${STEPS:-128}_$rep.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('gpurun_out/${T}_n${N}_fg${FG}_s${STEPS:-128}_$rep.json')); c=d['config']; print('shard-of $N fg $FG steps ${STEPS:-128} rep $rep', c['channels_per_gpu'], c['far_group'], round(d['value']), round(d['ms_per_step']*1e3,2))"
done; done; done
