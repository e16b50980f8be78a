#!/bin/bash
# PMC passes (one counter per rocprofv3 run, no tracing) over the c5 / c4 / c2 bench runs: the
# streaming step kernel (k_lvl_step), the plain step (k_upols_step), the batched pass
# (k_batch_mac, the offline leg) and the 4096-point FFT (k_c2c_lds). tools/pmc_summary.py <tag>
# turns them into profiles/<tag>_pmc_*.json.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-r2}
cd /tmp && export TMPDIR=/tmp
for W in c5full c5 c4 c2; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${W}_${C}_$TAG -o run -- \
      python3 $R/bench.py --workload $W --steps 32 --warmup 2 --no-cpu-baseline --no-parity --no-fft --no-paced --no-host-io \
      > $O/pmc_${W}_${C}_$TAG.log 2>&1 || exit $?
  done
done
echo pmc-ok
