#!/bin/bash
# PMC passes (counters only, one counter group per run) for the MAC and FFT kernels.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-r1}
cd /tmp && export TMPDIR=/tmp
# streaming runs: the plain step (k_upols_step) and the lookahead window pass (k_batch_mac)
for W in c5 c4 c2; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${W}_${C}_$TAG -o run -- \
      python3 $R/bench.py --workload $W --steps 64 --warmup 1 --no-cpu-baseline --no-offline \
      > $O/pmc_${W}_${C}_$TAG.log 2>&1 || exit $?
  done
done
# offline (batched) pass only: no lookahead, whole passes of 32 blocks
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $C --output-format csv -d $O/pmc_c5o_${C}_$TAG -o run -- \
    python3 $R/bench.py --workload c5 --steps 64 --warmup 1 --no-cpu-baseline --no-ahead \
    > $O/pmc_c5o_${C}_$TAG.log 2>&1 || exit $?
done
echo pmc-ok
