#!/bin/bash
# rocprofv3 kernel stats of the c5 bench for role-masked builds (tools/build_roles.sh)
set -o pipefail
R0=$(pwd); O=$R0/gpurun_out
cd /tmp && export TMPDIR=/tmp
for R in "$@"; do
  if [ "$R" = full ]; then L=""; else L=$R0/tools/ab/$R/libneo_hip.so; fi
  NEO_HIP_LIBRARY=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/profr_$R -o run -- python3 $R0/bench.py --steps 64 --warmup 5 --no-cpu-baseline --no-offline --no-parity --no-fft > $O/profr_$R.log 2>&1 || { echo "prof $R failed"; tail -3 $O/profr_$R.log; exit 1; }
  f=$(find $O/profr_$R -name "*kernel_stats.csv" | head -1)
  python3 -c "
import csv
for r in csv.DictReader(open('$f')):
    if 'lvl' in r['Name'] or 'k_upols_step' in r['Name']: print('$R', r['Name'][:40], r['Calls'], '%.2f us'%(float(r['AverageNs'])/1e3), 'min %.2f'%(float(r['MinNs'])/1e3))"
done
