#!/bin/bash
# PMC FETCH_SIZE / WRITE_SIZE of k_lvl_step for role-masked builds (separate passes)
set -o pipefail
R0=$(pwd); O=$R0/gpurun_out
cd /tmp && export TMPDIR=/tmp
for R in "$@"; do
  if [ "$R" = full ]; then L=""; else L=$R0/tools/ab/$R/libneo_hip.so; fi
  for C in FETCH_SIZE WRITE_SIZE; do
    NEO_HIP_LIBRARY=$L timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmcr_${R}_$C -o run -- python3 $R0/bench.py --steps 32 --warmup 2 --no-cpu-baseline --no-offline --no-parity --no-fft > $O/pmcr_${R}_$C.log 2>&1 || { echo "pmc $R $C failed"; tail -3 $O/pmcr_${R}_$C.log; exit 1; }
    f=$(find $O/pmcr_${R}_$C -name "*counter_collection.csv" | head -1)
    python3 -c "
import csv
v=[float(r['Counter_Value']) for r in csv.DictReader(open('$f')) if 'k_lvl_step' in r['Kernel_Name']]
print('$R $C step %.1f MB (n=%d)' % (sum(v)/len(v)*1024/1e6, len(v)))"
  done
done
