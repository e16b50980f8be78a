#!/bin/bash
# rocprofv3 kernel trace of the c5 bench for role-masked builds (tools/build_roles.sh):
# median / mean duration of the step kernel over its steady-state launches (full grids)
set -o pipefail
R0=$(pwd); O=$R0/gpurun_out
W=${W:-c5}
cd /tmp && export TMPDIR=/tmp
for R in "$@"; do
  if [ "$R" = full ]; then L=""; else L=$R0/tools/ab/$R/libneo_hip.so; fi
  NEO_HIP_LIBRARY=$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/profr_$R -o run -- python3 $R0/bench.py --workload $W --steps 64 --warmup 5 --no-cpu-baseline --no-offline --no-parity --no-fft > $O/profr_$R.log 2>&1 || { echo "prof $R failed"; tail -3 $O/profr_$R.log; exit 1; }
  f=$(find $O/profr_$R -name "*kernel_trace.csv" | head -1)
  python3 - "$f" "$R" <<'PY'
import csv, statistics, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'k_lvl_step' in r['Kernel_Name']]
g = collections.Counter(int(r['Grid_Size_X']) for r in rows)
grid = g.most_common(1)[0][0]
d = [(int(r['End_Timestamp']) - int(r['Start_Timestamp'])) / 1e3 for r in rows if int(r['Grid_Size_X']) == grid]
print(sys.argv[2], 'k_lvl_step grid %d x %s: n %d median %.2f us mean %.2f min %.2f' % (
    grid // int(rows[0]['Workgroup_Size_X']), rows[0]['Workgroup_Size_X'], len(d), statistics.median(d), statistics.mean(d), min(d)))
PY
done
