#!/bin/bash
# PMC passes over the c5 bench (one rocprofv3 run per counter set): per-launch averages of the
# steady-state step kernel (its most common grid) -> gpurun_out/pmc_<tag>_<n>.txt
set -o pipefail
R0=$(pwd); O=$R0/gpurun_out
W=${W:-c5}; TAG=${TAG:-step}; LIB=${LIB:-}
cd /tmp && export TMPDIR=/tmp
n=0
for SET in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM" \
           "GRBM_GUI_ACTIVE TA_BUSY_avr"; do
  n=$((n+1))
  NEO_HIP_LIBRARY=$LIB timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d $O/pmc_${TAG}_$n -o run -- python3 $R0/bench.py --workload $W --steps 32 --warmup 2 --no-cpu-baseline --no-offline --no-parity --no-fft > $O/pmc_${TAG}_$n.log 2>&1 || { echo "pmc pass $n ($SET) failed"; tail -3 $O/pmc_${TAG}_$n.log; continue; }
  f=$(find $O/pmc_${TAG}_$n -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$SET" <<'PY' | tee $O/pmc_${TAG}_$n.txt
import csv, sys, collections
rows = [r for r in csv.DictReader(open(sys.argv[1])) if 'k_lvl_step' in r['Kernel_Name']]
g = collections.Counter(r['Grid_Size'] for r in rows).most_common(1)[0][0]
by = collections.defaultdict(list)
for r in rows:
    if r['Grid_Size'] == g:
        by[r['Counter_Name']].append(float(r['Counter_Value']))
for k, v in sorted(by.items()):
    print('%-22s n %5d  mean %.4g' % (k, len(v), sum(v) / len(v)))
PY
rm -rf $O/pmc_${TAG}_$n
done
