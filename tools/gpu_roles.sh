#!/bin/bash
# time the slices kernel's roles apart (tools/build_roles.sh builds): c5 bench per variant
set -o pipefail
O=gpurun_out
W=${W:-c5}
for R in "$@"; do
  if [ "$R" = full ]; then L=""; else L=$(pwd)/tools/ab/$R/libneo_hip.so; fi
  NEO_HIP_LIBRARY=$L timeout -k 10 200 python bench.py --workload $W --steps 64 --warmup 5 --no-cpu-baseline --no-offline --no-parity --no-fft > $O/roles_$R.json 2> $O/roles_$R.err || { echo "variant $R rc=$?"; tail -5 $O/roles_$R.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/roles_$R.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$R', 'ms/step %.4f'%d['ms_per_step'], ' '.join('%s %.4f'%(k['kernel'].split()[1], k['ms_per_step']) for k in r.get('kernels',[])))"
done
