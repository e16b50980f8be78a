#!/bin/bash
# far window group A/B (tag $1) at the default step group: C5 / C4 with K = 2 / 3 / 4
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
T=${1:-kab}
F="--no-cpu-baseline --no-fft --no-offline --no-host-io --no-parity"
for w in c5 c4; do
  for k in 2 3 4; do
    timeout -k 10 300 python bench.py --workload $w --steps 128 --warmup 5 --far-group $k $F > $O/kab_${w}_k${k}_$T.json 2> $O/kab_${w}_k${k}_$T.err || exit 1
  done
done
for f in $O/kab_*_$T.json; do python - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(sys.argv[1].split("/")[-1], round(d["value"], 1), "ms/step", round(d["ms_per_step"], 4))
PY
done
