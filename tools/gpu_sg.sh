#!/bin/bash
# Step groups A/B on one box (tag $1): the step-group parity tests, then the C5 / C4 / c5full /
# C3 lines at step_group 1, 2 and 4. Every GPU step has its own time limit; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-sg}
timeout -k 10 600 python -u -m pytest tests/test_upols_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread -rf \
  -k "step_group" > $O/pytest_sg_$T.log 2>&1; rc=$?; echo "pytest exit=$rc" >> $O/pytest_sg_$T.log
tail -3 $O/pytest_sg_$T.log
[ $rc -eq 0 ] || exit $rc
F="--no-cpu-baseline --no-fft --no-offline --no-host-io --no-parity"
for w in c5 c4 c3 c5full; do
  for g in 1 2 4; do
    st=128; [ $w = c5full ] && st=20
    timeout -k 10 300 python bench.py --workload $w --steps $st --warmup 5 --step-group $g $F > $O/sg_${w}_g${g}_$T.json 2> $O/sg_${w}_g${g}_$T.err || exit 1
  done
done
for f in $O/sg_*_$T.json; do python - "$f" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
l = d.get("latency") or {}
print(sys.argv[1].split("/")[-1], round(d["value"], 1), "ms/step", round(d["ms_per_step"], 4), "gpu", round(d.get("gpu_ms_per_step") or 0, 4),
      "rt_p50", round(l.get("host_roundtrip_p50_us") or 0, 1), "lat_p50", round((l.get("p50_ms") or 0) * 1e3, 1))
PY
done
