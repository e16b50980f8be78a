#!/bin/bash
# step-group checks after a change (tag $1): the step-group parity tests, then C5 / C4 / c5full at
# the driver's 20 steps and C5 / C4 at 128
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
T=${1:-sg2}
timeout -k 10 600 python -u -m pytest tests/test_upols_gpu.py tests/test_group_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -rf \
  -k "step_group or full_size or group" > $O/pytest_sg2_$T.log 2>&1; rc=$?; echo "pytest exit=$rc" >> $O/pytest_sg2_$T.log
tail -2 $O/pytest_sg2_$T.log
[ $rc -eq 0 ] || exit $rc
F="--no-cpu-baseline --no-fft --no-offline --no-host-io --no-parity --warmup 5"
for ws in c5:20 c4:20 c5full:20 c5:128 c4:128; do
  w=${ws%%:*}; st=${ws##*:}
  timeout -k 10 300 python bench.py --workload $w --steps $st $F > $O/sg2_${w}_s${st}_$T.json 2> $O/sg2_${w}_s${st}_$T.err || exit 1
  python3 - $O/sg2_${w}_s${st}_$T.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; l = d["latency"]
ks = " ".join("%s %.2f" % (k["kernel"], k.get("ms_per_launch", k.get("ms_per_step", 0)) * 1e3) for k in r.get("kernels", []))
print(sys.argv[1].split("/")[-1], round(d["value"], 1), "us/step %.2f" % (d["ms_per_step"] * 1e3), ks, "rt_p50 %.1f" % l["host_roundtrip_p50_us"])
PY
done
