#!/bin/bash
# same-box A/B of the default build against tools/ab/<variant>/libneo_hip.so (tag $1, variant $2):
# C5 / C4 / c5full bench lines at the driver's 20 steps and C5 / C4 at 128, alternating builds
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
T=${1:-lab}; V=$2; shift 2
F="--no-cpu-baseline --no-fft --no-offline --no-host-io --no-parity --warmup 5 $*"
for ws in c5:20 c4:20 c5full:20 c5:128 c4:128; do
  for b in base $V; do
    w=${ws%%:*}; st=${ws##*:}
    if [ $b = base ]; then L=""; else L=$R/tools/ab/$V/libneo_hip.so; fi
    NEO_HIP_LIBRARY=$L timeout -k 10 300 python bench.py --workload $w --steps $st $F > $O/lab_${w}_s${st}_${b}_$T.json 2> $O/lab_${w}_s${st}_${b}_$T.err || exit 1
    python3 - $O/lab_${w}_s${st}_${b}_$T.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; l = d["latency"]
ks = " ".join("%s %.2f" % (k["kernel"], k.get("ms_per_launch", k.get("ms_per_step", 0)) * 1e3) for k in r.get("kernels", []))
print(sys.argv[1].split("/")[-1], round(d["value"], 1), "us/step %.2f" % (d["ms_per_step"] * 1e3), ks, "rt_p50 %.1f" % l["host_roundtrip_p50_us"])
PY
  done
done
