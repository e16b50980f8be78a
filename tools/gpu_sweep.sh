#!/bin/bash
# Option sweep on one box (tag $1): bench lines for every "workload:steps:far_group:step_group[:far_phase2[:far_level]]"
# item of $ITEMS, $REPS interleaved repetitions; one summary line per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-sweep}
F="--no-cpu-baseline --no-fft --no-offline --no-host-io --no-parity --warmup 5"
for rep in $(seq 1 ${REPS:-2}); do
  for it in $ITEMS; do
    IFS=: read -r w st fg sg f2 fl <<< "$it"; f2=${f2:-0}; fl=${fl:--1}
    f=$O/sw_${T}_${w}_s${st}_k${fg}_g${sg}_f${f2}_l${fl}_$rep.json
    NEO_HIP_LIBRARY=${LIB:-} timeout -k 10 300 python bench.py --workload $w --steps $st --far-group $fg --step-group $sg --far-phase2 $f2 --far-level $fl $F \
      > $f 2> ${f%.json}.err || { tail -3 ${f%.json}.err; exit 1; }
    python3 - $f "$it" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
r = d["roofline"]; l = d["latency"]
ks = " ".join("%s %.2f" % (k["kernel"][:16], k.get("ms_per_launch", k.get("ms_per_step", 0)) * 1e3) for k in r.get("kernels", []))
print(sys.argv[2], round(d["value"], 1), "us/step %.2f gpu %.2f" % (d["ms_per_step"] * 1e3, (d["gpu_ms_per_step"] or 0) * 1e3),
      ks, "rt_p50 %.1f" % l["host_roundtrip_p50_us"])
PY
  done
done
