#!/bin/bash
# Bench-flag experiments on one box, tag $1: the C3 line (latency mode leg), then step group 2 vs
# 4 at the driver's 20 steps and at 128 (value, host round trip p50 / p99).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-exp}
timeout -k 10 300 python bench.py --workload c3 --steps 256 --no-cpu-baseline --no-fft > $O/bench_c3_$T.json 2> $O/bench_c3_$T.err || exit 1
python - $O/bench_c3_$T.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print("c3", round(d["value"], 1), "rt", round(d["latency"]["host_roundtrip_p50_us"], 1), "lm", json.dumps(d["latency_mode"]))
PY
for W in c5 c4 c5full; do
  for SG in 4 2; do
    for S in 20 128; do
      timeout -k 10 300 python bench.py --workload $W --steps $S --warmup 5 --step-group $SG --no-cpu-baseline --no-fft \
        --no-offline --no-parity --no-host-io > $O/exp_${T}_${W}_sg${SG}_s$S.json 2> $O/exp_${T}_${W}_sg${SG}_s$S.err || exit 1
      python - $O/exp_${T}_${W}_sg${SG}_s$S.json $W $SG $S <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
l = d["latency"]
print(sys.argv[2], "sg", sys.argv[3], "steps", sys.argv[4], round(d["value"], 1), "us", round(d["ms_per_step"] * 1e3, 2),
      "rt p50/p99", round(l["host_roundtrip_p50_us"], 1), round(l["host_roundtrip_p99_us"], 1),
      "steady", round(d["steady"]["value"], 1), "ir", json.dumps(d["ir_change"]))
PY
    done
  done
done
