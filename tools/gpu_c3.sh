#!/bin/bash
# Latency mode check, tag $1: its GPU tests, then the C3 bench line (latency_mode leg).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-c3}
timeout -k 10 600 python -u -m pytest tests/test_persist_gpu.py -v --timeout 300 --timeout-method thread -m gpu \
  > $O/pytest_persist_$T.log 2>&1; rc=$?
tail -12 $O/pytest_persist_$T.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --workload c3 --steps 256 --no-cpu-baseline --no-fft > $O/bench_c3_$T.json 2> $O/bench_c3_$T.err || exit 1
python - $O/bench_c3_$T.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
lm = d["latency_mode"]
print("c3", round(d["value"], 1), "rt", round(d["latency"]["host_roundtrip_p50_us"], 1),
      "| latency mode", round(lm["value"], 1), "rt p50/p99", round(lm["host_roundtrip_p50_us"], 2),
      round(lm["host_roundtrip_p99_us"], 2), "gpu step p50/p99", lm["gpu_step_p50_us"], lm["gpu_step_p99_us"])
PY
