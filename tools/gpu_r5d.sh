#!/bin/bash
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out; mkdir -p $O; T=${1:-r5d}
timeout -k 10 600 python -u -m pytest tests/test_paced_gpu.py tests/test_persist_gpu.py tests/test_bringup_gpu.py -q -rf --timeout 300 --timeout-method thread > $O/pytest_$T.log 2>&1; rc=$?
tail -3 $O/pytest_$T.log; [ $rc -lt 124 ] || exit $rc
LD_LIBRARY_PATH=$R/tools/ab/gprobe timeout -k 10 300 tests/cpp/bin/bench_group 2048 16 > $O/group2048_$T.json 2> $O/group2048_$T.err && \
timeout -k 10 600 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-fft --no-host-io --no-offline > $O/bench_c5full_$T.json 2> $O/bench_c5full_$T.err && \
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --no-fft --no-host-io --no-offline > $O/bench_c5_$T.json 2> $O/bench_c5_$T.err
echo "exit=$?"
python - <<'PY'
import json
for w in ("c5full","c5"):
    try:
        d=json.load(open(f"gpurun_out/bench_{w}_r5d.json"))
        l=d["latency"]; print(w, d["value"], "rt", l["host_roundtrip_p50_us"], l["host_roundtrip_p99_us"], "paced", {k: l["paced"][k] for k in ("host_roundtrip_p50_us","host_roundtrip_p99_us","value")}, "paced2", {k: l["paced_two_pieces"][k] for k in ("host_roundtrip_p50_us","host_roundtrip_p99_us","value")})
    except Exception as e: print(w, e)
PY
