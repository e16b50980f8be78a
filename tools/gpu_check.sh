#!/bin/bash
# One GPU call after a change, tag $1: the whole -m gpu suite, smoke, the headline bench line
# at the driver's flags, the C5 shard and C4 lines, and a 2-rank torch.distributed.run
# rehearsal of the strong-scaling headline (both ranks on the box's one GPU: 1024 channels
# each). Every GPU step has its own time limit; stops at the first failure.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-chk}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -rf \
  > $O/pytest_gpu_$T.log 2>&1; rc=$?; echo "pytest exit=$rc" >> $O/pytest_gpu_$T.log
tail -3 $O/pytest_gpu_$T.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$T.log 2>&1 && \
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c5full_$T.json 2> $O/bench_c5full_$T.err && \
timeout -k 10 300 python bench.py --workload c5 --steps 20 --warmup 5 --no-cpu-baseline --no-fft > $O/bench_c5_$T.json 2> $O/bench_c5_$T.err && \
timeout -k 10 300 python bench.py --workload c4 --steps 128 --no-cpu-baseline --no-fft > $O/bench_c4_$T.json 2> $O/bench_c4_$T.err && \
timeout -k 10 300 python bench.py --workload c3 --steps 256 --no-cpu-baseline --no-fft > $O/bench_c3_$T.json 2> $O/bench_c3_$T.err && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 20 --warmup 5 --no-fft --no-host-io > $O/bench_c5full_n2_$T.json 2> $O/bench_c5full_n2_$T.err && \
echo benches-ok
st=$?
for f in $O/bench_*_$T.json; do python - "$f" <<'PY'
import json, sys
try:
    d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
    r = d.get("roofline", {})
    print(sys.argv[1].split("/")[-1], round(d["value"], 1), "ms/step", round(d["ms_per_step"], 4), "frac", round(r.get("frac") or 0, 3),
          "parity", (d.get("parity") or {}).get("parity_err"), "rt_p50", (d.get("latency") or {}).get("host_roundtrip_p50_us"))
except Exception as e:
    print(sys.argv[1], "unreadable", e)
PY
done
exit $st
