#!/bin/bash
# the driver's round-end sequence plus longer benches: GPU tests, smoke, bench (driver flags),
# bench at 128 steps, c4 and c3 workloads
set -o pipefail
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/f_t.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -3 $O/f_t.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/f_smoke.log 2>&1 || { echo "smoke failed"; tail -5 $O/f_smoke.log; exit 1; }
tail -1 $O/f_smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/f_b20.json 2> $O/f_b20.err || { echo "bench20 rc=$?"; tail -20 $O/f_b20.err; exit 1; }
timeout -k 10 300 python bench.py --steps 128 --warmup 10 --no-cpu-baseline --no-fft > $O/f_b128.json 2> $O/f_b128.err || { echo "bench128 rc=$?"; tail -20 $O/f_b128.err; exit 1; }
timeout -k 10 300 python bench.py --workload c4 --steps 128 --warmup 10 --no-cpu-baseline --no-fft > $O/f_b4.json 2> $O/f_b4.err || { echo "bench c4 rc=$?"; tail -20 $O/f_b4.err; exit 1; }
timeout -k 10 300 python bench.py --workload c3 --steps 128 --warmup 10 --no-cpu-baseline --no-fft > $O/f_b3.json 2> $O/f_b3.err || { echo "bench c3 rc=$?"; tail -20 $O/f_b3.err; exit 1; }
echo done
