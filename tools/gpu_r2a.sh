#!/bin/bash
# round 2: upols GPU tests, then the c5 bench at the driver's step count and at 128 steps
set -o pipefail
O=gpurun_out
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_upols_gpu.py > $O/t2.log 2>&1
echo "tests rc=$?"; tail -3 $O/t2.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/b20.json 2> $O/b20.err || { echo "bench20 rc=$?"; tail -20 $O/b20.err; exit 1; }
timeout -k 10 300 python bench.py --steps 128 --warmup 10 --no-cpu-baseline --no-fft > $O/b128.json 2> $O/b128.err || { echo "bench128 rc=$?"; tail -20 $O/b128.err; exit 1; }
timeout -k 10 300 python bench.py --workload c4 --steps 128 --warmup 10 --no-cpu-baseline --no-fft > $O/b4.json 2> $O/b4.err || { echo "bench c4 rc=$?"; tail -20 $O/b4.err; exit 1; }
echo done
