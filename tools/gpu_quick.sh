#!/bin/bash
# quick GPU loop: level diagnostics, the level tests, a c5 bench (no CPU baseline / FFT / offline)
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u tools/diag_levels.py > $O/q_diag.log 2>&1 || { echo "diag rc=$?"; tail -20 $O/q_diag.log; exit 1; }
cat $O/q_diag.log
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_upols_gpu.py -k "level or far or stream or ahead or full" > $O/q_t.log 2>&1 || { echo "tests rc=$?"; tail -30 $O/q_t.log; exit 1; }
tail -2 $O/q_t.log
timeout -k 10 300 python bench.py --steps 128 --warmup 10 --no-cpu-baseline --no-fft --no-offline > $O/q_b.json 2> $O/q_b.err || { echo "bench rc=$?"; tail -20 $O/q_b.err; exit 1; }
python -c "
import json;r=json.load(open('$O/q_b.json'))
print('value',r['value'],'ms',r['ms_per_step'],'parity',r['parity']['parity_err'],'lat',r['latency']['mean_ms'],r['latency']['max_over_mean'],'kern',r['roofline']['kernel_avg_ms'],'frac',r['roofline']['frac'],'plain',r['per_block_step']['value'])"
