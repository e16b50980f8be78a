#!/bin/bash
# the bench lines only (driver flags for c5, 128 steps, c4, c3), tag $1
set -o pipefail
T=${1:-r2}; O=gpurun_out
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c5_$T.json 2> $O/bench_c5_$T.err && \
timeout -k 10 300 python bench.py --steps 128 --no-cpu-baseline --no-fft > $O/bench_c5s128_$T.json 2> $O/bench_c5s128_$T.err && \
timeout -k 10 300 python bench.py --workload c4 --steps 128 --no-cpu-baseline --no-fft > $O/bench_c4_$T.json 2> $O/bench_c4_$T.err && \
timeout -k 10 300 python bench.py --workload c3 --steps 256 --no-cpu-baseline --no-fft > $O/bench_c3_$T.json 2> $O/bench_c3_$T.err && echo benches-ok
