#!/bin/bash
# 2-rank torch.distributed.run rehearsal of the default bench on the one box GPU (both ranks on
# device 0) and the default bench at 128 steps, tag $1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-n2}
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --no-fft > $O/bench_c5full_n2_$T.json 2> $O/bench_c5full_n2_$T.err && \
timeout -k 10 600 python bench.py --steps 128 --no-cpu-baseline --no-fft > $O/bench_c5full_s128_$T.json 2> $O/bench_c5full_s128_$T.err && \
echo n2-ok
