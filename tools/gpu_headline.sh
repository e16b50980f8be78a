#!/bin/bash
# Headline evidence for the default workload (c5full: 2048 ch on one GPU), tag $1: the bench
# line at the driver's flags, rocprofv3 kernel stats, the FETCH_SIZE / WRITE_SIZE PMC passes of
# the same command, and a 2-rank torch.distributed.run rehearsal of bench.py on the one GPU.
# Every GPU step has its own time limit; steps chained with && (stop at the first failure).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-r2h}
W=c5full
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_${W}_$T.json 2> $O/bench_${W}_$T.err && \
echo bench-ok && \
(cd /tmp && export TMPDIR=/tmp && \
 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_${W}_$T -o run -- \
   python3 $R/bench.py --workload $W --steps 64 --warmup 5 --no-cpu-baseline --no-parity --no-fft \
   > $O/prof_${W}_$T.log 2>&1) && \
echo prof-ok && \
(cd /tmp && export TMPDIR=/tmp && \
 for C in FETCH_SIZE WRITE_SIZE; do
   timeout -s KILL 400 rocprofv3 --pmc $C --output-format csv -d $O/pmc_${W}_${C}_$T -o run -- \
     python3 $R/bench.py --workload $W --steps 32 --warmup 2 --no-cpu-baseline --no-parity --no-fft \
     > $O/pmc_${W}_${C}_$T.log 2>&1 || exit $?
 done) && \
echo pmc-ok && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 5 --no-fft > $O/bench_${W}_n2_$T.json 2> $O/bench_${W}_n2_$T.err && \
echo n2-ok
st=$?; echo "headline exit=$st"; [ $st -eq 0 ] || exit $st
# role-masked builds (tools/build_roles.sh) at the headline workload, if built
if [ -d tools/ab/1 ]; then
  W=$W timeout -k 10 900 bash tools/gpu_prof_roles.sh full 1 2 4 8 16 30 29 27 23 15 > $O/roles_${W}_$T.log 2>&1
  echo "roles exit=$?"
fi
