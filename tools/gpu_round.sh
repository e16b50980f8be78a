#!/bin/bash
# One GPU session for the round's evidence: parity tests, smoke, bench lines (the driver's
# flags and longer runs), rocprofv3 kernel stats, PMC passes. Every GPU step has its own time
# limit; steps chained with && (stop at the first failure). PART=1: tests, smoke and bench lines;
# PART=2: rocprofv3 kernel stats, PMC passes and the counter calibration.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
TAG=${1:-r2}
if [ "$PART" != "2" ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 300 --timeout-method thread > $O/pytest_gpu_$TAG.log 2>&1; rc=$?; echo "pytest exit=$rc" >> $O/pytest_gpu_$TAG.log
tail -2 $O/pytest_gpu_$TAG.log
[ $rc -lt 124 ] || exit $rc  # a crash or a time limit: nothing more on the GPU in this call
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 && \
timeout -k 10 600 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c5full_$TAG.json 2> $O/bench_c5full_$TAG.err && \
timeout -k 10 300 python bench.py --steps 128 --warmup 5 --no-cpu-baseline --no-fft --no-host-io --no-offline > $O/bench_c5fulls128_$TAG.json 2> $O/bench_c5fulls128_$TAG.err && \
timeout -k 10 600 python bench.py --workload c5 --gpus 1 --steps 20 --warmup 5 --no-fft > $O/bench_c5_$TAG.json 2> $O/bench_c5_$TAG.err && \
timeout -k 10 300 python bench.py --workload c5 --steps 128 --no-cpu-baseline --no-fft > $O/bench_c5s128_$TAG.json 2> $O/bench_c5s128_$TAG.err && \
timeout -k 10 600 python bench.py --workload c2 --steps 20 --warmup 3 > $O/bench_c2_$TAG.json 2> $O/bench_c2_$TAG.err && \
timeout -k 10 300 python bench.py --workload c4 --steps 128 --no-cpu-baseline --no-fft > $O/bench_c4_$TAG.json 2> $O/bench_c4_$TAG.err && \
timeout -k 10 300 python bench.py --workload c3 --steps 256 --no-cpu-baseline --no-fft > $O/bench_c3_$TAG.json 2> $O/bench_c3_$TAG.err && \
timeout -k 10 300 python bench.py --workload c3long --steps 256 --no-cpu-baseline --no-fft > $O/bench_c3long_$TAG.json 2> $O/bench_c3long_$TAG.err && \
timeout -k 10 300 python bench.py --workload ref4096 --steps 256 --no-fft > $O/bench_ref4096_$TAG.json 2> $O/bench_ref4096_$TAG.err && \
timeout -k 10 300 python bench.py --workload c5 --host-io --steps 200 > $O/bench_c5_hostio_$TAG.json 2> $O/bench_c5_hostio_$TAG.err && \
timeout -k 10 300 tests/cpp/bin/bench_create 512 > $O/bench_create512_$TAG.json 2>&1 && \
timeout -k 10 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 \
  bench.py --gpus 2 --steps 20 --warmup 5 --no-fft --no-host-io > $O/bench_c5full_n2_$TAG.json 2> $O/bench_c5full_n2_$TAG.err || exit $?
fi
[ "$PART" = "1" ] && { echo "round part 1 exit=0"; exit 0; }
cd /tmp && export TMPDIR=/tmp && \
NEO_BENCH_MARK=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5full_$TAG -o run -- python3 $R/bench.py --steps 64 --warmup 5 --no-cpu-baseline --no-parity --no-fft --no-paced > $O/prof_c5full_$TAG.log 2>&1 && \
NEO_BENCH_MARK=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$TAG -o run -- python3 $R/bench.py --workload c5 --steps 64 --warmup 5 --no-cpu-baseline --no-parity --no-fft --no-paced > $O/prof_c5_$TAG.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2_$TAG -o run -- python3 $R/bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c2_$TAG.log 2>&1 && \
NEO_BENCH_MARK=1 timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4_$TAG -o run -- python3 $R/bench.py --workload c4 --steps 128 --no-cpu-baseline --no-parity --no-fft --no-paced > $O/prof_c4_$TAG.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_$TAG -o run -- python3 $R/bench.py --workload c3 --steps 256 --no-cpu-baseline --no-parity --no-fft --no-paced > $O/prof_c3_$TAG.log 2>&1 && \
cd $R && bash tools/gpu_pmc.sh $TAG && bash tools/gpu_calib.sh $TAG
echo "round exit=$?"
