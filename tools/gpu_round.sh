#!/bin/bash
# One GPU session: parity tests, smoke, bench lines, rocprofv3 kernel stats.
# Every GPU step has its own time limit; steps chained with && (stop at first failure).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
TAG=${1:-r1}
timeout -k 10 900 python -m pytest tests -m gpu -q -rf --timeout 600 > $O/pytest_gpu_$TAG.log 2>&1; echo "pytest exit=$?" >> $O/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke_$TAG.log 2>&1 && \
timeout -k 10 600 python bench.py > $O/bench_c5_$TAG.json 2> $O/bench_c5_$TAG.err && \
timeout -k 10 600 python bench.py --workload c2 --steps 20 --warmup 3 > $O/bench_c2_$TAG.json 2> $O/bench_c2_$TAG.err && \
timeout -k 10 300 python bench.py --workload c4 --steps 128 --no-cpu-baseline > $O/bench_c4_$TAG.json 2> $O/bench_c4_$TAG.err && \
timeout -k 10 300 python bench.py --workload c3 --steps 256 --no-cpu-baseline > $O/bench_c3_$TAG.json 2> $O/bench_c3_$TAG.err && \
timeout -k 10 300 python bench.py --host-io --steps 200 > $O/bench_c5_hostio_$TAG.json 2> $O/bench_c5_hostio_$TAG.err && \
cd /tmp && export TMPDIR=/tmp && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c5_$TAG -o run -- python3 $R/bench.py --steps 64 --warmup 5 --no-cpu-baseline --no-offline > $O/prof_c5_$TAG.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c2_$TAG -o run -- python3 $R/bench.py --workload c2 --steps 20 --warmup 3 --no-cpu-baseline > $O/prof_c2_$TAG.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4_$TAG -o run -- python3 $R/bench.py --workload c4 --steps 128 --no-cpu-baseline --no-offline > $O/prof_c4_$TAG.log 2>&1 && \
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_$TAG -o run -- python3 $R/bench.py --workload c3 --steps 256 --no-cpu-baseline --no-offline > $O/prof_c3_$TAG.log 2>&1 && \
cd $R && bash tools/gpu_pmc.sh $TAG
echo "round exit=$?"
