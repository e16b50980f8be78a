#!/bin/bash
# Same-box A/B/... of library builds: $LIBS = names under tools/ab/ ("main" = neo-dsp_amd/lib),
# the level GPU tests on the main build first, then interleaved bench lines at $WL, $REPS
# repetitions, tag $1.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-ab}
timeout -k 10 600 python -u -m pytest tests/test_upols_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "level or far or full_size or ahead or multi or before_any or c3" > $O/pytest_ab_$T.log 2>&1 || { tail -5 $O/pytest_ab_$T.log; exit 1; }
echo tests-ok
for rep in $(seq 1 ${REPS:-2}); do
  for W in ${WL:-c4 c5 c5full}; do
    for L in ${LIBS:-main}; do
      if [ $L = main ]; then LIB=""; else LIB=$R/tools/ab/$L/libneo_hip.so; fi
      NEO_HIP_LIBRARY=$LIB timeout -k 10 300 python bench.py --workload $W --steps ${STEPS:-64} --warmup 5 --no-cpu-baseline \
        --no-fft --no-offline --no-parity --no-host-io --no-paced > $O/ab_${T}_${W}_${L}_$rep.json 2> $O/ab_${T}_${W}_${L}_$rep.err || exit 1
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value'],1), 'wall', round(d['ms_per_step']*1e3,2), 'gpu', round(d['gpu_ms_per_step']*1e3,2))" $O/ab_${T}_${W}_${L}_$rep.json $W $L
    done
  done
done
