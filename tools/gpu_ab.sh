#!/bin/bash
# Same-box A/B of a candidate build (neo-dsp_amd/lib) against tools/ab/base/libneo_hip.so:
# the level GPU tests on the candidate, then interleaved bench lines (c4, c5, c5full), tag $1
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
T=${1:-ab}
timeout -k 10 600 python -u -m pytest tests/test_upols_gpu.py -x -q --timeout 120 --timeout-method thread \
  -k "level or far or full_size or ahead or multi or before_any" > $O/pytest_ab_$T.log 2>&1 || { tail -5 $O/pytest_ab_$T.log; exit 1; }
echo tests-ok
for rep in 1 2; do
  for W in c4 c5 c5full; do
    for L in base new; do
      if [ $L = base ]; then LIB=$R/tools/ab/base/libneo_hip.so; else LIB=""; fi
      NEO_HIP_LIBRARY=$LIB timeout -k 10 300 python bench.py --workload $W --steps 64 --warmup 5 --no-cpu-baseline \
        --no-fft --no-offline --no-parity > $O/ab_${T}_${W}_${L}_$rep.json 2> $O/ab_${T}_${W}_${L}_$rep.err || exit 1
      python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], sys.argv[3], round(d['value'],1), round(d['ms_per_step']*1e3,2), round(d['gpu_ms_per_step']*1e3,2))" $O/ab_${T}_${W}_${L}_$rep.json $W $L
    done
  done
done
