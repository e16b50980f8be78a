#!/bin/bash
# the plain step's latency mode (k_plain_persist): its tests, then a same-box A/B of the plain
# step kernel (tools/ab/head: the library before upols_step_wg) at ref4096 and c5
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out; T=${1:-pl}
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_persist_gpu.py tests/test_upols_gpu.py > gpurun_out/${T}_pytest.log 2>&1 || { tail -30 gpurun_out/${T}_pytest.log; exit 1; }
  tail -2 gpurun_out/${T}_pytest.log
fi
for rep in 1 2; do for L in ${LIBS:-main head}; do
  if [ $L = main ]; then unset NEO_HIP_LIBRARY; else export NEO_HIP_LIBRARY=$PWD/tools/ab/$L/libneo_hip.so; fi
  for w in ${WL:-ref4096 c5}; do
    timeout -k 10 300 python bench.py --workload $w --steps ${STEPS:-128} --warmup 5 --no-cpu-baseline --no-fft --no-host-io --no-offline --no-paced --no-parity > gpurun_out/${T}_${L}_${w}_$rep.json 2> gpurun_out/${T}_${L}_${w}_$rep.err || { tail -20 gpurun_out/${T}_${L}_${w}_$rep.err; exit 1; }
    python - <<PY
import json; d=json.load(open('gpurun_out/${T}_${L}_${w}_$rep.json')); p=d['per_block_step']; lm=d.get('latency_mode') or {}
print('$L $w $rep', round(d['value'],1), round(d['ms_per_step']*1e3,2), 'plain', round(p['kernel_avg_ms']*1e3,2), round(p['frac'],3),
      'lat', lm.get('available'), lm.get('host_roundtrip_p50_us'), lm.get('host_roundtrip_p99_us'), lm.get('gpu_step_p50_us'), lm.get('reason'),
      'rt', round(d['latency']['host_roundtrip_p50_us'],1))
PY
  done
done; done
