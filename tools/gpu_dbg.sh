#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p gpurun_out
for n in 0 5; do
timeout -k 10 60 python tools/dbg_hwq.py $n 2>&1 | grep -v amdgpu.ids
NEO_HIP_LIBRARY=$PWD/tools/ab/pshi/libneo_hip.so timeout -k 10 60 python tools/dbg_hwq.py $n 2>&1 | grep -v amdgpu.ids
done
echo "== bitexact main"; timeout -k 10 120 python tools/dbg_bitexact.py 2>&1 | grep -v amdgpu.ids
echo "== bitexact fpon"; NEO_HIP_LIBRARY=$PWD/tools/ab/fpon/libneo_hip.so timeout -k 10 120 python tools/dbg_bitexact.py 2>&1 | grep -v amdgpu.ids
for rep in 1 2; do for L in main fpon; do
  if [ $L = main ]; then unset NEO_HIP_LIBRARY; else export NEO_HIP_LIBRARY=$PWD/tools/ab/fpon/libneo_hip.so; fi
  for w in c5full c5 c4; do
    timeout -k 10 300 python bench.py --workload $w --steps 128 --warmup 5 --no-cpu-baseline --no-fft --no-host-io --no-offline --no-paced --no-parity > gpurun_out/ab_fp_${L}_${w}_$rep.json 2>/dev/null || exit 1
    python -c "import json,sys; d=json.load(open('gpurun_out/ab_fp_${L}_${w}_$rep.json')); print('$L $w', d['value'], d['ms_per_step'])"
  done
done; done
unset NEO_HIP_LIBRARY
