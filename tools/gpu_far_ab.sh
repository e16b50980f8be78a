#!/bin/bash
# Same-box A/B of far-MAC builds (NEO_HIP_FAR=1): default lib, tools/far_a (plain loads),
# tools/far_b (3 waves/SIMD), C5 and C4, two rounds each; stops at the first failing run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"; O=$R/gpurun_out; mkdir -p $O; TAG=${1:-ab}
export NEO_HIP_FAR=1
for r in 1 2; do for w in c5 c4; do for v in def a b; do
  lib=""; [ $v != def ] && lib=$R/tools/far_$v/libneo_hip.so
  NEO_HIP_LIBRARY=$lib timeout -k 10 200 python bench.py --workload $w --steps 128 --no-cpu-baseline --no-offline > $O/farab_${v}_${w}_${r}_$TAG.json 2> $O/farab_${v}_${w}_${r}_$TAG.err || exit $?
  echo "$v $w $r $(python -c "import json;print(json.load(open('$O/farab_${v}_${w}_${r}_$TAG.json'))['value'])")"
done; done; done
