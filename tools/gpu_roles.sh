#!/bin/bash
# Role-masked timings of the step kernel (tools/build_roles.sh builds) at the workloads given
# in $W (default "c5 c4"), tag $1: rocprofv3 kernel-trace medians per build.
set -o pipefail
R0=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R0"
T=${1:-roles}
for w in ${WL:-c5 c4}; do
  W=$w bash tools/gpu_prof_roles.sh full 1 2 4 8 16 30 29 27 23 15 > gpurun_out/roles_${w}_$T.txt 2>&1 || { cat gpurun_out/roles_${w}_$T.txt; exit 1; }
  echo "== $w"; cat gpurun_out/roles_${w}_$T.txt
done
