#!/bin/bash
# PMC calibration passes (tools/pmc_calib): FETCH_SIZE and WRITE_SIZE, one counter per run.
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out
TAG=${1:-calib}
mkdir -p $O
[ -x $R/tools/pmc_calib/pmc_calib ] || make -s -C $R/tools/pmc_calib || exit $?  # built here if the tree lacks it
cd /tmp && export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_calib_${C}_$TAG -o run -- \
    $R/tools/pmc_calib/pmc_calib > $O/pmc_calib_${C}_$TAG.log 2>&1 || exit $?
done
echo calib-ok
