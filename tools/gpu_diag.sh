#!/bin/bash
# Round 4 diagnostics: one handle's host round trip beside N idle handles; the group frame bench
# with the independent-mode staging variant (tools/ab/grp); then an A/B of the Toeplitz filter-row
# cache policy (tools/ab/hpol).
set -o pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R"
O=$R/gpurun_out
mkdir -p $O
for N in 1 256 2048; do
  timeout -k 10 300 tools/ab/diag/bench_handles $N >> $O/diag_handles.jsonl || exit $?
done
cat $O/diag_handles.jsonl
LD_LIBRARY_PATH=$R/tools/ab/grp timeout -k 10 300 tests/cpp/bin/bench_group 256 32 > $O/diag_group256_grp.json && \
LD_LIBRARY_PATH=$R/tools/ab/grp timeout -k 10 600 tests/cpp/bin/bench_group 2048 8 > $O/diag_group2048_grp.json || exit $?
cat $O/diag_group256_grp.json $O/diag_group2048_grp.json
LIBS="main hpol" WL="c5 c4 c5full" REPS=2 bash tools/gpu_abn.sh hpol
