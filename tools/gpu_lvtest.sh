#!/bin/bash
# level diagnostics, the level / far / full-size GPU tests, step-kernel timing at C5 and C3
set -o pipefail
timeout -k 10 300 python -u tools/diag_levels.py > gpurun_out/q_diag.log 2>&1 || { echo diag failed; tail -20 gpurun_out/q_diag.log; exit 1; }
grep -c ok gpurun_out/q_diag.log
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_upols_gpu.py -k "level or far or stream or ahead or full or multi" > gpurun_out/q_t.log 2>&1 || { echo tests failed; tail -30 gpurun_out/q_t.log; exit 1; }
tail -1 gpurun_out/q_t.log
bash tools/gpu_prof_roles.sh full
W=c3 bash tools/gpu_prof_roles.sh full
