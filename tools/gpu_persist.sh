#!/bin/bash
set -o pipefail
cd ${GRAFT_REPO_ROOT:-$(pwd)}; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_persist_gpu.py -x -v -rf --timeout 120 --timeout-method thread > gpurun_out/pytest_pf.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_pf.log | grep -E "PASS|FAIL|Error|assert|passed|failed"; exit $rc
