set -o pipefail
timeout -k 10 900 python -u -m pytest tests/test_group_gpu.py tests/test_overlap_gpu.py tests/test_cpp_api.py tests/test_upols_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -rf > gpurun_out/pytest_new.log 2>&1; rc=$?
tail -15 gpurun_out/pytest_new.log
exit $rc
