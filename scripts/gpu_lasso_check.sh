set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_lasso.py -m gpu -q -s --timeout 200 --timeout-method thread -k "potrs or lasso or device" > gpurun_out/r2h_tests.log 2>&1; rc=$?; tail -3 gpurun_out/r2h_tests.log; [ $rc -ne 0 ] && exit $rc
TAG=lasso2 bash scripts/lasso_gpu.sh
