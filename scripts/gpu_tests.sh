#!/bin/bash
# GPU-box test step: build, kernel tests, parity tests (each under its own time limit).
set -o pipefail
make -j8 > gpurun_out/build.log 2>&1 || { echo "build failed"; tail -20 gpurun_out/build.log; exit 1; }
timeout -k 10 ${KT:-300} python -u -m pytest tests/test_gpu_kernels.py -q --timeout 120 --timeout-method thread ${PYARGS} > gpurun_out/k.log 2>&1
rc=$?; echo "kernels rc=$rc"; tail -4 gpurun_out/k.log
[ $rc -ge 124 ] && exit $rc
timeout -k 10 ${PT:-500} python -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread ${PYARGS} > gpurun_out/p.log 2>&1
rc=$?; echo "parity rc=$rc"; tail -25 gpurun_out/p.log
exit $rc
