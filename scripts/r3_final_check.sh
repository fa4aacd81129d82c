#!/bin/bash
# GPU suite on the current library, then the lazy-C vs split-planner A/B
set -o pipefail
mkdir -p gpurun_out/r3i
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r3i/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 gpurun_out/r3i/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
bash scripts/r3_splitlazy.sh
