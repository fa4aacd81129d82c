#!/bin/bash
# Round-4 checkpoint: the GPU suite (verbose: parity prints), bench + rocprofv3 summary, PMC passes
# (FETCH / WRITE / MFMA busy) for this library hash.
set -o pipefail
OUT=gpurun_out/r4i
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
SKIP_TESTS=1 TAG=r4i PT=400 BT=400 bash scripts/gpu_round.sh
