#!/bin/bash
# Round 4: least-squares GPU tests + timing against host np.linalg.lstsq, the GPU suite (verbose:
# the parity prints go to the log), bench + rocprofv3 kernel-trace summary.
set -o pipefail
OUT=gpurun_out/r4e
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s -k "lstsq" --timeout 300 --timeout-method thread > $OUT/pytest_lstsq.log 2>&1
rc=$?; echo "pytest lstsq rc=$rc"; grep -E "lstsq n=|x\* rel|passed|failed|FAILED" $OUT/pytest_lstsq.log | tail -30
[ $rc -ne 0 ] && exit $rc
HOST_MAX=4096 timeout -k 10 600 python scripts/lstsq_time.py 1025 2048 4096 8193 2>&1 | tee $OUT/lstsq_time.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
SKIP_TESTS=1 SKIP_PMC=1 TAG=r4e PT=400 BT=400 bash scripts/gpu_round.sh
