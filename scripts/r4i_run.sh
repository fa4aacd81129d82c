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
# per-kernel times of the blocked Jacobi (one n = 2048 least-squares solve)
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
HOST_MAX=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4i/prof_lstsq -o run -- \
    python3 scripts/lstsq_time.py 2048 > gpurun_out/r4i/lstsq_prof.txt 2>&1
echo "lstsq rocprof rc=$?"
