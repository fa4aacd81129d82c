#!/bin/bash
# Round 4: least-squares A/B (two-stage Frobenius norm, 1024-thread subproblem sweeps; HEAD library
# build/abh/r4h vs this tree's), then the checkpoint of this tree's library: the GPU suite, bench +
# rocprofv3 summary + PMC passes (gpu_round.sh), and the least-squares kernel profile.
set -o pipefail
OUT=gpurun_out/r4k
mkdir -p $OUT
NEW=interiorpoint-gpu_amd/ipm355/libipm355.so
for lib in build/abh/r4h/libipm355.so $NEW; do
  HOST_MAX=0 IPM355_LIB=$PWD/$lib timeout -k 10 300 python scripts/lstsq_time.py 2048 4096 | sed "s|^|$lib |" || exit $?
done 2>&1 | grep -v amdgpu.ids | tee $OUT/lstsq_ab.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -2 $OUT/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
SKIP_TESTS=1 TAG=r4k PT=400 BT=400 bash scripts/gpu_round.sh || exit $?
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
HOST_MAX=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_lstsq -o run -- \
    python3 scripts/lstsq_time.py 2048 > $OUT/lstsq_prof.txt 2>&1
echo "lstsq rocprof rc=$?"
