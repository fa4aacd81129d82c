#!/bin/bash
# Round 4: (1) POTRF A/B of the round-3 library (build/abl/r3k) against this tree's (diag_role2
# out of the kernel: SGPR spills back to ~80), (2) least-squares GPU tests + timing against host
# np.linalg.lstsq, (3) KKT SYRK tile order A/B (IPM_SYRK_SB), (4) the GPU suite.  Every GPU step has its own time limit.
set -o pipefail
OUT=gpurun_out/r4d
mkdir -p $OUT
NEW=interiorpoint-gpu_amd/ipm355/libipm355.so
for r in 1 2; do
  for lib in build/abl/r3k/libipm355.so $NEW; do
    for n in "8193 9 8194" "2048 15" "4096 15"; do
      IPM355_LIB=$PWD/$lib timeout -k 10 120 python scripts/potrf_time.py $n | sed "s|^|$lib |" || exit $?
    done
  done
done 2>&1 | tee $OUT/potrf_ab.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
L=interiorpoint-gpu_amd/ipm355/libipm355.so
REPS=2 T=200 bash scripts/ab.sh $OUT/syrk "--steps 20 --warmup 2" IPM_SYRK_SB=0@$L IPM_SYRK_SB=8@$L IPM_SYRK_SB=4@$L \
    2>&1 | tee $OUT/syrk_ab.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s -k "lstsq" --timeout 300 --timeout-method thread > $OUT/pytest_lstsq.log 2>&1
rc=$?; echo "pytest lstsq rc=$rc"; grep -E "lstsq n=|passed|failed|FAILED" $OUT/pytest_lstsq.log | tail -30
[ $rc -ne 0 ] && exit $rc
HOST_MAX=4096 timeout -k 10 600 python scripts/lstsq_time.py 1025 2048 4096 8193 2>&1 | tee $OUT/lstsq_time.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest gpu rc=$rc"; tail -3 $OUT/pytest_gpu.log
exit $rc
