#!/bin/bash
# Round 4: persistent trailing-tile workers (IPM_SPERSIST=1: Cholesky GPU tests under the knob, then
# POTRF and bench A/B), blocked-Jacobi sweep counts, config-4 hardware-queue A/B, the other configs.
set -o pipefail
OUT=gpurun_out/r4g
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s -k "lstsq" --timeout 300 --timeout-method thread > $OUT/pytest_lstsq.log 2>&1
rc=$?; echo "pytest lstsq rc=$rc"; grep -E "lstsq n=|passed|failed|FAILED" $OUT/pytest_lstsq.log | tail -4
[ $rc -ne 0 ] && exit $rc
IPM_SPERSIST=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "potrf" --timeout 300 --timeout-method thread > $OUT/pytest_persist.log 2>&1
rc=$?; echo "pytest potrf persist rc=$rc"; tail -2 $OUT/pytest_persist.log
[ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in 0 1; do
    for n in "8193 9 8194" "2048 15" "4096 15"; do
      IPM_SPERSIST=$v timeout -k 10 120 python scripts/potrf_time.py $n || exit $?
    done
  done
done 2>&1 | tee $OUT/persist_ab.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
L=interiorpoint-gpu_amd/ipm355/libipm355.so
REPS=2 T=200 bash scripts/ab.sh $OUT/pab "--steps 20 --warmup 2" IPM_SPERSIST=0@$L IPM_SPERSIST=1@$L 2>&1 | tee $OUT/persist_bench_ab.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
for f in 1 0; do
  IPM_BJ_FUSED=$f IPM_BJ_DEBUG=1 HOST_MAX=0 timeout -k 10 300 python scripts/lstsq_time.py 2048 8193 > $OUT/lstsq_sweeps_f$f.txt 2>&1 || exit 1
  echo "fused=$f sweeps: $(grep -c sweep $OUT/lstsq_sweeps_f$f.txt)"; grep device_s $OUT/lstsq_sweeps_f$f.txt
done
for r in 1; do
  for q in 4 8 16; do
    IPM_HW_QUEUES=$q timeout -k 10 300 python bench.py --no-cpu --n 2048 --m 512 --instances 8 --concurrent --steps 20 --warmup 2 > $OUT/c4_q$q.json 2> $OUT/c4_q$q.err || exit 1
    python3 -c "import json;d=json.load(open('$OUT/c4_q$q.json'));print('c4 queues $q', round(d['value'],1))"
  done
done 2>&1 | tee $OUT/c4_queues.txt
[ ${PIPESTATUS[0]} -ne 0 ] && exit 1
TAG=r4g_cfg bash scripts/gpu_configs.sh
