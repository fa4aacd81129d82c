set -o pipefail
mkdir -p gpurun_out/r4a
bash scripts/diag2_lab.sh > gpurun_out/r4a/diag2_lab.txt 2>&1; rc=$?; echo "diag2 lab rc=$rc"; cat gpurun_out/r4a/diag2_lab.txt | head -40
if [ $rc -gt 1 ]; then exit $rc; fi
timeout -k 10 700 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread > gpurun_out/r4a/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "FAILED|ERROR|passed|failed" gpurun_out/r4a/pytest.log | tail -15
if [ $rc -gt 1 ]; then exit $rc; fi
REPS=2 scripts/ab.sh gpurun_out/r4a/ab "--steps 20 --warmup 2" build/abl/r3k/libipm355.so interiorpoint-gpu_amd/ipm355/libipm355.so
