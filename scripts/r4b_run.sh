set -o pipefail
mkdir -p gpurun_out/r4b
bash scripts/diag2_lab.sh > gpurun_out/r4b/diag2_lab.txt 2>&1; rc=$?; echo "diag2 lab rc=$rc"; cat gpurun_out/r4b/diag2_lab.txt | head -40
if [ $rc -gt 1 ]; then exit $rc; fi
REPS=2 scripts/ab.sh gpurun_out/r4b/ab "--steps 20 --warmup 2" build/abl/r3k/libipm355.so build/abl/spin/libipm355.so build/abl/d2v0/libipm355.so build/abl/d2v1/libipm355.so || exit $?
echo "--- n=2048 m=512"
REPS=2 scripts/ab.sh gpurun_out/r4b/ab2k "--n 2048 --m 512 --steps 40 --warmup 4" build/abl/r3k/libipm355.so build/abl/d2v0/libipm355.so build/abl/d2v1/libipm355.so
