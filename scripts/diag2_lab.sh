#!/bin/bash
# build (if needed) + run the round-4 diagonal-role lab on the GPU box (tools/diag2_lab.hip)
set -o pipefail
mkdir -p gpurun_out/diag2_lab build/lab4
for v in plain stamps; do
  f=""; [ $v = stamps ] && f="-DIPM_STAMPS2 -DSTAMP_V"
  [ -x build/lab4/diag2_lab_$v ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off $f -Iinclude \
    -Iinteriorpoint-gpu_amd/csrc tools/diag2_lab.hip -o build/lab4/diag2_lab_$v 2> gpurun_out/diag2_lab/build_$v.err \
    || { tail -20 gpurun_out/diag2_lab/build_$v.err; exit 1; }
  timeout -k 10 120 build/lab4/diag2_lab_$v ${REPS:-40} | tee gpurun_out/diag2_lab/$v.txt || exit $?
done
