#!/bin/bash
# build + run the diagonal-role lab on the GPU box (tools/chol_lab.hip)
set -o pipefail
mkdir -p gpurun_out/chol_lab build/lab
[ -x build/lab/chol_lab ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Iinteriorpoint-gpu_amd/csrc \
  tools/chol_lab.hip -o build/lab/chol_lab 2> gpurun_out/chol_lab/build.err || { tail -20 gpurun_out/chol_lab/build.err; exit 1; }
timeout -k 10 120 build/lab/chol_lab ${REPS:-40} | tee gpurun_out/chol_lab/out.txt
