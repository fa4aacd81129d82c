#!/bin/bash
# build + run the diagonal-role lab on the GPU box (tools/chol_lab.hip)
set -o pipefail
mkdir -p gpurun_out/chol_lab build/lab
[ -x build/lab/chol_lab ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinclude -Iinteriorpoint-gpu_amd/csrc \
  tools/chol_lab.hip -o build/lab/chol_lab 2> gpurun_out/chol_lab/build.err || { tail -20 gpurun_out/chol_lab/build.err; exit 1; }
[ -n "$SKIP_CHOL" ] || timeout -k 10 120 build/lab/chol_lab ${REPS:-40} | tee gpurun_out/chol_lab/out.txt
[ -x build/lab/leaf2_lab ] && timeout -k 10 60 build/lab/leaf2_lab | tee gpurun_out/chol_lab/leaf2.txt
[ -x build/lab/tile_lab ] && timeout -k 10 120 build/lab/tile_lab | tee gpurun_out/chol_lab/tile.txt
