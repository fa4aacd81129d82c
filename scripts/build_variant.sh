#!/bin/bash
# Variant library for A/B runs: build/r6ab/NAME.so = libipm355.so with ipm_blas.hip rebuilt under
# extra defines.   scripts/build_variant.sh NAME "-DIPM_DIAG_V=... [-DIPM_ROLE_TRACE]"
set -e
name=$1; defs=$2
make -s -j8 >/dev/null
mkdir -p build/r6ab build/vobj
H="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wno-unused-result -Wno-unused-value -Iinclude -Iinteriorpoint-gpu_amd/csrc"
/opt/rocm/bin/hipcc $H $defs -c interiorpoint-gpu_amd/csrc/ipm_blas.hip -o build/vobj/$name.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC build/vobj/$name.o build/obj/ipm_barrier.o \
  build/obj/ipm_engine.o build/obj/ipm_lasso.o build/obj/ipm_lstsq.o -o build/r6ab/$name.so
echo built build/r6ab/$name.so
