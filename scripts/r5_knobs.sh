#!/bin/bash
set -o pipefail
L=build/r5ab/lib_final.so
REPS=2 SIZES="8193:9:8194 4096:15" scripts/potrf_ab.sh gpurun_out/r5kn/ab.txt $L IPM_PAIR_MIN=5120@$L IPM_PAIR_MIN=7168@$L IPM_LA128_MIN=2048@$L IPM_LA128_MIN=4096@$L
