#!/bin/bash
# knob A/B of one library on the Cholesky alone: scripts/knob_ab.sh OUT LIB "VAR=a VAR=b ..."
# (env: REPS=2, SIZES as scripts/potrf_ab.sh)
set -o pipefail
out=$1; lib=$2; specs=""
for k in $3; do specs="$specs $k@$lib"; done
REPS=${REPS:-2} SIZES=${SIZES:-"8193:7:8194 2048:15"} scripts/potrf_ab.sh $out $specs
