#!/bin/bash
# A/B of library builds on the Cholesky alone (scripts/potrf_time.py: HIP-event median per size),
# alternating builds, REPS pairs.
#   scripts/potrf_ab.sh OUTFILE LIB1 LIB2 ...     (env: REPS=2, SIZES="8193:9:8194 4096:15 2048:25")
# A size entry is n:reps[:lda].  Knob A/B: VAR=value@lib (the same library twice, one knob set).
# Replaces round 4's one-off scripts/r4*_run.sh wrappers.
set -o pipefail
out=$1; shift
mkdir -p "$(dirname "$out")"
: > "$out"
for rep in $(seq 1 ${REPS:-2}); do
  for spec in "$@"; do
    envs=""; lib=$spec
    if [[ "$spec" == *@* ]]; then envs=${spec%@*}; lib=${spec##*@}; fi
    for sz in ${SIZES:-8193:9:8194 4096:15 2048:25}; do
      env $envs IPM355_LIB=$PWD/$lib timeout -k 10 120 python scripts/potrf_time.py ${sz//:/ } 2>&1 \
        | grep -v amdgpu.ids | sed "s|^|$spec |" | tee -a "$out"
      rc=${PIPESTATUS[0]}
      [ $rc -ne 0 ] && { echo "$spec n=$sz rc=$rc"; exit $rc; }
    done
  done
done
exit 0
