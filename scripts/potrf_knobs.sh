#!/bin/bash
# POTRF timing under each library knob combination (one process per configuration).
N=${1:-8192}
for cfg in "" "IPM_NO_FOLD=1" "IPM_LA_SIDE=1" "IPM_LA_SIDE=1 IPM_NO_FOLD=1" "IPM_EV_NOFENCE=1" \
           "IPM_EV_NOFENCE=1 IPM_LA_SIDE=1" "IPM_EV_NOFENCE=1 IPM_LA_SIDE=1 IPM_NO_FOLD=1" $EXTRA; do
  env $cfg timeout -k 10 120 python scripts/potrf_time.py $N || exit $?
done
