#!/bin/bash
# run-to-run determinism of the M3 phase-1 trajectory for several library specs (VAR=v@lib or lib)
#   scripts/traj_ab.sh OUTDIR REPS "spec spec ..."
set -o pipefail
o=$1; mkdir -p $o
for spec in $3; do
  envs=""; lib=$spec
  if [[ "$spec" == *@* ]]; then envs=${spec%@*}; lib=${spec##*@}; fi
  f=$o/$(echo $spec | tr '/=@' '___').txt
  env $envs IPM355_LIB=$PWD/$lib timeout -k 10 300 python -u scripts/traj_repeat.py m3_qp_ph1 $2 > $f 2>&1
  rc=$?; echo "$spec rc=$rc"; grep -c "rel 5.140e-14" $f; grep -v "rel 5.140e-14" $f | grep -v amdgpu
  [ $rc -ne 0 ] && exit $rc
done
exit 0
