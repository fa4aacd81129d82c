#!/bin/bash
# Run the full-solve parity tests against several prebuilt libraries (build/bisect/<tag>/).
set -o pipefail
mkdir -p gpurun_out/bisect
for lib in interiorpoint-gpu_amd/ipm355/libipm355.so build/bisect/*/libipm355.so; do
  tag=$(basename $(dirname $lib))
  IPM355_LIB=$PWD/$lib timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -q -k "${K:-full_solve}" \
      --timeout 120 --timeout-method thread > gpurun_out/bisect/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc: $(tail -1 gpurun_out/bisect/$tag.log)"
  grep FAILED gpurun_out/bisect/$tag.log | head -5
  [ $rc -ge 124 ] && exit $rc
done
exit 0
