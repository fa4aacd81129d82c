#!/bin/bash
# potrf tests, timing (fused vs two-stream), and a kernel trace of the fused path
set -o pipefail
O=gpurun_out/${TAG:-fused}
mkdir -p $O
timeout -k 10 240 python -m pytest tests/test_gpu_kernels.py -m gpu -x -q -k "potrf or potrs" > $O/t.log 2>&1
rc=$?; tail -3 $O/t.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python scripts/potrf_time.py ${N:-8192} 2>&1 | grep -v amdgpu.ids || exit 1
[ -n "$CMP" ] && { IPM_POTRF_LA=1 timeout -k 10 120 python scripts/potrf_time.py ${N:-8192} 2>&1 | grep -v amdgpu.ids || exit 1; }
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/tr -o run -- python3 scripts/potrf_once.py ${N:-8192} > $O/tr.log 2>&1
