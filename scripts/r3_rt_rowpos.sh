set -o pipefail
mkdir -p gpurun_out/rt3
export IPM355_LIB=/root/repo/build/rt/libipm355_trace.so
for cfg in "IPM_ROWPOS=0" "IPM_ROWPOS=1"; do
  for b in 2 4 8; do
    env $cfg IPM_TRACE_BLOCK=$b timeout -k 10 120 python scripts/role_trace.py 8192 > "gpurun_out/rt3/b${b}_${cfg}.txt" 2>&1 || exit 1
  done
done
