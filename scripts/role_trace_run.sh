set -o pipefail
mkdir -p gpurun_out/rt
export IPM355_LIB=/root/repo/build/rt/libipm355_trace.so
for b in 4 12 20 28; do
  IPM_TRACE_BLOCK=$b timeout -k 10 120 python scripts/role_trace.py 8192 > gpurun_out/rt/b$b.txt 2>&1 || exit 1
done
