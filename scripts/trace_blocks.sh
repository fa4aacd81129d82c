set -o pipefail
for b in 1 6; do IPM_TRACE_BLOCK=$b timeout -k 10 120 python scripts/role_trace.py 8192 || exit $?; done
