#!/bin/bash
set -o pipefail
o=gpurun_out/r5w; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/prof -o run -- python3 scripts/potrf_time.py 8193 3 8194 > $o/potrf.txt 2>&1 || exit 1
python scripts/potrf_launches.py $o/prof/run_kernel_trace.csv 32 > $o/launches_8193.txt
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/prof2 -o run -- python3 scripts/potrf_time.py 2048 3 > $o/potrf2.txt 2>&1 || exit 1
python scripts/potrf_launches.py $o/prof2/run_kernel_trace.csv 8 > $o/launches_2048.txt
rm -rf $o/prof $o/prof2
