#!/bin/bash
set -o pipefail
o=gpurun_out/${TAG:-r5y}; mkdir -p $o
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/prof -o run -- python3 bench.py --no-cpu --n 2048 --m 512 --steps 20 --warmup 2 > $o/c2.json 2> $o/c2.err || exit 1
python - <<PY > $o/c2_step.txt
import csv
rows=list(csv.DictReader(open('$o/prof/run_kernel_trace.csv')))
ks=sorted([(r['Kernel_Name'][:60], int(r['Start_Timestamp']), int(r['End_Timestamp'])) for r in rows], key=lambda k:k[1])
idx=[i for i,k in enumerate(ks) if 'k_mfma_gemm_split' in k[0]]
a,b=idx[-3],idx[-2]
prev=ks[a][1]
for nm,s,e in ks[a:b]:
    print(f"{(s-ks[a][1])/1e3:8.1f} +{(s-prev)/1e3:5.1f} {(e-s)/1e3:7.1f} {nm}")
    prev=e
print("step", (ks[b][1]-ks[a][1])/1e3)
PY
rm -rf $o/prof
