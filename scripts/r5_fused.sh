#!/bin/bash
set -o pipefail
o=gpurun_out/r5x; mkdir -p $o
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py > $o/parity.txt 2>&1 || { tail -40 $o/parity.txt; exit 1; }
tail -3 $o/parity.txt
for f in 0 1; do :; done
for f in 0 1; do
  IPM_FUSED_GRAD=$f timeout -k 10 300 python bench.py --no-cpu --n 2048 --m 512 --steps 40 --warmup 4 > $o/c2_f$f.json 2> $o/c2_f$f.err || exit 1
done
IPM_FUSED_GRAD=1 timeout -k 10 300 python bench.py --no-cpu --n 2048 --m 512 --instances 8 --concurrent --steps 20 --warmup 2 > $o/c4_f1.json 2> $o/c4.err || exit 1
IPM_FUSED_GRAD=0 timeout -k 10 300 python bench.py --no-cpu --n 2048 --m 512 --instances 8 --concurrent --steps 20 --warmup 2 > $o/c4_f0.json 2> $o/c4.err || exit 1
python - <<'PY'
import json
for c in ("c2_f0", "c2_f1", "c4_f0", "c4_f1"):
    d = json.load(open(f"gpurun_out/r5x/{c}.json"))
    print(c, round(d["value"], 1), d["ms_per_step"])
PY
IPM_SYNC_SPIN=0 timeout -k 10 300 python bench.py --no-cpu --n 2048 --m 512 --steps 40 --warmup 4 > $o/c2_spin0.json 2> $o/c2_spin0.err || exit 1
python -c "import json; d=json.load(open('$o/c2_spin0.json')); print('c2 sync_spin=0', round(d['value'],1))"
