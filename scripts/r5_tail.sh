#!/bin/bash
set -o pipefail
o=gpurun_out/r5v; mkdir -p $o
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_kernels.py -k "tail or ragged or split_trailing or potrf" > $o/tests.txt 2>&1 || { tail -30 $o/tests.txt; exit 1; }
tail -3 $o/tests.txt
for t in 0 1; do
  IPM_TAIL=$t timeout -k 10 300 python bench.py --no-cpu --n 2048 --m 512 --steps 40 --warmup 4 > $o/c2_tail$t.json 2> $o/c2_tail$t.err || exit 1
  IPM_TAIL=$t timeout -k 10 300 python bench.py --no-cpu --steps 12 --warmup 2 > $o/c1_tail$t.json 2> $o/c1_tail$t.err || exit 1
done
python - <<'PY'
import json
for c in ("c2", "c1"):
    for t in (0, 1):
        d = json.load(open(f"gpurun_out/r5v/{c}_tail{t}.json"))
        ph = d["phases"]
        print(c, "tail", t, round(d["value"], 1), {k: (round(v["iters_per_s"] or 0, 1), round(v["potrf_ms"], 3)) for k, v in ph.items()})
PY
