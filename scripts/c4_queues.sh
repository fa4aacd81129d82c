set -o pipefail
mkdir -p gpurun_out/r2q
for q in 16 8 32; do
  IPM_HW_QUEUES=$q timeout -k 10 200 python bench.py --no-cpu --n 2048 --m 512 --instances 8 --concurrent --steps 20 --warmup 2 > gpurun_out/r2q/c4_q$q.json 2> gpurun_out/r2q/c4_q$q.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/r2q/c4_q$q.json'));print($q, d['value'], d['potrf']['avg_ms'], d['kkt_syrk']['avg_launch_ms'])"
done
