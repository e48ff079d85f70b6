#!/bin/bash
# pooled-pass grid cap sweep (VB_POOL_WGS) on the cog and cog-ml bench lines
set -o pipefail
mkdir -p gpurun_out/sweep
for v in cog cog-ml; do
for w in ${WGS:-0 128 256 512 1024}; do
  VB_POOL_WGS=$w timeout -k 10 300 python bench.py --variant $v --no-pmc --no-cpu-baseline --no-dense > gpurun_out/sweep/b_${v}_$w.json 2> gpurun_out/sweep/b_${v}_$w.err
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/sweep/b_${v}_$w.json'));print('$v wgs=$w', d['value'], 'fps', d['ms_per_call'], 'ms/call', d['roofline']['avg_launch_ms'])"
done
done
