#!/bin/bash
# fused sampling/pool launches: GPU suite (fail fast), overlap A/B, quick bench lines
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/overlap_ab.py 2>&1 | grep -v amdgpu.ids
for v in cog wan; do
  timeout -k 10 600 python bench.py --variant $v --no-pmc --no-cpu-baseline > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err || exit 1
  python -c "import json;d=json.load(open('gpurun_out/bench_$v.json'));r=d['roofline'];print('$v', d['value'], 'fps', d['ms_per_call'], 'ms/call', r['avg_launch_ms'], 'ms attn', r['achieved'], 'TF/s', d.get('speedup_vs_dense_sdpa'))"
done
