#!/bin/bash
# quick loop: module-level GPU tests, then the three bench lines without PMC / CPU legs
set -o pipefail
mkdir -p gpurun_out/quick
timeout -k 10 600 python -m pytest tests/test_gpu_module.py tests/test_gpu_multilevel.py -x -q -p no:cacheprovider > gpurun_out/quick/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/quick/pytest.log
[ $rc -eq 0 ] || exit $rc
for v in ${VARIANTS:-cog wan cog-ml}; do
  timeout -k 10 600 python bench.py --variant $v --no-pmc --no-cpu-baseline $BENCH_ARGS > gpurun_out/quick/bench_$v.json 2> gpurun_out/quick/bench_$v.err
  rc=$?; echo "bench $v rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/quick/bench_$v.json'));r=d['roofline'];print('$v', d['value'], 'fps', d['ms_per_call'], 'ms/call', r['avg_launch_ms'], 'ms attn', r['achieved'], 'TF/s', d.get('speedup_vs_dense_sdpa'))"
done
