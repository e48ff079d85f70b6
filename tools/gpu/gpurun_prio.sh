#!/bin/bash
set -o pipefail
mkdir -p gpurun_out/prio
for rep in 1 2; do
for p in 0 1; do
  VB_PRIO=$p timeout -k 10 300 python bench.py --variant ${V:-cog} --no-pmc --no-cpu-baseline --no-dense > gpurun_out/prio/b_$p.json 2> gpurun_out/prio/b_$p.err
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -5 gpurun_out/prio/b_$p.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/prio/b_$p.json'));print('prio=$p', d['value'], 'fps', d['ms_per_call'], 'ms/call', d['roofline']['avg_launch_ms'])"
done
done
