#!/bin/bash
# BASELINE configs[2]: CogVideoX sparsity sweep 30/50/70 % (fixed block density 0.7/0.5/0.3),
# and configs[4]: the TDM-style training step (batch 5 x accum 4) on stand-in blocks
set -o pipefail
mkdir -p gpurun_out/sweep2
for d in 0.7 0.5 0.3; do
  timeout -k 10 600 python bench.py --density $d --no-pmc --no-cpu-baseline > gpurun_out/sweep2/cog_d$d.json 2> gpurun_out/sweep2/cog_d$d.err
  rc=$?; [ $rc -eq 0 ] || { echo "rc=$rc"; tail -3 gpurun_out/sweep2/cog_d$d.err; exit $rc; }
  python -c "import json;d=json.load(open('gpurun_out/sweep2/cog_d$d.json'));r=d['roofline'];print('density $d', d['value'], 'fps', d['ms_per_call'], 'ms/call', r['achieved'], 'TF/s', 'x', d['speedup_vs_dense_sdpa'], 'sparsity', d['mean_sparsity'])"
done
timeout -k 10 900 python tools/train_bench.py --layers 2 --batch 5 --accum 4 --steps 2 --warmup 1 > gpurun_out/sweep2/train.json 2> gpurun_out/sweep2/train.err
rc=$?; echo "train rc=$rc"; tail -1 gpurun_out/sweep2/train.json
