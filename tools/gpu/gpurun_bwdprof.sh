#!/bin/bash
# kernel-trace of the training-path backward (per-kernel durations)
mkdir -p gpurun_out/bwdprof
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/bwdprof -o run --output-format csv -- python3 tools/kbench.py --bwd > gpurun_out/bwdprof/kbench.log 2>&1
rc=$?; echo "rc=$rc"; grep -v amdgpu.ids gpurun_out/bwdprof/kbench.log | tail -4
f=$(find gpurun_out/bwdprof -name "*kernel_stats.csv" | head -1); cut -c1-220 "$f" | head -14
