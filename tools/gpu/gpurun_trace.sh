#!/bin/bash
# kernel timeline of a short bench run (for overlap / gap analysis)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/trace
timeout -k 10 600 rocprofv3 --kernel-trace -d gpurun_out/trace/prof -o run --output-format csv -- python3 bench.py --variant ${V:-cog} --steps 1 --warmup 1 --no-cpu-baseline --no-pmc --no-dense > gpurun_out/trace/bench.json 2> gpurun_out/trace/bench.err
rc=$?; echo "rc=$rc"; cat gpurun_out/trace/bench.json | cut -c1-300
f=$(find gpurun_out/trace/prof -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py "$f" > gpurun_out/trace/timeline.txt; head -60 gpurun_out/trace/timeline.txt
