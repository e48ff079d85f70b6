#!/bin/bash
mkdir -p gpurun_out/trace2
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/trace2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 1 --no-pmc --no-cpu-baseline --no-dense ${BENCH_ARGS} > gpurun_out/trace2/bench.json 2> gpurun_out/trace2/bench.err
echo "rc=$?"
