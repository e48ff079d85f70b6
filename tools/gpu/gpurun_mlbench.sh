#!/bin/bash
# Multi-level sampler path: bench line (with PMC traffic + CPU baseline) and its rocprofv3 stats.
set -o pipefail
TAG=${TAG:-r01_ml}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python bench.py --variant cog-ml > $OUT/bench_cogml.json 2> $OUT/bench_cogml.err
rc=$?; echo "bench cog-ml rc=$rc"; cat $OUT/bench_cogml.json; tail -3 $OUT/bench_cogml.err
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --variant cog-ml --steps 2 --warmup 1 --no-cpu-baseline --no-pmc --no-dense > $OUT/prof_bench.json 2> $OUT/prof_bench.err
rc=$?; echo "rocprof rc=$rc"
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); head -12 "$f" | cut -c1-220
