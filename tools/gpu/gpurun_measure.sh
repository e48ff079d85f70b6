#!/bin/bash
# Round measurement: GPU parity suite, the contract bench (cog + wan), and the rocprofv3
# kernel-trace summary of the same bench command. Usage: TAG=r01 bash tools/gpu/gpurun_measure.sh
set -o pipefail
TAG=${TAG:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py > $OUT/bench_cog.json 2> $OUT/bench_cog.err
rc=$?; echo "bench cog rc=$rc"; cat $OUT/bench_cog.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python bench.py --variant wan > $OUT/bench_wan.json 2> $OUT/bench_wan.err
rc=$?; echo "bench wan rc=$rc"; cat $OUT/bench_wan.json
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-pmc > $OUT/prof_bench.json 2> $OUT/prof_bench.err
rc=$?; echo "rocprof rc=$rc"
f=$(find $OUT/prof -name "*kernel_stats.csv" | head -1); head -12 "$f"
