#!/bin/bash
# Round 2 baseline of the current tree: whole -m gpu suite, then kernel-trace summaries of the
# bench (cog, wan) and of the backward (kbench --bwd, both workloads).
set -o pipefail
OUT=gpurun_out/r02_base
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
for var in cog wan; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$var -o run --output-format csv -- python3 bench.py --variant $var --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-pmc > $OUT/bench_$var.json 2> $OUT/bench_$var.err
  rc=$?; echo "bench $var rc=$rc"; cat $OUT/bench_$var.json | cut -c1-400
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_bwd -o run --output-format csv -- python3 tools/kbench.py --bwd > $OUT/kbench_bwd.log 2>&1
rc=$?; echo "kbench bwd rc=$rc"; grep -v amdgpu.ids $OUT/kbench_bwd.log | tail -4
python3 tools/kstats.py $OUT/prof_cog $OUT/prof_wan $OUT/prof_bwd
exit $rc
