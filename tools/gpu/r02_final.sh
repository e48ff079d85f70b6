#!/bin/bash
# Round-2 measurement of the current tree: the full bench line (all extras: PMC traffic, quality,
# density/Wan points, backward, CPU baseline), then kernel-trace summaries of the bench (cog, wan),
# of the backward and of the multi-level path.
set -o pipefail
OUT=gpurun_out/${TAG:-r02_final}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; cut -c1-600 $OUT/bench.json
[ $rc -eq 0 ] || { tail -20 $OUT/bench.err; exit $rc; }
for var in cog wan cog-ml; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$var -o run --output-format csv -- python3 bench.py --variant $var --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-pmc > $OUT/bench_$var.json 2> $OUT/bench_$var.err
  rc=$?; echo "prof $var rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_bwd -o run --output-format csv -- python3 tools/kbench.py --only-bwd > $OUT/kbench_bwd.log 2>&1
rc=$?; echo "prof bwd rc=$rc"; grep bwd $OUT/kbench_bwd.log | grep -v amdgpu
python3 tools/kstats.py $OUT/prof_cog $OUT/prof_wan $OUT/prof_cog-ml $OUT/prof_bwd | grep -E "==|vb::"
exit $rc
