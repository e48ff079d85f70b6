#!/bin/bash
# Full measurement of the current tree: the GPU suite, smoke, the default bench line (PMC traffic,
# quality, points, backward, CPU baseline), kernel-trace summaries of the bench (cog, wan, cog-ml)
# and of the backward, and the training steps. Usage: TAG=name bash tools/gpu/measure.sh
set -o pipefail
OUT=gpurun_out/${TAG:-measure}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail $OUT/smoke.log; exit 1; }
timeout -k 10 900 python bench.py > $OUT/bench.json 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || { tail -20 $OUT/bench.err; exit $rc; }
for var in cog wan cog-ml; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$var -o run --output-format csv -- python3 bench.py --variant $var --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-pmc > $OUT/bench_$var.json 2> $OUT/bench_$var.err
  rc=$?; echo "prof $var rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_bwd -o run --output-format csv -- python3 tools/kbench.py --only-bwd > $OUT/kbench_bwd.log 2>&1
rc=$?; echo "prof bwd rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/kstats.py $OUT/prof_cog $OUT/prof_wan $OUT/prof_cog-ml $OUT/prof_bwd | grep -E "==|vb::" | head -40
[ -n "$NO_TRAIN" ] && exit 0
timeout -k 10 400 python tools/train_bench.py --batch 5 --accum 4 --layers 2 > $OUT/train.json 2> $OUT/train.err; rc=$?; echo "train rc=$rc"; cut -c1-300 $OUT/train.json; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python tools/train_bench.py --batch 5 --accum 4 --layers 2 --tdm > $OUT/train_tdm.json 2> $OUT/train_tdm.err; rc=$?; echo "tdm rc=$rc"; cut -c1-300 $OUT/train_tdm.json; exit $rc
