#!/bin/bash
# BASELINE config 5 geometry on one GPU: the LoRA training step (B=5 x accum 4) and the two-model TDM step
set -o pipefail
OUT=gpurun_out/r02_train
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python tools/train_bench.py --layers 2 --batch 5 --accum 4 --steps 2 --warmup 1 > $OUT/train.json 2> $OUT/train.err
rc=$?; echo "train rc=$rc"; cat $OUT/train.json; [ $rc -eq 0 ] || { tail -5 $OUT/train.err; exit $rc; }
timeout -k 10 500 python tools/train_bench.py --tdm --layers 2 --batch 5 --accum 4 --steps 2 --warmup 1 > $OUT/tdm.json 2> $OUT/tdm.err
rc=$?; echo "tdm rc=$rc"; cat $OUT/tdm.json; [ $rc -eq 0 ] || tail -5 $OUT/tdm.err
exit $rc
