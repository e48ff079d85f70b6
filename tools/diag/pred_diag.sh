#!/bin/bash
# Predictor time decomposition with the diagnostic build (tools/build_variant.sh diag, VB_DIAG=1):
# VB_DEBUG_PRED = 0 full, 1 no epilogue, 4 K stream + epilogue (no MFMA/row max), 5 K stream only,
# 2 no main loop (prologue + epilogue).
set -o pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pred_diag
mkdir -p $OUT
for var in cog wan; do
  for d in 0 1 4 5 2; do
    rm -rf $OUT/p_${var}_$d
    VB_DEBUG_PRED=$d timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/p_${var}_$d -o run --output-format csv -- python3 tools/diag/pred_prof.py diag $var pred > $OUT/p_${var}_$d.log 2>&1
    rc=$?; [ $rc -eq 0 ] || { echo "fail $var $d rc=$rc"; tail -5 $OUT/p_${var}_$d.log; exit $rc; }
    echo "$var dbg=$d: $(grep mask_predict $OUT/p_${var}_$d/run_kernel_stats.csv | cut -d, -f2,4 | head -2 | tr '\n' ' ')"
  done
done
