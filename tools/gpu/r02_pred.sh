#!/bin/bash
# Predictor diagnostics: time split (diag build), PMC counters of mask_predict_kernel (score only)
set -o pipefail
OUT=gpurun_out/r02_pred
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python tools/pred_split.py pdiag > $OUT/split.txt 2>&1
rc=$?; echo "split rc=$rc"; cat $OUT/split.txt
[ $rc -eq 0 ] || exit $rc
PMC_WHAT=pred PMC_KERNEL=mask_predict timeout -k 10 600 bash tools/gpu/gpurun_pmc.sh > $OUT/pmc.txt 2>&1
rc=$?; echo "pmc rc=$rc"; cat $OUT/pmc.txt
