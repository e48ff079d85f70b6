#!/bin/bash
# Predictor-alone and per-call A/B of library variants: AB="base new ..." bash tools/gpu/ab_pred.sh
set -o pipefail
OUT=gpurun_out/ab_pred
mkdir -p $OUT
timeout -k 10 400 python tools/ab.py ${AB} --what pred --variant both > $OUT/pred.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/pred.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab.py ${AB} --what call --variant both > $OUT/call.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/call.log; exit $rc
