#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02_q5
mkdir -p $OUT
export TMPDIR=/tmp
true
rc=0
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab.py base q5 --what pred > $OUT/ab_pred.txt 2>&1
rc=$?; echo "ab pred rc=$rc"; grep -v amdgpu.ids $OUT/ab_pred.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab.py base q4 q5 p10 base q4 q5 p10 --what call > $OUT/ab_call.txt 2>&1
rc=$?; echo "ab call rc=$rc"; grep -v amdgpu.ids $OUT/ab_call.txt
