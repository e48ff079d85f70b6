#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02_p10
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_module.py -x -q --timeout 240 --timeout-method thread > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab.py base q3 q4 p10 --what pred > $OUT/ab_pred.txt 2>&1
rc=$?; echo "ab pred rc=$rc"; grep -v amdgpu.ids $OUT/ab_pred.txt
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab.py base q3 q4 p10 base q3 q4 p10 --what call > $OUT/ab_call.txt 2>&1
rc=$?; echo "ab call rc=$rc"; grep -v amdgpu.ids $OUT/ab_call.txt
