#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02_b9
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_train.py tests/test_gpu_multilevel.py -m gpu -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
