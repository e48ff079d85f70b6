#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02_b10
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_train.py -m gpu -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab.py bprev b10 bprev b10 --what bwd --rounds 6 > $OUT/ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $OUT/ab.txt
exit $rc
