#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02_ml
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_multilevel.py -m gpu -q --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab.py m0 m1 m0 m1 --what mlbwd --variant cog --rounds 6 > $OUT/ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $OUT/ab.txt
exit $rc
