#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02_b78
mkdir -p $OUT
export TMPDIR=/tmp
for tag in b7 b8; do
  VBLADE_LIB=$PWD/video-blade_amd/vblade/variants/lib_$tag.so timeout -k 10 600 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_train.py -m gpu -q --timeout 240 --timeout-method thread > $OUT/pytest_$tag.log 2>&1
  rc=$?; echo "pytest $tag rc=$rc"; tail -3 $OUT/pytest_$tag.log
  [ $rc -le 1 ] || exit $rc
done
timeout -k 10 400 python tools/ab.py b6 b7 b8 b6 b7 b8 --what bwd --rounds 6 > $OUT/ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $OUT/ab.txt
exit $rc
