#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02_voff
mkdir -p $OUT
export TMPDIR=/tmp
VBLADE_LIB=$PWD/video-blade_amd/vblade/variants/lib_v1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_module.py tests/test_gpu_multilevel.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab.py v0 v1 v0 v1 v0 v1 --what attn --variant both --rounds 8 > $OUT/ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $OUT/ab.txt | grep -v "max|out"
exit $rc
