#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02_o
mkdir -p $OUT
export TMPDIR=/tmp
VBLADE_LIB=$PWD/video-blade_amd/vblade/variants/lib_${OTAG:-m1}.so timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_module.py tests/test_gpu_config1.py -m gpu -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" $OUT/pytest.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 400 python tools/ab.py f0 ${OTAGS:-m1} f0 ${OTAGS:-m1} --what attn --variant cog --rounds 6 > $OUT/ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $OUT/ab.txt
timeout -k 10 400 python tools/ab.py f0 ${OTAGS:-m1} f0 ${OTAGS:-m1} --what call --variant cog --rounds 6 > $OUT/ab_call.txt 2>&1
rc=$?; echo "ab call rc=$rc"; grep -v amdgpu.ids $OUT/ab_call.txt
exit $rc
