#!/bin/bash
# ping-pong forward: parity through the module/forward tests on the variant library, then A/B
set -o pipefail
OUT=gpurun_out/r02_pp
mkdir -p $OUT
export TMPDIR=/tmp
VBLADE_LIB=$PWD/video-blade_amd/vblade/variants/lib_p1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_module.py tests/test_gpu_config1.py -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -15 $OUT/pytest.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/ab.py f0 p1 p2 f0 p1 p2 --what attn --variant cog --rounds 6 > $OUT/ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $OUT/ab.txt
exit $rc
