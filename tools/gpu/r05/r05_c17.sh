set -o pipefail
O=gpurun_out/r05_c17
mkdir -p $O
VBLADE_LIB=$PWD/video-blade_amd/vblade/variants/lib_dq64r2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread > $O/pytest_bwd_dq64r2.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur dq64r2 dq64r2w2 cur dq64r2 dq64r2w2 --what bwd --variant cog > $O/bwd_cog.log 2>&1
rc=$?; tail -n 2 $O/pytest_bwd_dq64r2.log; grep -h -E "median" $O/*.log; exit $rc
