set -o pipefail
O=gpurun_out/r05_c22
mkdir -p $O
VBLADE_LIB=$PWD/video-blade_amd/vblade/variants/lib_dqs5.so timeout -k 10 400 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_multilevel.py -x -q --timeout 120 --timeout-method thread > $O/pytest_dqs5.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur dqs3 dqs5 cur dqs3 dqs5 --what bwd --variant both > $O/bwd.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur dqs3 dqs5 --what mlbwd --variant cog > $O/mlbwd.log 2>&1
rc=$?; tail -n 2 $O/pytest_dqs5.log; grep -h -E "median" $O/*.log; exit $rc
