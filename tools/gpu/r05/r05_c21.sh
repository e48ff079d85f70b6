set -o pipefail
O=gpurun_out/r05_c21
mkdir -p $O
VBLADE_LIB=$PWD/video-blade_amd/vblade/variants/lib_kve.so timeout -k 10 400 python -u -m pytest tests/test_gpu_backward.py tests/test_gpu_multilevel.py -x -q --timeout 120 --timeout-method thread > $O/pytest_kve.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur kve cur kve --what bwd --variant both > $O/bwd.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur kve --what mlbwd --variant cog > $O/mlbwd.log 2>&1
rc=$?; tail -n 2 $O/pytest_kve.log; grep -h -E "median" $O/*.log; exit $rc
