set -o pipefail
O=gpurun_out/r05_c33
mkdir -p $O
VBLADE_LIB=$PWD/video-blade_amd/vblade/variants/lib_pyr2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_multilevel.py -x -q --timeout 120 --timeout-method thread > $O/pytest_ml.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur pyr2 cur pyr2 --what mlbwd --variant cog > $O/mlbwd.log 2>&1
rc=$?; tail -n 2 $O/pytest_ml.log; grep -E "Error|assert" $O/pytest_ml.log | head -3; grep -h -E "median|identical" $O/mlbwd.log; exit $rc
