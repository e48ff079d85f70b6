set -o pipefail
O=gpurun_out/r05_c25
mkdir -p $O
VBLADE_LIB=$PWD/video-blade_amd/vblade/variants/lib_kla2.so timeout -k 10 400 python -u -m pytest tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread > $O/pytest_kla2.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur kla2 kla3 cur kla2 kla3 --what bwd --variant both > $O/bwd.log 2>&1
rc=$?; tail -n 2 $O/pytest_kla2.log; grep -h -E "median" $O/*.log; exit $rc
