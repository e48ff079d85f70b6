set -o pipefail
O=gpurun_out/r05_c28
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_backward.py -x -q --timeout 200 --timeout-method thread > $O/pytest_bwd.log 2>&1
rc=$?; tail -n 3 $O/pytest_bwd.log; grep -E "Error|assert" $O/pytest_bwd.log | head -5; exit $rc
