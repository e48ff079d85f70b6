set -o pipefail
O=gpurun_out/r05_c26
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 200 --timeout-method thread > $O/pytest_fwd.log 2>&1
rc=$?; tail -n 3 $O/pytest_fwd.log; grep -E "Error|assert" $O/pytest_fwd.log | head -5; exit $rc
