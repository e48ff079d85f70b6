set -o pipefail
O=gpurun_out/r05_c29
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 200 --timeout-method thread -k "order" > $O/pytest_order.log 2>&1
rc=$?; tail -n 3 $O/pytest_order.log; grep -E "Error|assert" $O/pytest_order.log | head -8; exit $rc
