# New pooled-pass pipeline test (gaps around the group size, with/without rows, multi-item threads)
set -o pipefail
O=gpurun_out/r05_c43
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 200 --timeout-method thread -k "pool" > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head -8; exit $rc; }
