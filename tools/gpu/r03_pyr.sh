set -o pipefail
OUT=gpurun_out/r03_pyr; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_multilevel.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 300 python tools/ml_ab.py > $OUT/ml_ab.log 2>&1; rc=$?; grep -v amdgpu $OUT/ml_ab.log | tail -8; exit $rc
