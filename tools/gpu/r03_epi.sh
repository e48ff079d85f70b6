set -o pipefail
OUT=gpurun_out/r03_epi; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_module.py tests/test_gpu_forward.py tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 300 python tools/ab.py base epi base epi --what call > $OUT/ab_call.log 2>&1; rc=$?; grep -v amdgpu $OUT/ab_call.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/ab.py base epi --what pred > $OUT/ab_pred.log 2>&1; rc=$?; grep -v amdgpu $OUT/ab_pred.log | tail -6; exit $rc
