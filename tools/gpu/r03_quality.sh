set -o pipefail
OUT=gpurun_out/r03_quality; mkdir -p $OUT
timeout -k 10 700 python tools/quality_decomp.py --out $OUT/quality_decomp.json > $OUT/qd.log 2>&1; rc=$?; tail -2 $OUT/qd.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_fullsize.py -x -v --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -15 $OUT/pytest.log; exit $rc
