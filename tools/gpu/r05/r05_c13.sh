set -o pipefail
O=gpurun_out/r05_c13
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 120 --timeout-method thread -k "longest_first" > $O/pytest.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur@noorder cur cur@noorder cur --what attn --variant both > $O/attn.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur@noorder cur --what call --variant wan > $O/call.log 2>&1
rc=$?; tail -2 $O/pytest.log; grep -h -E "median" $O/attn.log $O/call.log; exit $rc
