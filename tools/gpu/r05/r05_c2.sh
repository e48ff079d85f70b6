set -o pipefail
O=gpurun_out/r05_c2
mkdir -p $O
timeout -k 10 300 python tools/ab.py base cur s1 s2 s4 n7s1 w7p128 k64 --what pred --variant cog > $O/pred_cog.log 2>&1; echo "pred cog rc=$?"
timeout -k 10 300 python tools/ab.py base cur s1 s2 s4 n7s1 w7p128 --what call --variant cog > $O/call_cog.log 2>&1; echo "call cog rc=$?"
timeout -k 10 300 python tools/ab.py base cur --what pred --variant wan > $O/pred_wan.log 2>&1; echo "pred wan rc=$?"
timeout -k 10 300 python tools/ab.py base cur --what call --variant wan > $O/call_wan.log 2>&1; echo "call wan rc=$?"
grep -h -E "median|identical" $O/*.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_forward.py tests/test_gpu_module.py -x -q --timeout 120 --timeout-method thread > $O/pytest_pred.log 2>&1
rc=$?; tail -3 $O/pytest_pred.log; exit $rc
