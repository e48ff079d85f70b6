# Pool/pyramid pass: rows entries pipelined one step ahead (vb_pool.hpp, vb_pyr.hpp). Parity of the
# pooled and pyramid passes, then A/B of the whole call against the round-5 base.
set -o pipefail
O=gpurun_out/r05_c34
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_module.py tests/test_gpu_multilevel.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head -8; exit $rc; }
timeout -k 10 300 python -u tools/ab.py pbase cur --what call --variant both > $O/ab_call.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab.py pbase cur --what pred --variant both > $O/ab_pred.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab.py pbase cur --what mlcall --variant cog > $O/ab_mlcall.log 2>&1 || exit $?
tail -n 4 $O/ab_call.log $O/ab_pred.log $O/ab_mlcall.log
