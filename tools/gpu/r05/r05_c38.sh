# New defaults (pipelined pool pass, non-temporal K/V reads, 320 Wan pooling workgroups): the GPU
# suite, then A/B against the round-5 base.
set -o pipefail
O=gpurun_out/r05_c38
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -n 3 $O/pytest.log; [ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head -8; exit $rc; }
timeout -k 10 400 python -u tools/ab.py pbase cur --what call --variant both --rounds 25 > $O/ab_call.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab.py pbase cur --what mlcall --variant cog --rounds 25 > $O/ab_mlcall.log 2>&1 || exit $?
grep -h "median\|identical" $O/ab_call.log $O/ab_mlcall.log
