set -o pipefail
O=gpurun_out/r05_c23
mkdir -p $O
VBLADE_LIB=$PWD/video-blade_amd/vblade/variants/lib_sum16.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest_sum16.log 2>&1; rc1=$?
# only assertion failures (pytest exit 1) may go on to the timing; a fault, abort or time limit ends here
if [ $rc1 -ne 0 ] && [ $rc1 -ne 1 ]; then tail -n 5 $O/pytest_sum16.log; exit $rc1; fi
timeout -k 10 300 python tools/ab.py cur sum16 cur sum16 --what attn --variant cog > $O/attn.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur sum16 --what call --variant cog > $O/call.log 2>&1
rc=$?; tail -n 3 $O/pytest_sum16.log; grep -E "FAIL|Error|assert" $O/pytest_sum16.log | head -5; grep -h -E "median|identical|diff" $O/*.log; exit $rc
