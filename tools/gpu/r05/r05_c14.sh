set -o pipefail
O=gpurun_out/r05_c14
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_forward.py -x -q --timeout 120 --timeout-method thread -k "longest_first" > $O/pytest_fwd.log 2>&1 && \
VB_BWD_DQ128=1 VB_BWD_DQ128_RING=2 timeout -k 10 400 python -u -m pytest tests/test_gpu_backward.py -x -q --timeout 120 --timeout-method thread > $O/pytest_bwd_dq2.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur dq4 dq2 dq2l3 kvslp allns --what bwd --variant wan > $O/bwd_wan.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur kvslp allns --what bwd --variant cog > $O/bwd_cog.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur@noorder cur cur@noorder cur --what attn --variant both > $O/attn.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur@noorder cur allns --what call --variant both > $O/call.log 2>&1
rc=$?; tail -n 2 $O/pytest_fwd.log $O/pytest_bwd_dq2.log; grep -h -E "median" $O/*.log; exit $rc
