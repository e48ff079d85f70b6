set -o pipefail
O=gpurun_out/r05_c5
mkdir -p $O
timeout -k 10 200 python tools/diag/pred_trace.py cog pred > $O/trace_cog_pred.log 2>&1 && \
timeout -k 10 200 python tools/diag/pred_trace.py cog call > $O/trace_cog_call.log 2>&1 && \
timeout -k 10 200 python tools/diag/pred_trace.py wan call > $O/trace_wan_call.log 2>&1 && \
timeout -k 10 300 python tools/ab.py base q2p384 q2p160 q2p256 q2l3p160 --what call --variant cog > $O/call.log 2>&1 && \
timeout -k 10 300 python tools/ab.py base q2p384 q2p160 q2l3p160 --what pred --variant cog > $O/pred.log 2>&1
rc=$?; cat $O/trace*.log | grep -v amdgpu.ids; grep -h -E "median|identical" $O/call.log $O/pred.log; exit $rc
