set -o pipefail
O=gpurun_out/r05_c8
mkdir -p $O
timeout -k 10 200 python tools/diag/pred_trace.py cog attn > $O/atrace_cog.log 2>&1 && \
timeout -k 10 200 python tools/diag/pred_trace.py wan attn > $O/atrace_wan.log 2>&1
rc=$?; cat $O/*.log | grep -v amdgpu.ids; exit $rc
