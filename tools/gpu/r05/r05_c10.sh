set -o pipefail
O=gpurun_out/r05_c10
mkdir -p $O
TRACE_OUT=$O/atrace_cog.npy timeout -k 10 200 python tools/diag/pred_trace.py cog attn > $O/atrace_cog.log 2>&1 && \
TRACE_OUT=$O/atrace_wan.npy timeout -k 10 200 python tools/diag/pred_trace.py wan attn > $O/atrace_wan.log 2>&1 && \
TRACE_OUT=$O/ptrace_cog.npy timeout -k 10 200 python tools/diag/pred_trace.py cog pred > $O/ptrace_cog.log 2>&1
rc=$?; cat $O/*.log | grep -v amdgpu.ids; exit $rc
