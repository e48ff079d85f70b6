# Pooling workgroups dispatched after the score workgroups (VB_FUSED_POOL_LAST=1, 384/256 of them),
# now that the pass is pipelined: they can fill the score kernel's partial last round.
set -o pipefail
O=gpurun_out/r05_c39
mkdir -p $O
for v in cog wan; do for t in ptrace ptlast; do
  timeout -k 10 200 python -u tools/diag/pred_trace.py $v call $t > $O/trace_${v}_$t.log 2>&1 || exit $?
done; done
grep -h "call:\|pool :\|score:\|residency" $O/trace_*.log
timeout -k 10 400 python -u tools/ab.py cur last384 last256 --what call --variant both --rounds 25 > $O/ab_call.log 2>&1 || exit $?
grep -h "median" $O/ab_call.log
