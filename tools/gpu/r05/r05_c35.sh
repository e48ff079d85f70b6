# Predictor-launch timeline (trace builds) with the pipelined pool pass vs the round-5 base.
set -o pipefail
O=gpurun_out/r05_c35
mkdir -p $O
for v in cog wan; do for t in ptbase ptrace; do
  timeout -k 10 200 python -u tools/diag/pred_trace.py $v call $t > $O/trace_${v}_$t.log 2>&1 || exit $?
done; done
grep -h "call:\|pool :\|score:\|residency" $O/trace_*.log
