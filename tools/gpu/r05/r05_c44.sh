# Split of the gathered-K/V attention cost: code path vs memory pattern (tools/diag/gather_cost.py)
set -o pipefail
O=gpurun_out/r05_c44
mkdir -p $O
timeout -k 10 300 python -u tools/diag/gather_cost.py cog > $O/cog.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/diag/gather_cost.py wan > $O/wan.log 2>&1 || exit $?
grep -h "attn\|identical" $O/cog.log $O/wan.log
