# gather_kv re-measured with the pipelined pool pass (copies now cost HBM time, not latency)
set -o pipefail
O=gpurun_out/r05_c40
mkdir -p $O
timeout -k 10 300 python -u tools/diag/overlap_ab.py --opt gather_kv > $O/gather1.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/diag/overlap_ab.py --opt gather_kv > $O/gather2.log 2>&1 || exit $?
grep -h median $O/gather1.log $O/gather2.log
