set -o pipefail
O=gpurun_out/r05_c24
mkdir -p $O
timeout -k 10 300 python tools/diag/overlap_ab.py --opt gather_kv > $O/gather.log 2>&1 && \
timeout -k 10 300 python tools/diag/overlap_ab.py --opt gather_kv > $O/gather2.log 2>&1
rc=$?; cat $O/gather.log $O/gather2.log | grep median; exit $rc
