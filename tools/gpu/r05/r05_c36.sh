# Pipelined pool pass: non-temporal K/V reads (nt1) / and copy stores (nt2), fewer pooling
# workgroups (w192: 192 CogVideoX / 256 Wan; w256: 256 / 384), vs the round-5 base and cur.
set -o pipefail
O=gpurun_out/r05_c36
mkdir -p $O
timeout -k 10 400 python -u tools/ab.py pbase cur nt1 nt2 w192 w256 --what call --variant both > $O/ab_call.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab.py pbase cur nt1 nt2 w192 w256 --what mlcall --variant cog > $O/ab_mlcall.log 2>&1 || exit $?
grep "median" $O/ab_call.log $O/ab_mlcall.log
