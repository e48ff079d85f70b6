# Pipelined pool pass: pooling-workgroup sweep per head dim (wanN: N at D=128; cog512: 512 at D=64).
set -o pipefail
O=gpurun_out/r05_c37
mkdir -p $O
timeout -k 10 400 python -u tools/ab.py pbase cur wan128 wan192 wan320 --what call --variant wan --rounds 25 > $O/ab_wan.log 2>&1 || exit $?
timeout -k 10 400 python -u tools/ab.py pbase cur nt1 w192 cog512 --what call --variant cog --rounds 25 > $O/ab_cog.log 2>&1 || exit $?
grep "median" $O/ab_wan.log $O/ab_cog.log
