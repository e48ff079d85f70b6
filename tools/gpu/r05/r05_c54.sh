# Multi-level call: the pyramid pass's K/V reads non-temporal (pyrnt) vs plain (cur)
set -o pipefail
O=gpurun_out/r05_c54
mkdir -p $O
timeout -k 10 300 python -u tools/ab.py cur pyrnt --what mlcall --variant cog --rounds 25 > $O/ab1.log 2>&1 || exit $?
timeout -k 10 300 python -u tools/ab.py cur pyrnt --what mlcall --variant cog --rounds 25 > $O/ab2.log 2>&1 || exit $?
grep -h median $O/ab1.log $O/ab2.log
