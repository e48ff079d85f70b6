set -o pipefail
O=gpurun_out/r05_c12
mkdir -p $O
timeout -k 10 300 python tools/ab.py cur@noorder cur@win:64 cur@win:128 cur@win:256 cur --what attn --variant both > $O/attn.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur@noorder cur@win:128 cur --what call --variant cog > $O/call.log 2>&1
rc=$?; grep -h -E "median" $O/attn.log $O/call.log; exit $rc
