set -o pipefail
O=gpurun_out/r05_c31
mkdir -p $O
timeout -k 10 300 python tools/ab.py cur kvp1 kvp2 cur kvp1 kvp2 --what bwd --variant cog > $O/bwd.log 2>&1
rc=$?; grep -h -E "median" $O/*.log; exit $rc
