set -o pipefail
O=gpurun_out/r05_c30
mkdir -p $O
timeout -k 10 300 python tools/ab.py cur dqp1 dqp2 cur dqp1 dqp2 --what bwd --variant both > $O/bwd.log 2>&1
rc=$?; grep -h -E "median" $O/*.log; exit $rc
