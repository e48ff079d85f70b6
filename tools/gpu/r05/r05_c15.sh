set -o pipefail
O=gpurun_out/r05_c15
mkdir -p $O
timeout -k 10 300 python tools/ab.py cur bwdns cur bwdns --what mlbwd --variant cog > $O/mlbwd.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur bwdns --what bwd --variant both > $O/bwd.log 2>&1 && \
TAG=r05_c15/m NO_TRAIN=1 bash tools/gpu/measure.sh
rc=$?; grep -h -E "median" $O/*.log; exit $rc
