set -o pipefail
O=gpurun_out/r05_c3
mkdir -p $O
timeout -k 10 300 python tools/ab.py base late3 b3 cur --what pred --variant both > $O/pred.log 2>&1 && \
timeout -k 10 300 python tools/ab.py base late3 b3 --what call --variant both > $O/call.log 2>&1
rc=$?; grep -h -E "median|identical" $O/*.log; exit $rc
