set -o pipefail
O=gpurun_out/r05_c18
mkdir -p $O
timeout -k 10 300 python tools/ab.py cur st12 st24 st48 cur st12 st24 st48 --what pred --variant both > $O/pred.log 2>&1 && \
timeout -k 10 300 python tools/ab.py cur st12 st24 st48 --what call --variant cog > $O/call.log 2>&1
rc=$?; grep -h -E "median|identical" $O/*.log; exit $rc
