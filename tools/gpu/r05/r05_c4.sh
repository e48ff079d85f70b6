set -o pipefail
O=gpurun_out/r05_c4
mkdir -p $O
timeout -k 10 300 python tools/ab.py base l3k64 l3k64w5 l3k64w5p512 late3 --what pred --variant cog > $O/pred.log 2>&1 && \
timeout -k 10 300 python tools/ab.py base l3k64 l3k64w5 l3k64w5p512 late3 --what call --variant cog > $O/call.log 2>&1
rc=$?; grep -h -E "median|identical" $O/*.log; exit $rc
