set -o pipefail
O=gpurun_out/r05_c9
mkdir -p $O
timeout -k 10 300 python tools/ab.py base cur base cur --what attn --variant both > $O/attn.log 2>&1 && \
timeout -k 10 300 python tools/ab.py base cur --what call --variant both > $O/call.log 2>&1 && \
timeout -k 10 300 python tools/ab.py base cur --what fwdlse --variant cog > $O/fwdlse.log 2>&1
rc=$?; grep -h -E "median|identical" $O/*.log; exit $rc
