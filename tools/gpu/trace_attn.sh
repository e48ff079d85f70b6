#!/bin/bash
# Attention residency traces (VB_ATTN_TRACE build variant "atrace"), persistent and one-workgroup-per-q-block launches
set -o pipefail
O=gpurun_out/${TAG:-trace_attn}
mkdir -p $O
for v in cog wan; do
  for pz in 1 0; do
    TRACE_PERSIST=$pz timeout -k 10 300 python -u tools/diag/pred_trace.py $v attn atrace > $O/trace_${v}_p$pz.log 2>&1 || exit 1
    grep -E "traced|duration|mean residency|per CU min" $O/trace_${v}_p$pz.log
  done
done
