#!/bin/bash
# effective clock and issue-busy counters of the attention kernel (one --pmc pass per group)
mkdir -p gpurun_out/clock
export TMPDIR=/tmp
i=0
for set in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $set --kernel-trace --output-format csv -d gpurun_out/clock/p$i -o run -- python3 tools/attn_only.py ${VAR:-cog} 5 attn > gpurun_out/clock/p$i.log 2>&1 || { echo "pass $i failed"; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/clock attn_fwd
f=$(find gpurun_out/clock/p1 -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv,sys
rows=[r for r in csv.DictReader(open(sys.argv[1])) if 'attn_fwd' in r['Kernel_Name']]
d=[(int(r['End_Timestamp'])-int(r['Start_Timestamp'])) for r in rows]
print('attn launches', len(d), 'avg ns', sum(d)/len(d))
PY
