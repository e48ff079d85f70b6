#!/bin/bash
# Backward kernel trace + PMC passes for one variant (default wan) on the GPU box.
# Usage: TAG=r04_kv VAR=wan bash tools/gpu/bwd_prof.sh
set -o pipefail
OUT=gpurun_out/${TAG:-bwdprof}
VAR=${VAR:-wan}
mkdir -p $OUT/pmc_bwd_$VAR
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_bwd_$VAR -o run --output-format csv -- python3 tools/kbench.py --only-bwd --variant $VAR > $OUT/kbench_bwd_$VAR.log 2>&1
rc=$?; echo "trace rc=$rc"; [ $rc -eq 0 ] || exit $rc
grep -h "bwd=" $OUT/kbench_bwd_$VAR.log
python3 tools/kstats.py $OUT/prof_bwd_$VAR | grep -E "==|vb::" | head -12
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
      "SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
      "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS")
[ -n "$NO_PMC" ] && exit 0
i=0
for set in "${SETS[@]}"; do
  i=$((i+1))
  rm -rf $OUT/pmc_bwd_$VAR/p$i
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc_bwd_$VAR/p$i -o run -- python3 tools/kbench.py --only-bwd --variant $VAR > $OUT/pmc_bwd_$VAR/p$i.log 2>&1
  rc=$?; echo "pmc pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py $OUT/pmc_bwd_$VAR bwd_ > $OUT/pmc_bwd_$VAR.txt
cat $OUT/pmc_bwd_$VAR.txt
