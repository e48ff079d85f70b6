#!/bin/bash
# PMC counter passes on the forward attention kernel (tools/attn_only.py), one pass per group
set -o pipefail
OUT=gpurun_out/r02_pmc_fwd_${PMC_VARIANT:-cog}
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT" \
           "SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32" ; do
  i=$((i+1))
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 tools/attn_only.py ${PMC_VARIANT:-cog} 3 attn > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || { tail -5 $OUT/p$i.log; exit $rc; }
done
python3 tools/pmc_summary.py $OUT attn_fwd_kernel
