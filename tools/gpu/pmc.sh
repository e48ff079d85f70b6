#!/bin/bash
# PMC counter passes (one rocprofv3 --pmc pass per counter group) on tools/attn_only.py
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT" ; do
  i=$((i+1))
  rm -rf gpurun_out/pmc/p$i
  timeout -k 10 300 rocprofv3 --pmc $set --output-format csv -d gpurun_out/pmc/p$i -o run -- python3 tools/attn_only.py ${PMC_VARIANT:-cog} 3 ${PMC_WHAT:-attn} > gpurun_out/pmc/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 tools/pmc_summary.py gpurun_out/pmc ${PMC_KERNEL:-attn_fwd}
