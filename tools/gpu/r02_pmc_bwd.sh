#!/bin/bash
# PMC counter passes on the training-path backward kernels (kbench --only-bwd), one pass per group
set -o pipefail
OUT=gpurun_out/r02_pmc_bwd
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" \
           "SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_FLAT" ; do
  i=$((i+1))
  rm -rf $OUT/p$i
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $OUT/p$i -o run -- python3 tools/kbench.py --only-bwd --variant ${VAR:-cog} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
for k in bwd_dq_kernel "bwd_dkdv_kernel<64, vb::BF16, false" "bwd_dkdv_kernel<64, vb::BF16, true" "bwd_dkdv_kernel<128, vb::BF16, false" bwd_prep; do
  echo "## $k"; python3 tools/pmc_summary.py $OUT "$k"
done
