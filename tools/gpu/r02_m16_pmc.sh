#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02_m16_pmc
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for tag in f0 m1; do
 for set in "SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"; do
  i=$((i+1))
  VBLADE_LIB=$PWD/video-blade_amd/vblade/variants/lib_$tag.so timeout -k 10 -s KILL 200 rocprofv3 --pmc $set --output-format csv -d $OUT/$tag/p$i -o run -- python3 tools/attn_only.py cog 3 attn > $OUT/$tag.p$i.log 2>&1
  rc=$?; echo "$tag pass $i rc=$rc"; [ $rc -eq 0 ] || exit $rc
 done
 echo "## $tag"; python3 tools/pmc_summary.py $OUT/$tag attn_fwd
done
