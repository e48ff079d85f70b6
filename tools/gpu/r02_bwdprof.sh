#!/bin/bash
# kernel trace of the backward (both workloads) + PMC issue/MFMA counters of its kernels (cog)
set -o pipefail
OUT=gpurun_out/${TAG:-r02_bwdprof}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 tools/kbench.py --only-bwd > $OUT/kbench.log 2>&1
rc=$?; echo "trace rc=$rc"; grep -v amdgpu.ids $OUT/kbench.log | grep bwd
[ $rc -eq 0 ] || exit $rc
python3 tools/kstats.py $OUT/trace | grep -E "bwd|pool_grad"
i=0
for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
           "SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" ; do
  i=$((i+1))
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc/p$i -o run -- python3 tools/kbench.py --only-bwd --variant ${VAR:-cog} > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
for k in bwd_dq_kernel "bwd_dkdv_kernel<64, vb::BF16, false" "bwd_dkdv_kernel<64, vb::BF16, true"; do
  echo "## $k"; python3 tools/pmc_summary.py $OUT/pmc "$k"
done
