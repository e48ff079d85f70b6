#!/bin/bash
# Round evidence on the GPU box: rocprofv3 kernel-trace summaries of the bench's three workloads
# and of the backward, then PMC counter passes (one rocprofv3 --pmc run per counter set) on the
# forward (CogVideoX, Wan) and on the backward. Usage: TAG=r04_x bash tools/gpu/evidence.sh
set -o pipefail
OUT=gpurun_out/${TAG:-evidence}
mkdir -p $OUT
export TMPDIR=/tmp
for var in cog wan cog-ml; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_$var -o run --output-format csv -- python3 bench.py --variant $var --steps 2 --warmup 1 --no-cpu-baseline --no-extras --no-pmc > $OUT/bench_$var.json 2> $OUT/bench_$var.err
  rc=$?; echo "trace $var rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_bwd -o run --output-format csv -- python3 tools/kbench.py --only-bwd > $OUT/kbench_bwd.log 2>&1
rc=$?; echo "trace bwd rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/kstats.py $OUT/prof_cog $OUT/prof_wan $OUT/prof_cog-ml $OUT/prof_bwd | grep -E "==|vb::" | head -40
SETS=("SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY"
      "SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
      "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS")
run_pmc() {   # name, kernel substring, command...
  local name=$1 pat=$2; shift 2
  local i=0
  for set in "${SETS[@]}"; do
    i=$((i+1))
    rm -rf $OUT/pmc_$name/p$i
    timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc_$name/p$i -o run -- "$@" > $OUT/pmc_$name/p$i.log 2>&1
    rc=$?; echo "pmc $name pass $i rc=$rc"; [ $rc -eq 0 ] || return $rc
  done
  python3 tools/pmc_summary.py $OUT/pmc_$name $pat > $OUT/pmc_$name.txt
}
mkdir -p $OUT/pmc_fwd_cog $OUT/pmc_fwd_wan $OUT/pmc_bwd_cog $OUT/pmc_bwd_wan
run_pmc fwd_cog attn_fwd_kernel python3 tools/attn_only.py cog 3 attn || exit 1
run_pmc fwd_wan attn_fwd_kernel python3 tools/attn_only.py wan 3 attn || exit 1
run_pmc bwd_cog bwd_ python3 tools/kbench.py --only-bwd --variant cog || exit 1
run_pmc bwd_wan bwd_ python3 tools/kbench.py --only-bwd --variant wan || exit 1
for f in $OUT/pmc_*.txt; do echo "== $f"; cat $f; done
