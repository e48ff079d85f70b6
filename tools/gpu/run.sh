#!/bin/bash
# One GPU call made of named steps, each under its own time limit, stopping at the first failure.
# Replaces the one-shot per-call scripts of earlier rounds.
#   TAG=name bash tools/gpu/run.sh 'STEP' ['STEP' ...]
# A STEP is one of
#   pytest ARGS...   python -u -m pytest -x -v --timeout 200 --timeout-method thread ARGS
#   ab ARGS...       python -u tools/ab.py ARGS                 (library/option A/B, one process)
#   bench ARGS...    python bench.py ARGS                       (the JSON line to STEPn.json)
#   trace NAME CMD   rocprofv3 --kernel-trace --stats of CMD into $OUT/prof_NAME, then kstats
#   pmc NAME KERNEL CMD  the counter passes of tools/gpu/pmc.sh on CMD, summary for KERNEL
#   anything else    run as given
# Outputs: gpurun_out/$TAG/stepN.log (and .json for bench); the summary lines are printed.
set -o pipefail
OUT=gpurun_out/${TAG:-run}
mkdir -p $OUT
export TMPDIR=/tmp
LIMIT=${LIMIT:-600}
n=0
for step in "$@"; do
  n=$((n+1))
  log=$OUT/step$n.log
  echo "== step $n: $step"
  set -- $step
  kind=$1; shift
  case $kind in
    pytest) timeout -k 10 $LIMIT python -u -m pytest -x -v --timeout 200 --timeout-method thread "$@" > $log 2>&1
            rc=$?; tail -2 $log; [ $rc -eq 0 ] || grep -E "^(FAILED|ERROR)|Error|assert" $log | head -12 ;;
    ab)     timeout -k 10 $LIMIT python -u tools/ab.py "$@" > $log 2>&1
            rc=$?; grep -v amdgpu.ids $log | grep -E "median|identical|Error|error" ;;
    bench)  timeout -k 10 $LIMIT python bench.py "$@" > $OUT/step$n.json 2> $log
            rc=$?; cut -c1-600 $OUT/step$n.json; [ $rc -eq 0 ] || tail -5 $log ;;
    trace)  name=$1; shift
            timeout -k 10 $LIMIT rocprofv3 --kernel-trace --stats -d $OUT/prof_$name -o run --output-format csv -- "$@" > $log 2>&1
            rc=$?; [ $rc -eq 0 ] && python3 tools/kstats.py $OUT/prof_$name | grep -E "==|vb::" | head -16 ;;
    pmc)    name=$1 pat=$2; shift 2
            i=0; rc=0
            for set in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY" \
                       "SQ_ACTIVE_INST_VALU SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
                       "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS" \
                       "FETCH_SIZE" "WRITE_SIZE"; do
              i=$((i+1)); rm -rf $OUT/pmc_$name/p$i
              timeout -k 10 -s KILL 120 rocprofv3 --pmc $set --output-format csv -d $OUT/pmc_$name/p$i -o run -- "$@" > $OUT/pmc_$name.p$i.log 2>&1
              rc=$?; [ $rc -eq 0 ] || { echo "pmc pass $i rc=$rc"; break; }
            done
            [ $rc -eq 0 ] && python3 tools/pmc_summary.py $OUT/pmc_$name $pat | tee $OUT/pmc_$name.txt | head -30 ;;
    *)      timeout -k 10 $LIMIT "$kind" "$@" > $log 2>&1
            rc=$?; tail -5 $log ;;
  esac
  echo "   rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
