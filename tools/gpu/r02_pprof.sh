#!/bin/bash
set -o pipefail
OUT=gpurun_out/r02_pprof
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
for tag in ${TAGS:-base p2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$tag -o run --output-format csv -- python3 tools/pred_prof.py $tag ${VAR:-cog} > $OUT/$tag.log 2>&1
  rc=$?; echo "$tag rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  f=$(find $OUT/$tag -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -12
done
