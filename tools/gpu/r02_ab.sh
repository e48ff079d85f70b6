#!/bin/bash
# generic A/B: AB_TAGS="a b ..." AB_WHAT=attn|bwd|call|pred AB_VAR=cog|wan|both
set -o pipefail
OUT=gpurun_out/r02_ab_${AB_NAME:-x}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 500 python tools/ab.py $AB_TAGS --what ${AB_WHAT:-attn} --variant ${AB_VAR:-both} --rounds ${AB_ROUNDS:-8} > $OUT/ab.txt 2>&1
rc=$?; echo "ab rc=$rc"; grep -v amdgpu.ids $OUT/ab.txt
exit $rc
