#!/bin/bash
# Per-call A/B of library variants: AB="base new ..." bash tools/gpu/ab_call.sh (main and multi-level module)
set -o pipefail
OUT=gpurun_out/ab_call
mkdir -p $OUT
timeout -k 10 400 python tools/ab.py ${AB} --what call --variant both > $OUT/call.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/call.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/ab.py ${AB} --what mlcall --variant cog > $OUT/mlcall.log 2>&1
rc=$?; grep -v amdgpu.ids $OUT/mlcall.log; exit $rc
